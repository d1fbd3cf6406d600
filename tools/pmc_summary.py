"""Per-kernel-class summary of tools/pmc.sh output (last forward's dispatches).
usage: python tools/pmc_summary.py OUTDIR"""
import glob
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    """Readable kernel name: the identifier inside an anonymous-namespace mangled name."""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)
    if m:
        n = int(m.group(1))
        base = name[m.end():m.end() + n]
        t = re.search(r"I(DF16b|f)L", name)
        return base + ("_bf16" if t and t.group(1) == "DF16b" else "")
    return name


def load(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select dispatch_id, kernel_name, counter_name, value, grid_size, workgroup_size "
                          "from counters_collection order by dispatch_id"))
    per = defaultdict(dict)
    names = {}
    for d, k, cn, v, g, w in rows:
        per[d][cn] = per[d].get(cn, 0) + v
        names[d] = (short(k), g // max(w, 1))
    return per, names


def main():
    out = sys.argv[1]
    merged = defaultdict(lambda: defaultdict(float))
    for db in sorted(glob.glob(os.path.join(out, "g*", "*.db"))):
        per, names = load(db)
        # last forward: dispatches from the last pack_input through the last decoder
        ids = sorted(per)
        dec = [d for d in ids if names[d][0].startswith("decoder")]
        pk = [d for d in ids if names[d][0].startswith("pack_input") and d < dec[-1]]
        sel = [d for d in ids if pk[-1] <= d <= dec[-1]]
        for k, d in enumerate(sel):
            key = (k, names[d][0][:16], names[d][1])
            for cn, v in per[d].items():
                merged[key][cn] += v
    cols = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
            "SQ_ACTIVE_INST_LDS", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
            "GRBM_GUI_ACTIVE", "TCC_HIT_sum", "TCC_MISS_sum", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "TA_BUSY_avr",
            "TA_FLAT_READ_WAVEFRONTS_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum"]
    print("idx kernel            grid   " + " ".join(f"{c[3:15]:>12s}" for c in cols))
    for key in sorted(merged):
        m = merged[key]
        print(f"{key[0]:3d} {key[1]:16s} {key[2]:6d} " + " ".join(f"{m.get(c, 0):12.3g}" for c in cols))
    # derived
    print("\nderived per kernel: mfma_busy = VALU_MFMA_BUSY / (GRBM_GUI_ACTIVE * 4 SIMD * 32 CU... see notes)")
    for key in sorted(merged):
        m = merged[key]
        wave = m.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{key[0]:3d} {key[1]:16s} wait_any {m.get('SQ_WAIT_ANY', 0) / wave:5.2f} wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / wave:5.2f} "
              f"valu {m.get('SQ_ACTIVE_INST_VALU', 0) / wave:5.2f} lds {m.get('SQ_ACTIVE_INST_LDS', 0) / wave:5.2f} "
              f"bank_conf/lds_active {m.get('SQ_LDS_BANK_CONFLICT', 0) / max(m.get('SQ_LDS_IDX_ACTIVE', 1), 1):5.2f} "
              f"mfma_busy/gui {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(m.get('GRBM_GUI_ACTIVE', 1), 1):8.2f} "
              f"L2hit {m.get('TCC_HIT_sum', 0) / max(m.get('TCC_HIT_sum', 0) + m.get('TCC_MISS_sum', 0), 1):5.2f} "
              f"ta_busy/gui {m.get('TA_BUSY_avr', 0) / max(m.get('GRBM_GUI_ACTIVE', 1), 1):5.2f}")


if __name__ == "__main__":
    main()

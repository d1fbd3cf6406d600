"""Per-kernel-class summary of tools/pmc.sh output (last forward's dispatches).
usage: python tools/pmc_summary.py OUTDIR"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def load(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select dispatch_id, kernel_name, counter_name, value, grid_size, workgroup_size "
                          "from counters_collection order by dispatch_id"))
    per = defaultdict(dict)
    names = {}
    for d, k, cn, v, g, w in rows:
        per[d][cn] = per[d].get(cn, 0) + v
        names[d] = (k, g // max(w, 1))
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
            "GRBM_GUI_ACTIVE", "TCC_HIT_sum", "TCC_MISS_sum", "SQ_INSTS_MFMA", "SQ_INSTS_VALU"]
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
              f"L2hit {m.get('TCC_HIT_sum', 0) / max(m.get('TCC_HIT_sum', 0) + m.get('TCC_MISS_sum', 0), 1):5.2f}")


if __name__ == "__main__":
    main()

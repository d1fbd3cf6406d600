"""Mean per-dispatch PMC values per kernel from tools/pmc_cb.sh passes (rocprofv3 csv output).
usage: python tools/pmc_cb_summary.py OUTDIR"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)
    if m:
        return name[m.end():m.end() + int(m.group(1))] + re.sub(r"^.*?(I.*?E)EEv.*$", r"<\1>", name[m.end() + int(m.group(1)):])[:20]
    return name.split("(")[0][:60]


def main():
    out = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        kn = {}
        for r in csv.DictReader(open(f)):
            d = r["Dispatch_Id"]
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            kn[d] = short(r["Kernel_Name"])
        for d, cs in per.items():
            for c, v in cs.items():
                vals[kn[d]][c].append(v)
    for k, cs in vals.items():
        print(f"== {k}")
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(m):
            print(f"  {c:28s} {m[c]:16.1f}")
        if "SQ_WAVE_CYCLES" in m:
            w = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"  {c + '/WAVE':28s} {m[c] / w:16.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m and "SQ_BUSY_CYCLES" in m:
            # MFMA busy per SIMD: busy cycles summed over SIMDs / (SIMDs x elapsed cycles per XCD-avg)
            print(f"  {'MFMA_BUSY/(GRBM*1024/8)':28s} {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):16.3f}")
        if "FETCH_SIZE" in m:
            print(f"  {'FETCH_MB(x2 corrected)':28s} {2 * m['FETCH_SIZE'] / 1024:16.1f}")
        if "WRITE_SIZE" in m:
            print(f"  {'WRITE_MB':28s} {m['WRITE_SIZE'] / 1024:16.1f}")


if __name__ == "__main__":
    main()

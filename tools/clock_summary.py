"""Effective shader clock and MFMA-pipe occupancy per kernel from one rocprofv3 kernel trace and one
PMC pass of GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CYCLES (MI355X_MICROARCH.md, DVFS
give-back: effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time).

usage: python tools/clock_summary.py TRACE_DB PMC_DB
"""
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__file__))
from prof_summary import short  # noqa: E402

N_SIMD = 256 * 4


def main():
    tr = sqlite3.connect(sys.argv[1])
    dur = defaultdict(list)
    for n, d in tr.execute("select name, duration from kernels"):
        dur[short(n)].append(d)
    pm = sqlite3.connect(sys.argv[2])
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    names = {}
    for n, did, cn, v in pm.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection"):
        per[did][cn] += v
        names[did] = short(n)
    agg = defaultdict(lambda: defaultdict(list))
    for did, cs in per.items():
        for cn, v in cs.items():
            agg[names[did]][cn].append(v)
    print(f"{'kernel':22s} {'avg_us':>8s} {'GHz_eff':>8s} {'mfma_busy':>10s} {'sq_busy':>8s}")
    for k in sorted(agg, key=lambda k: -sum(dur.get(k, [0]))):
        if k not in dur:
            continue
        d = sum(dur[k]) / len(dur[k])  # ns
        g = agg[k].get("GRBM_GUI_ACTIVE", [0])
        grbm = sum(g) / len(g)
        ghz = grbm / 8 / d if d else 0.0
        cyc = grbm / 8
        mb = agg[k].get("SQ_VALU_MFMA_BUSY_CYCLES", [0])
        sb = agg[k].get("SQ_BUSY_CYCLES", [0])
        mfma = (sum(mb) / len(mb)) / (cyc * N_SIMD) if cyc else 0.0
        sq = (sum(sb) / len(sb)) / cyc if cyc else 0.0
        print(f"{k[:22]:22s} {d / 1e3:8.1f} {ghz:8.3f} {mfma:10.3f} {sq:8.2f}")


if __name__ == "__main__":
    main()

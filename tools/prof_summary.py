"""Summarise rocprofv3 SQLite outputs (kernel trace + FETCH_SIZE / WRITE_SIZE PMC passes).

usage: python tools/prof_summary.py TRACE_DB [FETCH_DB WRITE_DB] > profiles/rNN_summary.txt

Per kernel: calls, total/avg duration. Per model forward (one clasfv_forward = every conv_igemm
launch between two decoder launches + the decoder): GPU time, and HBM bytes from the PMC passes
with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of wide
streaming reads -> x2; WRITE_SIZE exact for 16-B stores).
"""
import sqlite3
import sys
from collections import defaultdict


KNOWN = ("conv_proj_x3", "conv_patch32_bf16", "conv_twalk_bf16", "conv_patch_bf16", "conv_winot", "conv_wino4w", "conv_wino4r", "conv_wino4", "conv_wino_q", "conv_wino_w", "conv_wino_r", "conv_wino", "conv_dma_x3", "conv_dma_w", "conv_dma", "conv_stem_x3", "conv_stem_f32", "pack_input_kernel", "decoder_kernel",
         "preprocess_video_kernel", "fuse_simple_fast_kernel", "fuse_simple_kernel", "fuse_majority_kernel",
         "build_clips_kernel", "pass_labels_kernel", "normalize_kernel", "minmax_partial_kernel", "warp_kernel",
         "warp_backward_kernel")


def short(name):
    """Kernel name without template arguments (rocprofv3 -T leaves some templates mangled)."""
    for k in KNOWN:
        if k in name:
            return k
    return name


def kernels(db):
    c = sqlite3.connect(db)
    return [(short(r[0]),) + tuple(r[1:]) for r in
            c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels order by start")]


def pmc(db, counter):
    c = sqlite3.connect(db)
    return [(short(n), v) for n, v in
            c.execute("select kernel_name, value from counters_collection where counter_name=? order by dispatch_id",
                      (counter,))]


def forwards(seq, name_of=lambda r: r[0]):
    """Split a dispatch sequence into forwards: [conv..., decoder]."""
    out, cur = [], []
    for r in seq:
        n = name_of(r)
        if "conv_" in n or n.startswith("pack_input"):
            cur.append(r)
        elif n.startswith("decoder_kernel"):
            cur.append(r)
            out.append(cur)
            cur = []
    return out


def main():
    tr = kernels(sys.argv[1])
    stats = defaultdict(lambda: [0, 0.0])
    for r in tr:
        stats[r[0]][0] += 1
        stats[r[0]][1] += r[1]
    tot = sum(v[1] for v in stats.values())
    print(f"{'kernel':40s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'pct':>6s}")
    for k, (n, d) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[:40]:40s} {n:6d} {d / 1e6:10.3f} {d / n / 1e3:10.2f} {100 * d / tot:6.2f}")
    fw = forwards(tr)
    if fw:
        last = fw[-1]
        t = sum(r[1] for r in last)
        print(f"\nforwards: {len(fw)}; last forward: {len(last)} dispatches, GPU time {t / 1e6:.3f} ms")
        ts = sorted(sum(r[1] for r in f) for f in fw)
        print(f"forward GPU time median {ts[len(ts) // 2] / 1e6:.3f} ms (min {ts[0] / 1e6:.3f})")
        print("\nper-dispatch (last forward): us, grid")
        for r in last:
            print(f"  {r[0][:18]:18s} {r[1] / 1e3:9.1f}  grid=({r[2] // max(r[5], 1)},{r[3]},{r[4]})")
    if len(sys.argv) > 3:
        for db, cn, corr in ((sys.argv[2], "FETCH_SIZE", 2.0), (sys.argv[3], "WRITE_SIZE", 1.0)):
            ev = pmc(db, cn)
            fws = forwards(ev)
            if fws:
                kb = sum(v for _, v in fws[-1])
                print(f"\n{cn} last forward: {kb / 1024:.1f} MiB raw, x{corr:g} corrected = {kb * corr / 1024:.1f} MiB")
                conv_kb = sum(v for n, v in fws[-1] if "conv_" in n)
                dec_kb = sum(v for n, v in fws[-1] if n.startswith("decoder"))
                print(f"  conv kernels {conv_kb * corr / 1024:.1f} MiB, decoder {dec_kb * corr / 1024:.1f} MiB")
        # per-kernel lines for bench.py (profiled_traffic): bytes of the last forward's launches
        per = defaultdict(lambda: [0, 0.0, 0.0])
        for col, db, corr in ((1, sys.argv[2], 2.0), (2, sys.argv[3], 1.0)):
            fws = forwards(pmc(db, "FETCH_SIZE" if col == 1 else "WRITE_SIZE"))
            if not fws:
                continue
            for n, v in fws[-1]:
                per[n][col] += v * corr / 1024
                if col == 1:
                    per[n][0] += 1
        print()
        for n, (cnt, f, w) in sorted(per.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
            print(f"pmc {n} launches={cnt} fetch_mib={f:.1f} write_mib={w:.1f}")


if __name__ == "__main__":
    main()

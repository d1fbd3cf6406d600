"""CLAS-FV throughput benchmark: 32-frame 112x112 clips/s on MI355X (BASELINE.json metric).

One step = the hot path over one batch of synthetic input, inputs already resident in HBM: per GPU
one 200-frame 112x112 video, 5 temporally shifted passes (30 clips of 32 frames, BASELINE
config[1]), clips built on the device, R(2+1)D encoder-decoder forward on every clip, softmax ->
temporal re-interpolation -> argmax per pass, SIMPLE label fusion per frame. With N GPUs the batch
is N videos; the global clip list is sharded clip-wise across ranks and each rank fuses the videos
whose clips it holds (one video per GPU: no exchange -- weak scaling).

Also reported on the same line (rank 0):
  roofline      the dominant kernel: MFMA work it issues (Winograd-domain products, padded
                channels) / its mean launch time, HIP events on the launch stream, vs the fp32 peak;
                algorithmic_equiv_tflops credits the direct-convolution MACs it replaces instead
  parity        fused-mask Dice delta and EF delta of this run vs the CPU reference path on the same
                video (tests/golden/northstar_c1.npz, produced by the oracle in the build container)
  cpu_baseline  the oracle (op-for-op torch-CPU restatement of the reference model + numpy plumbing)
                timed on this host: 3 warm-up + 5 timed batch-1 clip forwards (median), as the
                reference's -d cpu loop runs them (src/fuse_utils.py:53-61), plus one video's plumbing
  bf16          BASELINE config[4]: the same workload with the bf16 encoder
  config3       BASELINE config[3]: 64-frame 224x224 clips through the model forward
  stream        the same per-video work fed from HOST uint8 frames through the pipelined front end
                (pinned H2D overlapped with compute, device preprocessing, async D2H of the masks):
                the PCIe-inclusive rate, never the headline value

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 via torch.distributed.run.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "32f×112×112 clips/sec at 1/2/4/8 MI355X; Dice Δ vs CPU ref"
GFLOP_PER_CLIP = 167.59          # algorithmic (comb_1 commuted), SURVEY.md §8(d)
GFLOP_PER_CLIP_C3 = 1340.68      # 64x224x224 clip, BASELINE.md §2
FP32_PEAK_TFLOPS = 157.3         # MI355X fp32 (vector = MFMA), MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0        # MI355X bf16 MFMA dense
NORTHSTAR = {"echo": os.path.join(REPO, "tests", "golden", "northstar_c1.npz"),
             "random": os.path.join(REPO, "tests", "golden", "northstar_c1_random.npz"),
             "deep": os.path.join(REPO, "tests", "golden", "northstar_c1_deep.npz")}
BENCH_WEIGHTS = "echo"           # seeded weights whose masks follow the synthetic LV (weights.echo_state_dict)
DICE_BAR = {"fp32": 1e-3, "bf16": 1e-2}  # north_star: Dice within 1e-3 (fp32), 1e-2 (bf16/fp16)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU). Without WORLD_SIZE in the environment bench.py starts the N "
                         "rank processes itself (torch.distributed.run on 127.0.0.1); under a launcher WORLD_SIZE "
                         "must equal --gpus")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--videos-per-gpu", type=int, default=1)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--fuse", type=int, default=None, help="shifted passes per video (c1: 5, c2: 1)")
    ap.add_argument("--step", type=int, default=1)
    ap.add_argument("--fuse-method", default="simple")
    ap.add_argument("--batch-size", type=int, default=32, help="clips per forward call")
    ap.add_argument("--inflight", type=int, default=2,
                    help="c1: consecutive steps issued round-robin on this many HIP streams (videos in flight)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 at N=1")
    ap.add_argument("--parity-random", type=int, default=1,
                    help="also check the same workload with the random and deep weight recipes against their CPU "
                         "fixtures (one untimed step each; reported as 'parity_random_weights' / "
                         "'parity_deep_weights', and in the bf16 object)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo (rehearsal, several ranks on one GPU)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"], help="encoder compute dtype of the headline run")
    ap.add_argument("--extra-bf16", type=int, default=1,
                    help="also time the bf16 path (BASELINE config[4]) on the same workload; reported as 'bf16'")
    ap.add_argument("--extra-c3", type=int, default=1,
                    help="also time BASELINE config[3] (64x224x224 clips, model forward); reported as 'config3'")
    ap.add_argument("--c3-batch", type=int, default=8, help="64x224x224 clips per forward in the config3 run")
    ap.add_argument("--extra-stream", type=int, default=1,
                    help="also time the pipelined front end on host uint8 videos (PCIe-inclusive); reported as 'stream'")
    ap.add_argument("--workload", default="c1", choices=["c1", "c2", "c3"],
                    help="c1: config[1] fused video pipeline per GPU (headline, weak scaling); c2: config[2], a fixed "
                         "batch of --c2-videos full videos sharded clip-wise over the ranks (strong scaling); "
                         "c3: only the config[3] forward")
    ap.add_argument("--c2-videos", type=int, default=64, help="videos in the config[2] batch")
    ap.add_argument("--c2-lengths", default="equal", choices=["equal", "ragged"],
                    help="config[2] video lengths: equal (--frames each) or ragged (seeded EchoNet-like 100-300 "
                         "frames: videos straddle the ranks' clip blocks and the owner all_to_all moves margins)")
    ap.add_argument("--extra-c2-ragged", type=int, default=1,
                    help="c1 at N > 1: also time the ragged config[2] batch (f = 1) so the multi-GPU run measures "
                         "the RCCL exchange; reported as 'c2_ragged'")
    ap.add_argument("--c2-extra-fuse", type=int, default=5,
                    help="c2: also time the same batch with this many shifted passes (0: off); reported as 'fuse_extra'")
    ap.add_argument("--master-port", type=int, default=0, help="rendezvous port of the self-launched ranks (0: free)")
    args = ap.parse_args(argv)
    if args.fuse is None:
        args.fuse = 1 if args.workload == "c2" else 5
    return args


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """--gpus N without WORLD_SIZE: start the N rank processes (torch.distributed.run, rendezvous on
    127.0.0.1) and return their exit code. Runs before this process touches the GPU (no HIP call has
    been made: device_count does not initialise it on this image), so only the children own devices."""
    import subprocess
    if args.dist_backend == "nccl" and torch.cuda.device_count() < args.gpus:
        sys.exit(f"error: --gpus {args.gpus} with RCCL needs {args.gpus} visible GPUs "
                 f"({torch.cuda.device_count()} visible); use --dist-backend gloo to rehearse on fewer")
    port = args.master_port or free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, BENCH_SELF_LAUNCHED="1")
    return subprocess.run(cmd, env=env).returncode


def host_cpus():
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU quota when one is set (a
    GPU box's share of the host is 16 CPUs while os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def timed(fn, steps, warmup, engine, world, dev, kt_fn=None):
    """Run fn warmup times, then time exactly `steps` calls bracketed by barrier + synchronize (the
    throughput pass, no per-launch events). Then a kernel-timing pass: `steps` more calls of kt_fn
    (default fn) with the engine's per-kernel HIP events on. kt_fn is the one-stream form of a step
    whose throughput pass keeps several steps in flight on different streams: there an event interval
    would also hold the other streams' kernels, so per-launch durations come from the serial pass.
    Returns (max-over-ranks seconds of the throughput pass, kernel timing, last result)."""
    out = None
    for _ in range(warmup):
        out = fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    engine.set_kernel_timing(True)
    for _ in range(steps):
        (kt_fn or fn)()
    torch.cuda.synchronize()
    kt = engine.kernel_timing()
    engine.set_kernel_timing(False)
    return float(t.item()), kt, out


# The matrix pipe each kernel issues to, per engine dtype. The engine counts every kernel's issued work
# in its own pipe's products (clasfv_kernel_timing xgflop): f32 MFMA products for the Winograd / f32
# kernels, bf16 MFMA products for the split-bf16 ("x3": six products per fp32 product) and bf16 ones.
BF16_PIPE = {"conv_dma_x3", "conv_stem_x3", "conv_proj_x3", "conv_stem_bf16", "conv_patch_bf16", "conv_patch32_bf16",
             "conv_twalk_bf16",
             "conv_dma_w", "decoder_kernel"}
PIPE_PEAK = {"f32": FP32_PEAK_TFLOPS, "bf16": BF16_PEAK_TFLOPS}


def pipe_of(kernel, engine_dtype):
    if kernel in BF16_PIPE or (kernel == "conv_dma" and engine_dtype == "bf16"):
        return "bf16"
    return "f32"


def pmc_mfma_busy(dtype):
    """{kernel: (MFMA-pipe busy fraction, effective GHz)} from the newest committed
    profiles/r*_clock_mfma_busy*.txt of this dtype (tools/clock_summary.py: SQ_VALU_MFMA_BUSY_CYCLES over
    GRBM_GUI_ACTIVE / 8 x 1,024 SIMDs, one PMC pass), with the file name."""
    import glob
    import re
    suffix = "" if dtype == "fp32" else "_" + dtype
    files = [f for f in glob.glob(os.path.join(REPO, "profiles", f"r*_clock_mfma_busy{suffix}.txt"))
             if dtype != "fp32" or re.search(r"_clock_mfma_busy\.txt$", f)]
    if not files:
        return {}, None
    def tag(path):
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    f = sorted(files, key=tag)[-1]
    out = {}
    for ln in open(f).read().splitlines()[1:]:
        parts = ln.split()
        if len(parts) >= 5:
            try:
                out[parts[0]] = (float(parts[3]), float(parts[2]))
            except ValueError:
                pass
    return out, os.path.basename(f)


def kernel_table(kt, engine_dtype):
    """Per kernel class: launches, summed ms, the work it issues on ITS matrix pipe (f32 or bf16) as a
    rate and a fraction of that pipe's peak, the algorithmic (direct-convolution) rate, and the PMC
    MFMA-busy fraction from the committed clock / busy summary."""
    busy, src = pmc_mfma_busy(engine_dtype)
    out = {}
    for k, v in kt.items():
        pipe = pipe_of(k, engine_dtype)
        r = v["xgflop"] / max(v["ms"], 1e-9)
        b = busy.get(k[:22])
        out[k] = {"launches": v["launches"], "ms": round(v["ms"], 3), "pipe": pipe,
                  "issued_tflops": round(r, 2), "issued_frac_of_pipe_peak": round(r / PIPE_PEAK[pipe], 4),
                  "algorithmic_tflops": round(v["gflop"] / max(v["ms"], 1e-9), 2),
                  "committed_pmc_mfma_busy": b and b[0], "committed_pmc_clock_ghz": b and b[1]}
    return {"kernels": out, "committed_pmc_source": src,
            "note": "issued = products the kernel issues to the matrix pipe it runs on (f32: 157.3 TFLOP/s; "
                    "bf16: 2.5 PFLOP/s dense; split-bf16 x3 kernels: 6 bf16 products per fp32 product since "
                    "round 5 -- earlier rounds' bench lines counted them as fp32 products, so their "
                    "issued_tflops are not comparable) / its summed HIP-event time, THIS run; "
                    "committed_pmc_mfma_busy / committed_pmc_clock_ghz = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x "
                    "1,024 SIMDs) and GRBM_GUI_ACTIVE / 8 / wall time from the committed PMC pass "
                    "committed_pmc_source, profiled on the build that file's round tag names -- NOT measured "
                    "in this run and possibly on older kernels (null: kernel not in it)"}


def forward_stats(kt, clips, gflop_per_clip, peak, engine_dtype="fp32"):
    ms = sum(v["ms"] for v in kt.values())
    alg = gflop_per_clip * clips / (ms * 1e-3) / 1e3 if ms > 0 else 0.0
    # time the matrix pipes would need at their peaks for the work issued, over the summed kernel time
    pipe_ms = sum(v["xgflop"] / PIPE_PEAK[pipe_of(k, engine_dtype)] for k, v in kt.items())
    return {"forward_ms_per_clip": round(ms / max(clips, 1), 4), "kernel_ms_sum": round(ms, 3),
            "algorithmic_tflops": round(alg, 3), "algorithmic_frac": round(alg / peak, 4),
            "mfma_pipe_time_frac": round(pipe_ms / max(ms, 1e-9), 4),
            "gflop_per_clip": gflop_per_clip,
            "note": "sum of the per-kernel HIP-event times of every clasfv_forward launch; the decoder "
                    "projections of the stem/layer1, layer2 and layer3 taps run on a side stream concurrently "
                    "with layer4, so their intervals overlap the layer4 launches' and the sum exceeds the "
                    "forwards' device time by about that overlap (rates over this sum are conservative); "
                    "algorithmic = direct-convolution GFLOP of the graph (comb_1 commuted) over the " + str(peak) +
                    " TFLOP/s peak of the engine dtype; mfma_pipe_time_frac = sum over kernels of (work issued "
                    "/ the peak of the pipe it runs on) / the summed time"}


def kernel_roofline(ktimes, peak, dtype):
    """Roofline object of the dominant kernel (largest summed device time in the timed region):
    achieved = the MFMA GFLOP its launches issue / their summed duration (HIP events recorded by the
    engine on the launch stream); traffic = HBM bytes per launch from the committed rocprofv3 PMC
    summary (profiles/, FETCH_SIZE x2 + WRITE_SIZE) when one exists for this kernel."""
    if not ktimes:
        return None
    name, k = max(ktimes.items(), key=lambda kv: kv[1]["ms"])
    n = max(k["launches"], 1)
    tflops = k["xgflop"] / max(k["ms"], 1e-9)  # GFLOP/ms = TFLOP/s
    peak = PIPE_PEAK[pipe_of(name, dtype.split("_")[0])]  # the peak of the pipe this kernel issues to
    tr = profiled_traffic(name, dtype)
    return {"bound": "mfma", "achieved": round(tflops, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(tflops / peak, 4), "traffic": tr and tr["bytes_per_launch"],
            "kernel": name, "launches": k["launches"], "avg_launch_ms": round(k["ms"] / n, 4),
            "issued_gflop_per_launch": round(k["xgflop"] / n, 3),
            "algorithmic_gflop_per_launch": round(k["gflop"] / n, 3),
            "algorithmic_equiv_tflops": round(k["gflop"] / max(k["ms"], 1e-9), 3),
            "traffic_source": tr and tr["source"],
            "note": "achieved = MFMA work issued (Winograd F(4x4,3x3): 36 of the 144 direct products per 4x4 "
                    "tile, 16-tile MFMA groups; F(2x2,3x3): 16 of 36 per 2x2 tile; F(4,3): 6 of 12 per 4 frames; "
                    "padded channels and partial tiles counted; split-bf16 kernels: their bf16 products, rated against the bf16 pipe) / time; algorithmic_equiv_tflops = the direct-"
                    "convolution FLOPs of the same launches / time"}


def profiled_traffic(kernel, dtype):
    """HBM bytes per launch of `kernel` (averaged over one forward) from the newest committed
    rocprofv3 PMC summary: 'pmc <kernel> launches=L fetch_mib=F write_mib=W' lines written by
    tools/prof_summary.py, FETCH already x2-corrected (MI355X_MICROARCH.md HBM section)."""
    import glob
    import re
    def tag(path):  # r<round><letters>_...: round, then a..z, aa..zz (profile series order)
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_traffic_{dtype}.txt")), key=tag)
    if not files:
        return None
    m = re.search(r"^pmc %s launches=(\d+) fetch_mib=([\d.]+) write_mib=([\d.]+)" % re.escape(kernel),
                  open(files[-1]).read(), re.M)
    if not m:
        return None
    n, f, w = int(m.group(1)), float(m.group(2)), float(m.group(3))
    return {"bytes_per_launch": int((f + w) * 2**20 / max(n, 1)), "source": os.path.basename(files[-1])}


def northstar_parity(args, fused_video0, dtype, recipe=BENCH_WEIGHTS):
    """Dice delta (1 - Dice of the LV class, src/clasfv_losses.py:60-68) of this run's fused masks of
    video 0 and the |EF delta| (compute_ef_using_putative_clips, src/fuse_utils.py:105-148) against
    the CPU reference path on the same video, when the workload is the fixture's (config[1])."""
    import clasfv_amd.weights as W
    from clasfv_amd.echo import categorical_dice, compute_ef_using_putative_clips
    path = NORTHSTAR[recipe]
    if not os.path.exists(path):
        return None
    g = np.load(path, allow_pickle=False)
    if (args.frames, args.fuse, args.step) != (int(g["T"]), int(g["fuse"]), int(g["step"])) or \
            int(g["weights_seed"]) != W.DEFAULT_SEED or str(g["weights_recipe"]) != recipe or \
            f"fused_{args.fuse_method}" not in g:
        return None
    shp = tuple(g[f"fused_{args.fuse_method}_shape"])
    ref = np.unpackbits(g[f"fused_{args.fuse_method}"])[: int(np.prod(shp))].reshape(shp).astype(np.int64)
    got = fused_video0.to(torch.int64).cpu().numpy()
    efs, pairs = compute_ef_using_putative_clips(got, "bench", return_edes=True)
    ref_ef = g[f"ef_{args.fuse_method}"]
    same_pairs = np.array(pairs, np.int64).reshape(-1, 2).tolist() == g[f"pairs_{args.fuse_method}"].tolist()
    if same_pairs and len(efs):
        d = np.abs(np.array(efs) - ref_ef)
        ef_delta = float(np.nanmax(d)) if np.isfinite(d).any() else 0.0
        mean_delta = float(abs(np.nanmean(efs) - np.nanmean(ref_ef)))
    else:
        ef_delta = mean_delta = None
    dice = float(1.0 - categorical_dice(got, ref, 1))
    # when an ED / ES frame moved (a mask at the decision margin on one frame), the systoles still pair
    # up by index: the largest frame shift and the EF deltas of the index-matched systoles
    gp, rp = np.array(pairs, np.int64).reshape(-1, 2), np.asarray(g[f"pairs_{args.fuse_method}"]).reshape(-1, 2)
    matched = None
    if not same_pairs and len(gp) == len(rp) and len(efs):
        d = np.abs(np.array(efs) - ref_ef)
        matched = {"max_frame_shift": int(np.abs(gp - rp).max()),
                   "ef_delta_max": float(np.nanmax(d)) if np.isfinite(d).any() else None}
    return {"dice_delta_fused_masks": round(dice, 9), "ef_delta_max_per_systole": ef_delta, "ef_delta_mean": mean_delta,
            "ed_es_pairs_equal": same_pairs, "index_matched_systoles": matched, "bar": DICE_BAR[dtype], "within_bar": dice <= DICE_BAR[dtype],
            "efs_gpu": [round(float(e), 4) for e in efs], "efs_cpu": [round(float(e), 4) for e in ref_ef],
            "weights": recipe,
            "reference": "tests/golden/%s (oracle CPU path, same video and weights, fuse=%s)"
                         % (os.path.basename(path), args.fuse_method)}


def random_recipe_parity(args, model, step, dtype, recipe="random"):
    """One untimed step of the same workload with another weight recipe against its CPU fixture; the
    bench weights are restored afterwards. "random": every layer at full gain (the echo recipe's LV
    decision runs through the stem, layer1 and the decoder only), degenerate EFs; "deep": the echo
    segmentation routed through layer2-4 at full gain, physiological EFs."""
    import clasfv_amd.weights as W
    if not os.path.exists(NORTHSTAR[recipe]):
        return None
    torch.cuda.synchronize()  # no step in flight reads the weights being replaced
    model.load_state_dict(W.recipe_state_dict(recipe, W.DEFAULT_SEED))
    try:
        out = step()  # the one-stream step: its masks are read on this stream
        torch.cuda.synchronize()
        return northstar_parity(args, out[0], dtype, recipe=recipe) if 0 in out else None
    finally:
        model.load_state_dict(W.recipe_state_dict(BENCH_WEIGHTS, W.DEFAULT_SEED))


def cpu_baseline(args, S):
    """Reference-style CPU path (oracle = op-for-op restatement of the reference, torch CPU): batch-1
    clip forwards as src/fuse_utils.py:53-61 runs them (3 warm-up + 5 timed, median), plus the CPU
    plumbing + fusion of one whole video with the clip forwards replaced by cached logits."""
    from oracle import fuse_ref, r2plus1d_ref
    import clasfv_amd.weights as W
    threads = host_cpus()  # every CPU this process may use (affinity / cgroup quota)
    torch.set_num_threads(threads)
    model = r2plus1d_ref.OracleModel(W.synthetic_state_dict())
    v = fuse_ref.zeroone_normalizer(S.echo_video(args.frames, seed=0))
    clips = fuse_ref.divide_to_consecutive_clips(v, interpolate_last=True)
    times, seg = [], None
    for i in range(8):
        t0 = time.perf_counter()
        seg, _ = model(clips[i % len(clips)][None])
        if i >= 3:
            times.append(time.perf_counter() - t0)
    t_clip = float(np.median(times))
    cached = (seg.numpy(), None)
    t1 = time.perf_counter()
    fuse_ref.segment_a_video_with_fusion(v, lambda c: cached, step=args.step, num_clips=args.fuse,
                                         fuse_method=args.fuse_method)
    t_plumb = time.perf_counter() - t1
    k = fuse_ref.clamp_num_clips(args.frames, args.fuse, args.step)
    n_total = sum(fuse_ref.n_clip_frames(args.frames - j * args.step) // 32 for j in range(k))
    per_video = n_total * t_clip + t_plumb
    return {"value": round(n_total / per_video, 4), "unit": "clips/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(),
            "sample": f"median of 5 timed batch-1 32x112x112 clip forwards (after 3 warm-up) of the torch-CPU "
                      f"oracle on {threads} threads ({t_clip:.2f} s/clip) + CPU plumbing and "
                      f"{args.fuse_method} fusion of one {args.frames}-frame video ({t_plumb:.2f} s), per the "
                      f"{n_total} clips of one step"}


def gather_ranks(obj, world):
    """Every rank's `obj` on every rank (list in rank order)."""
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            sys.exit(launch_ranks(args))
    elif int(env_world) != args.gpus:
        sys.exit(f"error: WORLD_SIZE={env_world} (launcher) but --gpus {args.gpus}: they must agree")
    world = int(env_world or 1)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:  # rehearsal of the exchange with several ranks on one GPU
            dist.init_process_group(args.dist_backend)

    from clasfv_amd.model import R2plus1D_18_MotionNet
    model = R2plus1D_18_MotionNet(pretrained=False, dtype=args.dtype, device=dev, weights=BENCH_WEIGHTS)
    run = {"c1": run_c1, "c2": run_c2, "c3": run_c3_only}[args.workload]
    line = run(args, model, world, rank, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def c3_run(args, model, world, dev, steps, warmup):
    import clasfv_amd.synthetic as S
    from clasfv_amd.preprocess import zeroone_normalize_
    eng = model.engine
    x = torch.cat([zeroone_normalize_(torch.from_numpy(S.echo_video(64, H=224, W=224, seed=21 + i)).to(dev))[None]
                   for i in range(args.c3_batch)])
    # consecutive forwards round-robin on `inflight` streams (one engine workspace per stream)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(max(1, args.inflight) - 1)]
    issued = [0]

    def fwd():
        s = streams[issued[0] % len(streams)]
        issued[0] += 1
        with torch.cuda.stream(s):
            return model(x)

    torch.cuda.synchronize()
    dt, kt, _ = timed(fwd, steps, warmup, eng, world, dev, kt_fn=lambda: model(x))
    n = args.c3_batch * steps * world
    peak = BF16_PEAK_TFLOPS if eng.dtype == "bf16" else FP32_PEAK_TFLOPS
    return {"value": round(n / dt, 3), "unit": "64x224x224 clips/s", "ms_per_step": round(dt / steps * 1e3, 3),
            "clips_per_step": args.c3_batch * world,
            "forward": forward_stats(kt, args.c3_batch * steps, GFLOP_PER_CLIP_C3, peak, eng.dtype),
            "roofline": kernel_roofline(kt, peak, eng.dtype + "_c3"),  # no c3 PMC profile: traffic null
            "note": "BASELINE config[3]: (N,3,64,224,224) model forward (seg + motion), the reference's "
                    "forward signature; the CLI path is fixed at 112x112 (src/fuse_utils.py:22)"}


def run_c3_only(args, model, world, rank, dev):
    res = c3_run(args, model, world, dev, args.steps, args.warmup)
    return {"metric": "64f×224×224 clips/sec (BASELINE config[3])", "value": res["value"], "unit": res["unit"],
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": model.engine.dtype,
            "data": "synthetic", "config": {"workload": "BASELINE config[3]: 64-frame 224x224 clips, model forward",
                                            "batch": args.c3_batch},
            "roofline": res["roofline"], "forward": res["forward"]}


def make_videos(args, lengths, needed, dev):
    """Synthetic EchoNet-style videos (seed = video index), normalised on the device; None for the
    videos this rank does not hold (not timed)."""
    import clasfv_amd.synthetic as S
    from clasfv_amd.preprocess import zeroone_normalize_
    out = [None] * len(lengths)
    for v in needed:
        x = torch.from_numpy(S.echo_video(lengths[v], seed=v)).to(dev)
        out[v] = zeroone_normalize_(x.contiguous())
    return out


def c2_lengths(args):
    import clasfv_amd.synthetic as S
    if args.c2_lengths == "ragged":
        return S.echonet_like_lengths(args.c2_videos)
    return [args.frames] * args.c2_videos


def c2_measure(args, model, world, rank, dev, lengths, fuse, steps, warmup):
    """One config[2]-style run: the batch of videos `lengths` sharded clip-wise over the ranks, fused on
    each video's owner; the owner all_to_all (dist.exchange_to_owners) is timed with events on the
    compute stream around the margin computation and the collective (max over ranks)."""
    from clasfv_amd import dist as D
    eng = model.engine
    peak = BF16_PEAK_TFLOPS if args.dtype == "bf16" else FP32_PEAK_TFLOPS
    needed = D.videos_needed(lengths, fuse, args.step, rank, world)
    videos = make_videos(args, lengths, needed, dev)
    plans, n_total = D.global_clip_plan(lengths, fuse, args.step)
    lo, hi = D.shard_bounds(n_total, rank, world)
    evs = []
    # steps in flight as in run_c1 (only without a data exchange: every rank's collectives keep one
    # order); the exchange events are recorded in the serial kernel-timing pass
    inflight = max(1, args.inflight) if D.rows_exchanged(D.owner_of_clips(plans, world), world) == 0 else 1
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(inflight - 1)]
    issued = [0]

    def serial_step(ev=None):
        return D.segment_videos_sharded(videos, model, num_clips=fuse, step=args.step,
                                        fuse_method=args.fuse_method, rank=rank, world=world,
                                        batch_size=args.batch_size, lengths=lengths, exchange_events=ev)

    def step():
        s = streams[issued[0] % len(streams)]
        issued[0] += 1
        with torch.cuda.stream(s):
            return serial_step()

    torch.cuda.synchronize()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dt, kt, out = timed(step, steps, 0, eng, world, dev, kt_fn=lambda: serial_step(evs))
    ex_ms = sum(a.elapsed_time(b) for a, b in evs) / steps if evs else 0.0
    t = torch.tensor([ex_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    fwd = forward_stats(kt, (hi - lo) * steps, GFLOP_PER_CLIP, peak, args.dtype)
    rows, nbytes = D.exchange_stats(lengths, fuse, args.step, world)
    xfer_ms = exchange_transfer_ms(lengths, fuse, args.step, rank, world, dev) if rows else 0.0
    mine = {"rank": rank, "clips": hi - lo, "videos_held": len(needed), "videos_fused": len(out),
            "forward_ms_per_step": round(sum(v["ms"] for v in kt.values()) / steps, 3)}
    per_rank = gather_ranks(mine, world)
    del videos
    torch.cuda.empty_cache()
    return {"value": round(n_total * steps / dt, 3), "unit": "clips/s", "ms_per_step": round(dt / steps * 1e3, 3),
            "clips_per_step": n_total, "fuse": fuse, "steps_in_flight": inflight, "forward": fwd, "per_rank": per_rank,
            "rows_exchanged_per_step": rows, "bytes_exchanged_per_step": nbytes,
            "exchange_ms_per_step": round(float(t.item()), 4),
            "exchange_transfer_ms": round(xfer_ms, 4),
            "exchange_note": "margin planes (fp32, 32 x 112 x 112 per crossing clip) through one all_to_all_single "
                             "(RCCL over xGMI with nccl; host-staged with gloo). exchange_ms_per_step = events on the "
                             "compute stream around logit_margin + the collective inside the timed steps, max over "
                             "ranks: it includes waiting for the slowest rank's forward (skew); "
                             "exchange_transfer_ms = the same all_to_all alone, every rank entering together "
                             "(barrier + synchronize before it), median of 5, max over ranks: the transfer",
            "roofline": kernel_roofline(kt, peak, args.dtype), "kt": kt, "out": out}


def exchange_transfer_ms(lengths, fuse, step, rank, world, dev, reps=5):
    """The owner all_to_all of one sharded pass alone (same split sizes as the timed steps, zero margin
    planes), with the ranks synchronised before each repetition so no forward skew is included:
    median of `reps`, max over ranks."""
    from clasfv_amd import dist as D
    plans, n_total = D.global_clip_plan(lengths, fuse, step)
    owners = D.owner_of_clips(plans, world)
    lo, hi = D.shard_bounds(n_total, rank, world)
    local = torch.zeros((hi - lo, 32, 112, 112), dtype=torch.float32, device=dev)
    times = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        dist.barrier()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        D.exchange_to_owners(local, owners, rank, world)
        b.record()
        torch.cuda.synchronize()
        times.append(a.elapsed_time(b))
    t = torch.tensor([float(np.median(times[1:]))], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    del local
    return float(t.item())


def run_c2(args, model, world, rank, dev):
    """BASELINE config[2]: a fixed batch of full videos (64 x 200 frames, or seeded ragged 100-300-frame
    lengths with --c2-lengths ragged) sharded clip-wise over the ranks (strong scaling). f = 1: 384
    clips for the equal batch; the fuse_extra run repeats it with f = 5."""
    lengths = c2_lengths(args)
    main_run = c2_measure(args, model, world, rank, dev, lengths, args.fuse, args.steps, args.warmup)
    extra = None
    if args.c2_extra_fuse and args.c2_extra_fuse != args.fuse:
        extra = c2_measure(args, model, world, rank, dev, lengths, args.c2_extra_fuse, max(2, args.steps // 3), 1)
        extra = {k: v for k, v in extra.items() if k not in ("kt", "out")}
    lv = [float(o.float().mean().item()) for o in main_run["out"].values()]
    lv_all = gather_ranks(lv, world)
    desc = (f"{args.c2_videos} videos x {args.frames} frames" if args.c2_lengths == "equal" else
            f"{args.c2_videos} videos of seeded EchoNet-like lengths 100-300 frames ({sum(lengths)} frames)")
    return {
        "metric": METRIC, "value": main_run["value"], "unit": "clips/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": main_run["ms_per_step"], "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic EchoNet-style videos (seeded), seeded synthetic weights (" + BENCH_WEIGHTS + " recipe)",
        "config": {"workload": f"BASELINE config[2]: batch of {desc}, "
                               f"{args.fuse} shifted pass(es), clips sharded over {world} rank(s) + per-frame "
                               f"{args.fuse_method} fusion on each video's owner",
                   "videos": args.c2_videos, "frames": args.frames if args.c2_lengths == "equal" else lengths,
                   "fuse": args.fuse, "step": args.step,
                   "clips_per_step": main_run["clips_per_step"], "batch_size": args.batch_size,
                   "parallelism": f"clip-shard x{world} ({args.dist_backend}); owner all_to_all of logit margins "
                                  f"only for straddling videos"},
        "roofline": main_run["roofline"], "forward": main_run["forward"], "per_rank": main_run["per_rank"],
        "rows_exchanged_per_step": main_run["rows_exchanged_per_step"],
        "bytes_exchanged_per_step": main_run["bytes_exchanged_per_step"],
        "exchange_ms_per_step": main_run["exchange_ms_per_step"],
        "exchange_transfer_ms": main_run["exchange_transfer_ms"], "exchange_note": main_run["exchange_note"],
        "fuse_extra": extra, "lv_fraction": round(float(np.mean(sum(lv_all, []))), 4),
    }


def run_c1(args, model, world, rank, dev):
    """BASELINE config[1] per GPU (the headline): each rank fuses its own 200-frame video(s) with 5
    shifted passes (weak scaling)."""
    from clasfv_amd import dist as D
    eng = model.engine
    n_videos = args.videos_per_gpu * world
    lengths = [args.frames] * n_videos
    needed = D.videos_needed(lengths, args.fuse, args.step, rank, world)
    videos = make_videos(args, lengths, needed, dev)
    plans, n_total = D.global_clip_plan(lengths, args.fuse, args.step)
    lo, hi = D.shard_bounds(n_total, rank, world)

    # steps in flight: consecutive steps round-robin on `inflight` streams, so step k + 1's stem / layer1
    # grids overlap step k's small-grid tail (layer3 / layer4, decoder, fusion); the engine keeps one
    # workspace per stream. Only where no step moves data between ranks (the c1 layout: one video per
    # rank), so every rank's collectives stay in one order.
    inflight = max(1, args.inflight) if world == 1 or D.rows_exchanged(D.owner_of_clips(plans, world), world) == 0 else 1
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(inflight - 1)]
    issued = [0]
    torch.cuda.synchronize()  # the videos exist before any stream reads them

    def serial_step():
        return D.segment_videos_sharded(videos, model, num_clips=args.fuse, step=args.step,
                                        fuse_method=args.fuse_method, rank=rank, world=world,
                                        batch_size=args.batch_size, lengths=lengths)

    def step():
        s = streams[issued[0] % len(streams)]
        issued[0] += 1
        with torch.cuda.stream(s):
            return serial_step()

    dt, ktimes, out = timed(step, args.steps, args.warmup, eng, world, dev, kt_fn=serial_step)
    value = n_total * args.steps / dt
    peak = BF16_PEAK_TFLOPS if args.dtype == "bf16" else FP32_PEAK_TFLOPS
    fwd = forward_stats(ktimes, (hi - lo) * args.steps, GFLOP_PER_CLIP, peak, args.dtype)
    lv_frac = float(np.mean([o.float().mean().item() for o in out.values()])) if out else 0.0
    parity = northstar_parity(args, out[0], args.dtype) if 0 in out else None
    parity_random = random_recipe_parity(args, model, serial_step, args.dtype) if world == 1 and args.parity_random else None
    parity_deep = (random_recipe_parity(args, model, serial_step, args.dtype, "deep")
                   if world == 1 and args.parity_random else None)

    bf16 = None
    if args.extra_bf16 and args.dtype == "fp32":
        ref_masks = {k: v.clone() for k, v in out.items()}
        model.set_compute_dtype("bf16")
        dt16, k16, out16 = timed(step, args.steps, args.warmup, eng, world, dev, kt_fn=serial_step)
        from clasfv_amd.echo import categorical_dice
        d16 = [1.0 - categorical_dice(out16[k].cpu().numpy(), ref_masks[k].cpu().numpy(), 1) for k in out16]
        bf16 = {"value": round(n_total * args.steps / dt16, 3), "unit": "clips/s",
                "ms_per_step": round(dt16 / args.steps * 1e3, 3),
                "forward": forward_stats(k16, (hi - lo) * args.steps, GFLOP_PER_CLIP, BF16_PEAK_TFLOPS, "bf16"),
                "dice_delta_vs_fp32_fused_masks": round(float(max(d16)) if d16 else 0.0, 6),
                "parity_vs_cpu": northstar_parity(args, out16[0], "bf16") if 0 in out16 else None,
                "parity_vs_cpu_random_weights": (random_recipe_parity(args, model, serial_step, "bf16")
                                                 if world == 1 and args.parity_random else None),
                "parity_vs_cpu_deep_weights": (random_recipe_parity(args, model, serial_step, "bf16", "deep")
                                               if world == 1 and args.parity_random else None),
                "roofline": kernel_roofline(k16, BF16_PEAK_TFLOPS, "bf16"),
                "kernels": kernel_table(k16, "bf16"),
                "note": "BASELINE config[4]: bf16 activations/weights, fp32 accumulate, fp32 decoder head; "
                        "Dice tolerance 1e-2"}
        model.set_compute_dtype("fp32")

    c3 = c3_run(args, model, world, dev, max(2, args.steps // 2), 1) if args.extra_c3 else None

    # N > 1: the ragged config[2] batch, whose straddling videos move logit margins between ranks (the
    # c1 layout, one equal video per rank, exchanges nothing)
    c2r = None
    if args.extra_c2_ragged and world > 1:
        import clasfv_amd.synthetic as S
        c2r = c2_measure(args, model, world, rank, dev, S.echonet_like_lengths(args.c2_videos), 1,
                         max(2, args.steps // 2), 1)
        c2r = {k: v for k, v in c2r.items() if k not in ("kt", "out", "roofline")}
        c2r["workload"] = (f"BASELINE config[2] with ragged lengths: {args.c2_videos} seeded EchoNet-like videos of "
                           f"100-300 frames, f = 1, clips sharded over {world} ranks (strong scaling)")

    stream = None
    if args.extra_stream and world == 1:
        import clasfv_amd.synthetic as S
        from clasfv_amd.stream import VideoStream
        hv = [S.echo_video_uint8(args.frames, seed=v) for v in range(8)]
        vs = VideoStream(model, num_clips=args.fuse, step=args.step, fuse_method=args.fuse_method,
                         batch_size=args.batch_size)
        vs.run(hv[:2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vs.run(hv)
        dts = time.perf_counter() - t0
        stream = {"value": round(n_total * len(hv) / dts, 3), "unit": "clips/s", "videos": len(hv),
                  "ms_per_video": round(dts / len(hv) * 1e3, 3),
                  "note": "host (T,112,112,3) uint8 frames -> pinned H2D on a copy stream overlapped with the "
                          "previous video's compute -> device resize/normalise -> clips -> forward -> fusion -> "
                          "async D2H of the uint8 masks; PCIe-inclusive, one host sync per batch of videos"}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        import clasfv_amd.synthetic as S
        cpu = cpu_baseline(args, S)

    return {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "clips/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "dtype_note": ("fp32 activations, weights and accumulation; the Winograd convs (layer1-3) on f32 "
                       "MFMAs; the stem, strided / 1x1x1 convs, layer4 convs, decoder projections, comb_2 "
                       "and heads on split-bf16 MFMAs (3 bf16 pieces per operand, 6 products, fp32 "
                       "accumulation: fp32-accurate; variants no_stem_x3 / no_dma_x3 / no_decoder_x3 run "
                       "them on f32 MFMAs)") if args.dtype == "fp32" else None,
        "data": "synthetic EchoNet-style video (seeded), seeded synthetic weights (" + BENCH_WEIGHTS + " recipe)",
        "config": {"workload": "BASELINE config[1] per GPU: 200-frame 112x112 video, 5 shifted passes "
                               "(30 x 32-frame clips) + per-frame SIMPLE label fusion",
                   "videos_per_gpu": args.videos_per_gpu, "frames": args.frames, "fuse": args.fuse,
                   "step": args.step, "clips_per_step": n_total, "batch_size": args.batch_size,
                   "steps_in_flight": inflight,
                   "timing": "value / ms_per_step: the throughput pass, consecutive steps round-robin on "
                             "steps_in_flight HIP streams (one engine workspace per stream), no per-launch "
                             "events; roofline / forward / kernels: a second pass of the same steps on one "
                             "stream with the engine's per-launch HIP events",
                   "parallelism": f"clip-shard x{world}; videos fused on the rank holding their clips "
                                  f"(owner all_to_all of logit margins only for straddling videos)"},
        "roofline": kernel_roofline(ktimes, peak, args.dtype),
        "forward": fwd,
        "kernels": kernel_table(ktimes, args.dtype),
        "cpu_baseline": cpu,
        "dice_delta_vs_cpu": parity and parity["dice_delta_fused_masks"],
        "ef_delta_vs_cpu": parity and parity["ef_delta_max_per_systole"],
        "parity": parity,
        "parity_random_weights": parity_random,
        "parity_deep_weights": parity_deep,
        "bf16": bf16,
        "config3": c3,
        "c2_ragged": c2r,
        "stream": stream,
        "lv_fraction": round(lv_frac, 4),
    }


if __name__ == "__main__":
    main()

"""CLAS-FV throughput benchmark: 32-frame 112x112 clips/s on MI355X (BASELINE.json metric).

One step = the hot path over one batch of synthetic EchoNet-shaped input, inputs already resident
in HBM: per GPU one 200-frame 112x112 video, 5 temporally shifted passes (30 clips of 32 frames,
BASELINE config[1]), clips built on the device, R(2+1)D encoder-decoder forward on every clip,
softmax -> temporal re-interpolation -> argmax per pass, SIMPLE label fusion per frame. With N GPUs
the batch is N videos; the global clip list is sharded clip-wise across ranks, each rank fuses the
videos it owns and per-clip logits computed away from their owner move by one RCCL all_to_all (none
at one video per GPU: weak scaling).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 via torch.distributed.run.
Prints one JSON line on rank 0.
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
GFLOP_PER_CLIP_AS_WRITTEN = 218.29
FP32_PEAK_TFLOPS = 157.3         # MI355X fp32 (vector = MFMA), MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0        # MI355X bf16 MFMA dense


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--videos-per-gpu", type=int, default=1)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--fuse", type=int, default=5)
    ap.add_argument("--step", type=int, default=1)
    ap.add_argument("--fuse-method", default="simple")
    ap.add_argument("--batch-size", type=int, default=32, help="clips per forward call")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 at N=1")
    ap.add_argument("--cpu-sample-clips", type=int, default=4)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo (rehearsal on one GPU)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"], help="encoder compute dtype of the headline run")
    ap.add_argument("--extra-bf16", type=int, default=1,
                    help="also time the bf16 path (BASELINE config[4]) on the same workload; reported as 'bf16'")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:  # rehearsal of the exchange with several ranks on one GPU
            dist.init_process_group(args.dist_backend)

    import clasfv_amd.synthetic as S
    from clasfv_amd import dist as D
    from clasfv_amd import fuse_utils as FU
    from clasfv_amd.model import R2plus1D_18_MotionNet
    from clasfv_amd.preprocess import zeroone_normalize_

    model = R2plus1D_18_MotionNet(pretrained=False, dtype=args.dtype)
    n_videos = args.videos_per_gpu * world
    videos = []
    for v in range(n_videos):  # synthetic EchoNet-style videos, normalised on the device (not timed)
        x = torch.from_numpy(S.echo_video(args.frames, seed=v)).to(dev)
        videos.append(zeroone_normalize_(x.contiguous()))

    fwd_events = []

    class TimedModel:
        """Records HIP events around each forward launch sequence on the current stream."""
        engine = model.engine

        def __call__(self, x):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            out = model(x)
            b.record()
            fwd_events.append((a, b, x.shape[0]))
            return out

    timed = TimedModel()

    def step():
        return D.segment_videos_sharded(videos, timed, num_clips=args.fuse, step=args.step,
                                        fuse_method=args.fuse_method, rank=rank, world=world,
                                        batch_size=args.batch_size)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    fwd_events.clear()
    model.engine.set_kernel_timing(True)  # per-kernel HIP events on the forward's stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ktimes = model.engine.kernel_timing()
    model.engine.set_kernel_timing(False)
    fwd_ms = sum(a.elapsed_time(b) for a, b, _ in fwd_events)
    fwd_clips = sum(n for _, _, n in fwd_events)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    plans, n_total = D.global_clip_plan([v.shape[1] for v in videos], args.fuse, args.step)
    clips_per_step = n_total
    value = clips_per_step * args.steps / dt
    achieved_tflops = GFLOP_PER_CLIP * fwd_clips / (fwd_ms * 1e-3) / 1e3 if fwd_ms > 0 else 0.0

    # Dice parity of this run's fused masks vs the CPU oracle is checked by the tests; here a cheap
    # on-line sanity figure: LV fraction of the last step's masks.
    lv_frac = float(np.mean([o.float().mean().item() for o in out.values()])) if out else 0.0

    cpu, dice = None, None
    if rank == 0 and world == 1 and args.cpu_baseline:
        cpu, dice = cpu_baseline(args, S, model)

    bf16 = None
    if args.extra_bf16 and args.dtype == "fp32":
        # same workload with the bf16 encoder; Dice of its fused masks against this run's fp32 masks
        ref_masks = {k: v.clone() for k, v in out.items()}
        model.set_compute_dtype("bf16")
        for _ in range(args.warmup):
            step()
        fwd_events.clear()
        model.engine.set_kernel_timing(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out16 = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt16 = time.perf_counter() - t0
        k16 = model.engine.kernel_timing()
        model.engine.set_kernel_timing(False)
        t = torch.tensor([dt16], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt16 = float(t.item())
        f16_ms = sum(a.elapsed_time(b) for a, b, _ in fwd_events)
        f16_clips = sum(n for _, _, n in fwd_events)
        from clasfv_amd.echo import categorical_dice
        d16 = [1.0 - categorical_dice(out16[k].cpu().numpy(), ref_masks[k].cpu().numpy(), 1) for k in out16]
        bf16 = {"value": round(clips_per_step * args.steps / dt16, 3), "unit": "clips/s",
                "ms_per_step": round(dt16 / args.steps * 1e3, 3),
                "forward_ms_per_clip": round(f16_ms / max(f16_clips, 1), 4),
                "dice_delta_vs_fp32_fused_masks": round(float(max(d16)) if d16 else 0.0, 6),
                "roofline": kernel_roofline(k16, BF16_PEAK_TFLOPS, "bf16"),
                "note": "BASELINE config[4]: bf16 activations/weights, fp32 accumulate, fp32 decoder head; "
                        "Dice tolerance 1e-2"}

    if rank == 0:
        line = {
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
            "dtype": "fp32",
            "data": "synthetic EchoNet-style video (seeded), seeded synthetic weights",
            "config": {"workload": "BASELINE config[1] per GPU: 200-frame 112x112 video, 5 shifted passes "
                                   "(30 x 32-frame clips) + per-frame SIMPLE label fusion",
                       "videos_per_gpu": args.videos_per_gpu, "frames": args.frames, "fuse": args.fuse,
                       "step": args.step, "clips_per_step": clips_per_step, "batch_size": args.batch_size,
                       "parallelism": f"clip-shard x{world}, owner all_to_all of per-clip logits (skipped when every video is rank-local)"},
            "roofline": kernel_roofline(ktimes, FP32_PEAK_TFLOPS, "fp32"),
            "forward": {"achieved_tflops": round(achieved_tflops, 3), "peak": FP32_PEAK_TFLOPS,
                        "frac": round(achieved_tflops / FP32_PEAK_TFLOPS, 4), "gflop_per_clip": GFLOP_PER_CLIP,
                        "forward_ms_per_clip": round(fwd_ms / max(fwd_clips, 1), 4),
                        "note": "whole clasfv_forward (all conv + decoder launches), HIP events around each call"},
            "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                            "tflops": round(v["gflop"] / max(v["ms"], 1e-9), 2)} for k, v in ktimes.items()},
            "cpu_baseline": cpu,
            "dice_delta_vs_cpu": dice,
            "bf16": bf16,
            "lv_fraction": round(lv_frac, 4),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def kernel_roofline(ktimes, peak, dtype):
    """Roofline object of the dominant kernel (largest summed device time in the timed region):
    achieved = its algorithmic GFLOP per launch / its mean launch duration (HIP events recorded by
    the engine on the launch stream), traffic = HBM bytes per launch from the committed rocprofv3
    PMC summary (profiles/, FETCH_SIZE x2 + WRITE_SIZE) when one exists for this kernel."""
    if not ktimes:
        return None
    name, k = max(ktimes.items(), key=lambda kv: kv[1]["ms"])
    n = max(k["launches"], 1)
    tflops = k["gflop"] / max(k["ms"], 1e-9)  # GFLOP/ms = TFLOP/s
    tr = profiled_traffic(name, dtype)
    return {"bound": "mfma", "achieved": round(tflops, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(tflops / peak, 4), "traffic": tr and tr["bytes_per_launch"],
            "kernel": name, "launches": k["launches"], "avg_launch_ms": round(k["ms"] / n, 4),
            "gflop_per_launch": round(k["gflop"] / n, 3),
            "traffic_source": tr and tr["source"],
            "note": "algorithmic GFLOP = direct-convolution MACs x 2 over unpadded channels (Winograd kernels "
                    "execute fewer MFMA flops than they are credited)"}


def profiled_traffic(kernel, dtype):
    """HBM bytes per launch of `kernel` (averaged over one forward) from the newest committed
    rocprofv3 PMC summary: 'pmc <kernel> launches=L fetch_mib=F write_mib=W' lines written by
    tools/prof_summary.py, FETCH already x2-corrected (MI355X_MICROARCH.md HBM section)."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_traffic_{dtype}.txt")))
    if not files:
        return None
    m = re.search(r"^pmc %s launches=(\d+) fetch_mib=([\d.]+) write_mib=([\d.]+)" % re.escape(kernel),
                  open(files[-1]).read(), re.M)
    if not m:
        return None
    n, f, w = int(m.group(1)), float(m.group(2)), float(m.group(3))
    return {"bytes_per_launch": int((f + w) * 2**20 / max(n, 1)), "source": os.path.basename(files[-1])}


def cpu_baseline(args, S, gpu_model):
    """Reference-style CPU path (oracle = op-for-op restatement of the reference, torch CPU):
    per-clip batch-1 forwards as src/fuse_utils.py:53-61 does, on a bounded sample of clips, plus the
    CPU plumbing of one whole video with the clip forwards replaced by cached logits.
    Also returns the Dice delta (1 - Dice of the LV masks) of the GPU forward vs these CPU clips."""
    from oracle import fuse_ref, r2plus1d_ref
    import clasfv_amd.weights as W
    threads = min(os.cpu_count() or 1, 16)
    torch.set_num_threads(threads)
    sd = W.synthetic_state_dict()
    model = r2plus1d_ref.OracleModel(sd)
    v = fuse_ref.zeroone_normalizer(S.echo_video(args.frames, seed=0))
    clips = fuse_ref.divide_to_consecutive_clips(v, interpolate_last=True)
    model(clips[:1])  # warm-up
    t0 = time.perf_counter()
    n = 0
    cached = None
    cpu_masks = []
    for i in range(args.cpu_sample_clips):
        seg, _ = model(clips[i % len(clips)][None])
        cached = (seg.numpy(), None)
        cpu_masks.append(seg[0, 1].numpy() > seg[0, 0].numpy())
        n += 1
    t_clip = (time.perf_counter() - t0) / n
    from clasfv_amd.echo import categorical_dice
    gseg, _ = gpu_model(torch.from_numpy(np.stack([clips[i % len(clips)] for i in range(n)])))
    gseg = gseg.cpu().numpy()
    gpu_masks = gseg[:, 1] > gseg[:, 0]
    dice = float(1.0 - categorical_dice(gpu_masks, np.stack(cpu_masks), 1))
    t1 = time.perf_counter()
    k = fuse_ref.clamp_num_clips(args.frames, args.fuse, args.step)
    out = fuse_ref.segment_a_video_with_fusion(v, lambda c: cached, step=args.step, num_clips=args.fuse,
                                               fuse_method=args.fuse_method)
    t_plumb = time.perf_counter() - t1
    _, n_total = 0, sum(fuse_ref.n_clip_frames(args.frames - j * args.step) // 32 for j in range(k))
    per_video = n_total * t_clip + t_plumb
    return {"value": round(n_total / per_video, 4), "unit": "clips/s", "cores": threads, "kind": "port",
            "sample": f"{n} batch-1 clip forwards of the torch-CPU oracle ({t_clip:.2f} s/clip) + CPU plumbing "
                      f"and SIMPLE fusion of one {args.frames}-frame video ({t_plumb:.2f} s), extrapolated to "
                      f"the {n_total} clips of one step",
            "out_shape": list(out.shape)}, round(dice, 7)


if __name__ == "__main__":
    main()

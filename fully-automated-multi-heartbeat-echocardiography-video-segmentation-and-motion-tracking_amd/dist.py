"""Clip-wise sharding of a batch of videos across ranks (one process per GPU).

Every 32-frame clip of every temporally shifted pass of every video is independent
(src/fuse_utils.py:45-61), so the global clip list is partitioned into contiguous blocks, one per
rank; each rank runs the encoder-decoder on its block only. Fusion is split by video: video v is
fused by its owner, the rank whose block holds most of v's clips (ties -> the lower rank), so only
the clips of videos that straddle a block boundary have to move. They move by one all_to_all over
RCCL/xGMI ("owner-gather") as a single fp32 plane per clip frame, the logit
margin d = l1 - l0: the 2-class softmax the reference takes (src/fuse_utils.py:60) depends on the
logits only through fl(l1 - l0) (max-subtraction makes one exponent exp(0) = 1 and the other
exp(-|d|)), so fusing from d is bit-identical to fusing from both logit planes at half the bytes.
When every video lies inside one block -- e.g. equal-length videos, a whole number per rank, the
weak-scaling layouts of bench.py -- nothing crosses xGMI and the collective is skipped on every rank
(the decision is a pure function of the global plan, so all ranks agree). The result is
bit-identical to the 1-GPU run: the per-clip computation is placement independent.
``all_gather_clips`` / ``run_clip_shard`` (every rank gets every clip) remain for callers that need
all logits everywhere.
"""
import torch
import torch.distributed as dist

from . import fuse_utils as FU


def shard_bounds(n, rank, world):
    """Contiguous block [lo, hi) of n items for rank; sizes differ by at most one."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def global_clip_plan(video_lengths, num_clips, step, interpolate_last=True):
    """Per video: (K, table, clip0) and the global offset of its first clip."""
    plans, off = [], 0
    for t in video_lengths:
        k = FU.clamp_num_clips(t, num_clips, step)
        if k == 0:
            raise IndexError("list index out of range")
        table, clip0 = FU.clip_table(t, k, step, interpolate_last)
        plans.append({"T": t, "K": k, "table": table, "clip0": clip0, "offset": off, "n": len(table)})
        off += len(table)
    return plans, off


def all_gather_clips(local, n_total, rank, world, group=None, force=False):
    """Gather per-clip tensors (n_local, ...) from every rank into (n_total, ...) in global order.
    Blocks are padded to the largest shard so one all_gather_into_tensor moves everything.
    ``force``: run the collective even on one rank (tests drive RCCL with a world-size-1 group)."""
    if world == 1 and not force:
        return local
    sizes = [shard_bounds(n_total, r, world) for r in range(world)]
    mx = max(hi - lo for lo, hi in sizes)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    if dist.get_backend(group) == "gloo":  # CPU test path: gloo has no all_gather_into_tensor
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
        out = torch.cat(bufs)
    else:
        out = torch.empty((world * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, pad, group=group)
    parts = [out[r * mx: r * mx + (hi - lo)] for r, (lo, hi) in enumerate(sizes)]
    return torch.cat(parts)


def run_clip_shard(n_total, rank, world, compute, empty):
    """Run ``compute(lo, hi) -> (hi-lo, ...)`` on this rank's block of the global clip list and
    all-gather every block: returns the (n_total, ...) result in global clip order on every rank.
    ``empty`` is a zero-row tensor of the right trailing shape/dtype/device for an idle rank."""
    lo, hi = shard_bounds(n_total, rank, world)
    local = compute(lo, hi) if hi > lo else empty
    return all_gather_clips(local.contiguous(), n_total, rank, world)


def video_owners(plans, world):
    """Owner rank of every video: the rank whose shard_bounds block holds most of its clips (ties
    -> the lower rank). A video that lies inside one block is owned by the rank that computes it."""
    n_total = sum(p["n"] for p in plans)
    blocks = [shard_bounds(n_total, r, world) for r in range(world)]
    owners = []
    for p in plans:
        a, b = p["offset"], p["offset"] + p["n"]
        best, best_n = 0, -1
        for r, (lo, hi) in enumerate(blocks):
            n = max(0, min(b, hi) - max(a, lo))
            if n > best_n:
                best, best_n = r, n
        owners.append(best)
    return owners


def owner_of_clips(plans, world):
    """Owner rank of every global clip (the owner of its video, see video_owners)."""
    own = []
    for o, p in zip(video_owners(plans, world), plans):
        own.extend([o] * p["n"])
    return own


def exchange_counts(owners, world):
    """counts[s][o] = clips computed by rank s (its shard_bounds block) and fused by rank o."""
    n_total = len(owners)
    counts = [[0] * world for _ in range(world)]
    for s_ in range(world):
        lo, hi = shard_bounds(n_total, s_, world)
        for g in range(lo, hi):
            counts[s_][owners[g]] += 1
    return counts


def rows_exchanged(owners, world):
    """Clips that cross ranks in exchange_to_owners (0: the collective is skipped)."""
    c = exchange_counts(owners, world)
    return sum(c[s_][o] for s_ in range(world) for o in range(world) if s_ != o)


def exchange_to_owners(local, owners, rank, world, group=None, force=False):
    """Route per-clip rows to their owners. ``local`` holds rows [lo, hi) of the global clip list
    (this rank's shard_bounds block); ``owners[g]`` is the owner rank of global clip g. Returns the
    rows of every clip this rank owns, in global clip order. One all_to_all_single; skipped when no
    clip is computed away from its owner (all ranks derive that from the same plan) unless ``force``
    (tests drive RCCL with a world-size-1 group)."""
    n_total = len(owners)
    counts = exchange_counts(owners, world)
    lo, hi = shard_bounds(n_total, rank, world)
    if not force and (world == 1 or rows_exchanged(owners, world) == 0):
        keep = [g - lo for g in range(lo, hi) if owners[g] == rank]
        if len(keep) == hi - lo:
            return local
        return local[torch.tensor(keep, dtype=torch.long, device=local.device)]
    order = sorted(range(lo, hi), key=lambda g: (owners[g], g))  # by destination, then global order
    send = local[torch.tensor([g - lo for g in order], dtype=torch.long, device=local.device)] if order else local
    send_sizes = counts[rank]
    recv_sizes = [counts[s_][rank] for s_ in range(world)]
    # gloo (the CPU / several-ranks-on-one-GPU rehearsal of the RCCL path) exchanges host tensors
    stage = local.is_cuda and dist.get_backend(group) == "gloo"
    dev = "cpu" if stage else local.device
    out = torch.empty((sum(recv_sizes),) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    dist.all_to_all_single(out, send.contiguous().to(dev), output_split_sizes=recv_sizes, input_split_sizes=send_sizes,
                           group=group)
    # source blocks are in rank order and each is in global order: global order overall
    return out.to(local.device) if stage else out


def videos_needed(lengths, num_clips, step, rank, world, interpolate_last=True):
    """Indices of the videos rank must hold on its device: those with a clip in its block. A rank
    only materialises these (e.g. config[2], 64 videos over 8 ranks: 8 per rank)."""
    plans, n_total = global_clip_plan(lengths, num_clips, step, interpolate_last)
    lo, hi = shard_bounds(n_total, rank, world)
    return [vi for vi, p in enumerate(plans) if max(lo, p["offset"]) < min(hi, p["offset"] + p["n"])]


def exchange_stats(lengths, num_clips, step, world, h=112, w=112, interpolate_last=True):
    """(clips crossing ranks, bytes on the wire) of one sharded pass over videos of these lengths:
    one fp32 logit-margin plane of 32 frames per exchanged clip."""
    plans, _ = global_clip_plan(lengths, num_clips, step, interpolate_last)
    rows = rows_exchanged(owner_of_clips(plans, world), world) if world > 1 else 0
    return rows, rows * FU.CLIP * h * w * 4


def segment_videos_sharded(videos_dev, model, num_clips=5, step=1, fuse_method="simple", interpolate_last=True,
                           rank=0, world=1, batch_size=None, clip_fn=None, lengths=None, force_exchange=False,
                           exchange_events=None):
    """Fuse a batch of device videos (each (3,T,H,W)) with clips sharded over ranks.

    Returns {video index: fused (T',H,W) uint8 device tensor} for the videos this rank owns
    (video_owners). ``clip_fn(clips) -> logits`` overrides the model call. With ``lengths`` (the
    frame count of every video) ``videos_dev`` may hold None for videos outside this rank's block
    (``videos_needed``). ``force_exchange``: ship logit margins through the all_to_all even when no
    clip crosses ranks (tests; the result is the same). ``exchange_events``: a list that receives one
    (start, end) pair of timing events on the current stream around the margin computation and the
    all_to_all, when the exchange runs (bench.py reports their elapsed time)."""
    if lengths is None:
        lengths = [v.shape[1] for v in videos_dev]
    plans, n_total = global_clip_plan(list(lengths), num_clips, step, interpolate_last)
    present = [v for v in videos_dev if v is not None]
    if not present:
        raise ValueError("no video tensor on this rank")
    h, w = present[0].shape[-2:]
    dev = present[0].device

    def compute(lo, hi):
        mine = []
        for vi, p in enumerate(plans):  # overlap of each video's clip range with [lo, hi)
            a, b = max(lo, p["offset"]), min(hi, p["offset"] + p["n"])
            if a < b:
                if videos_dev[vi] is None:
                    raise ValueError(f"video {vi} has clips in rank {rank}'s block but is not on this rank")
                mine.append(FU.build_clips(videos_dev[vi], p["table"][a - p["offset"]: b - p["offset"]],
                                           interpolate_last))
        clips = torch.cat(mine) if len(mine) > 1 else mine[0]
        return clip_fn(clips) if clip_fn else FU.run_model(model, clips, batch_size)

    empty = torch.empty((0, 2, FU.CLIP, h, w), device=dev, dtype=torch.float32)
    lo, hi = shard_bounds(n_total, rank, world)
    local = compute(lo, hi) if hi > lo else empty
    owners = owner_of_clips(plans, world)
    margin = force_exchange or (world > 1 and rows_exchanged(owners, world) > 0)
    ev = None
    if margin and exchange_events is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    if margin:  # ship one fp32 plane per clip frame instead of two (bit-identical labels, see above)
        local = FU.logit_margin(local) if local.shape[0] else local[:, 0]
    mine = exchange_to_owners(local.contiguous(), owners, rank, world, force=force_exchange)
    if ev is not None:
        ev[1].record()
        exchange_events.append(ev)
    vown = video_owners(plans, world)
    out, at = {}, 0
    for vi, p in enumerate(plans):
        if vown[vi] != rank:
            continue
        lg = mine[at: at + p["n"]]
        at += p["n"]
        labels = FU.pass_labels(lg, p["clip0"], p["T"], step, interpolate_last, margin=margin)
        out[vi] = FU.fuse_votes(labels, step, fuse_method)
    return out

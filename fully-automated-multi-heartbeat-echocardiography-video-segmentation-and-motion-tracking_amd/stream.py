"""Pipelined multi-video front end.

The reference processes one video at a time, synchronously: decode (motion_segment.py:80-94), float
conversion, resize and normalisation on the host (:96-106), then batch-1 clip forwards with a
device->host copy after each (src/fuse_utils.py:53-61) and fusion on the host. Here a stream of
videos flows through the engine with no host synchronisation between videos:

* each video's uint8 frames (the decoder's output, a quarter of the float video's bytes) are staged
  in a reused ring of pinned host buffers and copied to HBM on a dedicated copy stream, one video
  ahead of the compute stream, so PCIe overlaps the previous video's forward;
* resize + zero-one normalisation (clasfv_preprocess_video / clasfv_zeroone_normalize), clip
  building, the batched forward, softmax -> resample -> argmax and label fusion run on the compute
  stream (fuse_utils.segment_a_video_with_fusion_device);
* consecutive videos alternate between ``inflight`` compute streams (the caller's and private ones
  ordered after it), so video i + 1's clip building, stem and layer1 overlap video i's small-grid
  tail -- layer3 / layer4, the decoder, pass labels and fusion (the engine keeps one workspace per
  stream; bench.py measures the same overlap on device-resident videos: +3 % fp32, +5 % bf16);
* the fused uint8 masks go back to one pinned host buffer asynchronously; the host waits once, at
  the end, and widens them to the reference's int64.

Results are identical to calling segment_a_video_with_fusion per video (same kernels, same inputs).
"""
import numpy as np
import torch

from . import fuse_utils as FU
from .preprocess import preprocess_video


class VideoStream:
    """``run(frame_videos) -> [int64 (T', H, W) masks]`` for a list of (T, Hs, Ws, 3) uint8 videos.

    All compute is ordered after the stream that is current for the device when ``run`` is called
    (so ``with torch.cuda.stream(s): vs.run(...)`` works), and that stream is ordered after all of it
    when ``run`` returns device masks; with ``inflight`` > 1 every other video runs on a private
    compute stream. Uploads use a private copy stream and a ring of two pinned staging buffers that
    is reused across videos and calls."""

    RING = 2

    def __init__(self, model, num_clips=5, step=1, fuse_method="simple", height=112, width=112,
                 batch_size=None, interpolate_last=True, strict_reference=True, inflight=2):
        self.model = model
        self.device = FU._device_of(model)
        self.kw = dict(interpolate_last=interpolate_last, step=step, num_clips=num_clips, fuse_method=fuse_method,
                       batch_size=batch_size, strict_reference=strict_reference)
        self.height, self.width = height, width
        self.copy_stream = torch.cuda.Stream(self.device)
        self.lanes = [torch.cuda.Stream(self.device) for _ in range(max(1, inflight) - 1)]  # private compute streams
        self._ring = [None] * self.RING     # pinned uint8 staging buffers
        self._ring_ev = [None] * self.RING  # copy-stream event of the H2D last issued from each slot
        self._slot = 0

    def _staging(self, nbytes):
        """Next ring slot with room for nbytes; waits (host) until the H2D last issued from it has
        finished reading it."""
        i = self._slot
        self._slot = (i + 1) % self.RING
        if self._ring_ev[i] is not None:
            self._ring_ev[i].synchronize()
        if self._ring[i] is None or self._ring[i].numel() < nbytes:
            self._ring[i] = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
        return i, self._ring[i][:nbytes]

    def _upload(self, frames):
        """Copy into a pinned ring slot + async H2D on the copy stream; returns (device tensor, ready event)."""
        host = frames if torch.is_tensor(frames) else torch.from_numpy(np.ascontiguousarray(frames))
        if host.dtype != torch.uint8 or host.dim() != 4 or host.shape[-1] != 3:
            raise ValueError(f"expected (T,H,W,3) uint8 frames, got {tuple(host.shape)} {host.dtype}")
        if host.is_pinned():
            src, slot = host, None
        else:
            slot, buf = self._staging(host.numel())
            src = buf.view(host.shape)
            src.copy_(host)
        with torch.cuda.stream(self.copy_stream):
            dev = src.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        if slot is not None:
            self._ring_ev[slot] = ev
        return dev, ev, (host if slot is None else None)

    def run(self, frame_videos, return_device=False):
        videos = list(frame_videos)
        if not videos:
            return []
        compute = torch.cuda.current_stream(self.device)
        lanes = [compute] + self.lanes
        for ls in self.lanes:
            ls.wait_stream(compute)
        outs, keep, host_out = [], [], []
        pending = self._upload(videos[0])
        for i in range(len(videos)):
            dev, ev, pinned_src = pending
            if i + 1 < len(videos):  # the next video's PCIe copy overlaps this video's compute
                pending = self._upload(videos[i + 1])
            cs = lanes[i % len(lanes)]
            cs.wait_event(ev)
            dev.record_stream(cs)  # allocated on the copy stream, used on the compute stream
            with torch.cuda.stream(cs):
                video = preprocess_video(dev, self.height, self.width, device=self.device)
                fused = FU.segment_a_video_with_fusion_device(video, self.model, **self.kw)
            if cs is not compute:
                fused.record_stream(compute)  # read by the caller's stream (D2H copies, return_device)
            if return_device:
                outs.append(fused)
            else:
                outs.append(fused)
                host_out.append(fused.shape)
            if pinned_src is not None:
                keep.append(pinned_src)  # caller-pinned sources stay alive until their copies retire
        for ls in self.lanes:
            compute.wait_stream(ls)
        if return_device:
            compute.synchronize()
            self.copy_stream.synchronize()
            return outs
        # one pinned buffer for every mask of the call, filled by async D2H copies on the compute stream
        total = sum(int(np.prod(sh)) for sh in host_out)
        flat = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=True)
        res, at = [], 0
        for fused in outs:
            n = fused.numel()
            dst = flat[at:at + n].view(fused.shape)
            dst.copy_(fused, non_blocking=True)
            res.append(dst)
            at += n
        compute.synchronize()
        self.copy_stream.synchronize()
        return [r.numpy().astype(np.int64) for r in res]


def segment_videos(frame_videos, model, num_clips=5, step=1, fuse_method="simple", height=112, width=112,
                   batch_size=None, strict_reference=True):
    """Convenience wrapper: VideoStream(...).run(frame_videos)."""
    return VideoStream(model, num_clips, step, fuse_method, height, width, batch_size,
                       strict_reference=strict_reference).run(frame_videos)

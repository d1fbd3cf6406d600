"""Pipelined multi-video front end.

The reference processes one video at a time, synchronously: decode (motion_segment.py:80-94), float
conversion, resize and normalisation on the host (:96-106), then batch-1 clip forwards with a
device->host copy after each (src/fuse_utils.py:53-61) and fusion on the host. Here a stream of
videos flows through the engine with no host synchronisation between videos:

* each video's uint8 frames (the decoder's output, a quarter of the float video's bytes) are copied
  from pinned host memory to HBM on a dedicated copy stream, one video ahead of the compute stream,
  so PCIe overlaps the previous video's forward;
* resize + zero-one normalisation (clasfv_preprocess_video / clasfv_zeroone_normalize), clip
  building, the batched forward, softmax -> resample -> argmax and label fusion run on the compute
  stream (fuse_utils.segment_a_video_with_fusion_device);
* the fused uint8 masks go back to pinned host buffers asynchronously; the host waits once, at the
  end, and widens them to the reference's int64.

Results are identical to calling segment_a_video_with_fusion per video (same kernels, same inputs).
"""
import numpy as np
import torch

from . import fuse_utils as FU
from .preprocess import preprocess_video


class VideoStream:
    """``run(frame_videos) -> [int64 (T', H, W) masks]`` for a list of (T, Hs, Ws, 3) uint8 videos."""

    def __init__(self, model, num_clips=5, step=1, fuse_method="simple", height=112, width=112,
                 batch_size=None, interpolate_last=True):
        self.model = model
        self.device = FU._device_of(model)
        self.kw = dict(interpolate_last=interpolate_last, step=step, num_clips=num_clips, fuse_method=fuse_method,
                       batch_size=batch_size)
        self.height, self.width = height, width
        self.copy_stream = torch.cuda.Stream(self.device)
        self.compute_stream = torch.cuda.current_stream(self.device)

    def _upload(self, frames):
        """Pinned host copy + async H2D on the copy stream; returns (device tensor, ready event)."""
        host = frames if torch.is_tensor(frames) else torch.from_numpy(np.ascontiguousarray(frames))
        if host.dtype != torch.uint8 or host.dim() != 4 or host.shape[-1] != 3:
            raise ValueError(f"expected (T,H,W,3) uint8 frames, got {tuple(host.shape)} {host.dtype}")
        if not host.is_pinned():
            host = host.pin_memory()
        with torch.cuda.stream(self.copy_stream):
            dev = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        return dev, ev, host

    def run(self, frame_videos, return_device=False):
        videos = list(frame_videos)
        if not videos:
            return []
        outs, keep = [], []
        pending = self._upload(videos[0])
        for i in range(len(videos)):
            dev, ev, host = pending
            if i + 1 < len(videos):  # the next video's PCIe copy overlaps this video's compute
                pending = self._upload(videos[i + 1])
            self.compute_stream.wait_event(ev)
            dev.record_stream(self.compute_stream)  # allocated on the copy stream, used here
            video = preprocess_video(dev, self.height, self.width, device=self.device)
            fused = FU.segment_a_video_with_fusion_device(video, self.model, **self.kw)
            if return_device:
                outs.append(fused)
            else:
                h = torch.empty(fused.shape, dtype=torch.uint8, pin_memory=True)
                h.copy_(fused, non_blocking=True)
                outs.append(h)
            keep.append(host)  # pinned source buffers stay alive until the copies retire
        torch.cuda.current_stream(self.device).synchronize()
        self.copy_stream.synchronize()
        if return_device:
            return outs
        return [o.numpy().astype(np.int64) for o in outs]


def segment_videos(frame_videos, model, num_clips=5, step=1, fuse_method="simple", height=112, width=112,
                   batch_size=None):
    """Convenience wrapper: VideoStream(...).run(frame_videos)."""
    return VideoStream(model, num_clips, step, fuse_method, height, width, batch_size).run(frame_videos)

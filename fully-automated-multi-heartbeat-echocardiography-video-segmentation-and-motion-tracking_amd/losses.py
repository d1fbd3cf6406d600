"""Training-side CLAS-FV losses on the HIP warp.

Drop-ins, by name, argument meaning and value, for ``src/clasfv_losses.py`` and the helpers it uses
from ``src/loss_functions.py``. The definitions are re-derived from SURVEY.md sections 3.3 / 3.5:

* ``deformation_motion_loss(source_videos, motion_field)`` (OTA, src/clasfv_losses.py:29-56): every
  frame t < T-1 is warped onto frame t+1 with the forward field (channels 0,1 at t) and frame t+1
  onto frame t with the backward field (channels 2,3 at t+1); the loss is the per-pair mean squared
  error plus 0.005 x the smoothness penalty of both fields, summed over pairs, / 2 / (T-1).
  Here all T-1 frame pairs are warped by ONE ``clasfv_warp`` launch each way (time folded into the
  batch dimension; the warp is per-image independent, so every warped frame is bit-identical to
  the frame-by-frame form).
* ``motion_seg_loss(label_ed, label_es, ed_index, es_index, motion_output, seg_softmax, start, end,
  seg_criterion)`` (SGS / OTS, src/clasfv_losses.py:71-136): the one-hot ED and ES labels are
  propagated frame by frame through the forward fields to the end of the clip and through the
  backward fields to its start; each propagated label is scored with ``seg_criterion`` against the
  softmax of the frame it lands on, except the ED->ES and ES->ED landings, which are scored with a
  Dice loss against the true ES / ED labels (OTS). Returns (flow_loss / (2 (T-2)), ots_loss / 2).
  The ED- and ES-seeded chains of one direction share their motion fields frame by frame, so they
  advance together: one stacked warp per frame instead of two.
* ``DiceLoss`` (src/clasfv_losses.py:11-26), ``huber_loss`` (src/loss_functions.py:66-77),
  ``convert_to_1hot`` (src/loss_functions.py:123-134), ``categorical_dice`` (the numpy metric).
"""
import numpy as np
import torch
from torch import nn

from .echo import categorical_dice  # noqa: F401  (re-exported: src/clasfv_losses.py:60-68)
from .warp import warp


def soft_dice_loss(pred, target, smooth=1.0):
    """1 - (2 <pred, target> + smooth) / (|pred|_1 + |target|_1 + smooth) over all elements."""
    p, t = pred.reshape(-1), target.reshape(-1)
    return 1 - (2.0 * torch.dot(p, t) + smooth) / (p.sum() + t.sum() + smooth)


class DiceLoss(nn.Module):
    """nn.Module form of soft_dice_loss; ``forward(inputs, targets, smooth=1)``."""

    def __init__(self, weight=None, size_average=True):
        super().__init__()

    def forward(self, inputs, targets, smooth=1):
        return soft_dice_loss(inputs, targets, smooth)


def _smoothness(field):
    """Per-leading-index smoothness of a (..., N, C, H, W) field: sqrt(0.01 + (sum of squared
    differences along W / H + sum along H / W) / N)."""
    n, h, w = field.shape[-4], field.shape[-2], field.shape[-1]
    gx = field[..., :, 1:] - field[..., :, :-1]
    gy = field[..., 1:, :] - field[..., :-1, :]
    sx = (gx * gx).sum(dim=(-4, -3, -2, -1))
    sy = (gy * gy).sum(dim=(-4, -3, -2, -1))
    return torch.sqrt(0.01 + (sx / h + sy / w) / n)


def huber_loss(x):
    """Smoothness penalty of one (N,C,H,W) displacement field (src/loss_functions.py:66-77)."""
    return _smoothness(x)


def convert_to_1hot(label, n_class, device=None):
    """(N,1,H,W) integer label map (numpy or tensor) -> (N,n_class,H,W) float32 one-hot on the device."""
    lab = torch.as_tensor(np.asarray(label) if not torch.is_tensor(label) else label)
    if device is None:
        device = lab.device if lab.is_cuda else torch.device("cuda", torch.cuda.current_device())
    lab = lab.to(device=device, dtype=torch.int64)
    classes = torch.arange(n_class, device=device).view(1, n_class, *([1] * (lab.dim() - 2)))
    return (lab == classes).to(torch.float32)


def _time_major(x):
    """(N, C, P, H, W) -> (P*N, C, H, W) with the P frames outermost (contiguous)."""
    n, c, p, h, w = x.shape
    return x.permute(2, 0, 1, 3, 4).reshape(p * n, c, h, w)


def deformation_motion_loss(source_videos, motion_field):
    """OTA loss of source_videos (N,C,T,H,W) under motion_field (N,4,T,H,W), both on the device."""
    n, c, t, h, w = source_videos.shape
    pairs = t - 1
    prev_frames = _time_major(source_videos[:, :, :-1])
    next_frames = _time_major(source_videos[:, :, 1:])
    fwd = motion_field[:, 0:2, :-1]
    bwd = motion_field[:, 2:4, 1:]
    to_next = warp(prev_frames, _time_major(fwd))
    to_prev = warp(next_frames, _time_major(bwd))
    per_pair = lambda d: (d * d).reshape(pairs, -1).mean(dim=1)  # noqa: E731
    mse = per_pair(to_next - next_frames) + per_pair(to_prev - prev_frames)
    smooth = _smoothness(fwd.permute(2, 0, 1, 3, 4)) + _smoothness(bwd.permute(2, 0, 1, 3, 4))
    return (0.005 * smooth.sum() + mse.sum()) / 2 / pairs


def _propagate(seeds, fields, direction, start, end):
    """Advance label chains through per-frame displacement fields.

    seeds: {name: (first_frame, one-hot (N,2,H,W))}; a chain seeded at frame f is warped by
    fields[:, :, f] and lands on f + direction, then by the field of that frame, and so on. As in the
    reference's loops, forward chains run while the landing frame is < end (range(seed, end - 1),
    src/clasfv_losses.py:83,97) and backward chains while the warped frame is > start
    (range(seed, start, -1), :111,125): neither direction looks at the other bound. Chains active
    at the same frame are stacked into one warp launch. Returns {name: [(landing_frame, warped
    label), ...]} in propagation order."""
    n = fields.shape[0]
    frames = {k: f for k, (f, _) in seeds.items()}
    state = {k: lab for k, (_, lab) in seeds.items()}
    out = {k: [] for k in seeds}
    first = min(frames.values()) if direction > 0 else max(frames.values())
    f = first
    while True:
        land = f + direction
        if (land >= end) if direction > 0 else (f <= start):
            break
        active = [k for k in seeds if (frames[k] <= f if direction > 0 else frames[k] >= f)]
        if active:
            stacked = torch.cat([state[k] for k in active])
            moved = warp(stacked, fields[:, :, f].repeat(len(active), 1, 1, 1))
            for i, k in enumerate(active):
                state[k] = moved[i * n:(i + 1) * n]
                out[k].append((land, state[k]))
        f = land
    return out


def motion_seg_loss(label_ed, label_es, ed_index, es_index, motion_output, seg_softmax, start=0, end=32,
                    seg_criterion=DiceLoss()):
    """SGS and OTS losses (see module docstring). Returns (flow_loss, OTS_loss)."""
    dev = motion_output.device
    ed1 = convert_to_1hot(label_ed, 2, dev)
    es1 = convert_to_1hot(label_es, 2, dev)
    ed_index, es_index = int(ed_index), int(es_index)
    fwd = motion_output[:, 0:2]
    bwd = motion_output[:, 2:4]
    flow, ots = 0, 0

    # forward in time: both chains run until they land on frame end-1
    chains = _propagate({"ed": (ed_index, ed1), "es": (es_index, es1)}, fwd, +1, start, end)
    for land, lab in chains["ed"]:
        if land == es_index:
            ots = ots + soft_dice_loss(lab, es1)
        else:
            flow = flow + seg_criterion(seg_softmax[:, :, land], lab)
    for land, lab in chains["es"]:
        flow = flow + seg_criterion(seg_softmax[:, :, land], lab)

    # backward in time: both chains run until they land on frame start
    chains = _propagate({"es": (es_index, es1), "ed": (ed_index, ed1)}, bwd, -1, start, end)
    for land, lab in chains["es"]:
        if land == ed_index:
            ots = ots + soft_dice_loss(lab, ed1)
        else:
            flow = flow + seg_criterion(seg_softmax[:, :, land], lab)
    for land, lab in chains["ed"]:
        flow = flow + seg_criterion(seg_softmax[:, :, land], lab)

    return flow / ((motion_output.shape[2] - 2) * 2), ots / 2

"""Training-side CLAS-FV losses on the HIP warp.

Drop-ins for ``src/clasfv_losses.py`` and the helpers it uses from ``src/loss_functions.py``, with
the same names, arguments and values; every motion warp runs through ``warp.warp`` (the fused
``clasfv_warp`` kernel forward, ``clasfv_warp_backward`` under autograd) instead of
``generate_2dmotion_field`` + ``F.grid_sample``. The reductions around the warps (MSE, Huber
smoothness, Dice) are a handful of small tensor ops and stay in PyTorch.

* ``deformation_motion_loss`` -- OTA loss, src/clasfv_losses.py:29-56
* ``motion_seg_loss``         -- SGS / OTS losses, src/clasfv_losses.py:71-136
* ``DiceLoss``                -- src/clasfv_losses.py:11-26
* ``huber_loss``              -- src/loss_functions.py:66-77
* ``convert_to_1hot``         -- src/loss_functions.py:123-134 (returns a float32 device tensor)
* ``categorical_dice``        -- src/clasfv_losses.py:59-68 (numpy metric, not a loss)
"""
import numpy as np
import torch
from torch import nn

from .warp import warp


class DiceLoss(nn.Module):
    """1 - (2*sum(x*y) + smooth) / (sum(x) + sum(y) + smooth) over all elements."""

    def __init__(self, weight=None, size_average=True):
        super().__init__()

    def forward(self, inputs, targets, smooth=1):
        inputs = inputs.reshape(-1)
        targets = targets.reshape(-1)
        intersection = (inputs * targets).sum()
        dice = (2. * intersection + smooth) / (inputs.sum() + targets.sum() + smooth)
        return 1 - dice


def huber_loss(x):
    """sqrt(0.01 + (sum(dx^2)/H + sum(dy^2)/W) / N) of a (N,C,H,W) field (src/loss_functions.py:66-77)."""
    bsize, _, height, width = x.size()
    d_x = x[:, :, :, 1:] - x[:, :, :, :-1]
    d_y = x[:, :, 1:, :] - x[:, :, :-1, :]
    err = torch.sum(torch.mul(d_x, d_x)) / height + torch.sum(torch.mul(d_y, d_y)) / width
    err /= bsize
    return torch.sqrt(0.01 + err)


def convert_to_1hot(label, n_class, device=None):
    """(N,1,H,W) integer label map (numpy or tensor) -> (N,n_class,H,W) float32 one-hot on the device."""
    lab = torch.as_tensor(np.asarray(label) if not torch.is_tensor(label) else label)
    if device is None:
        device = lab.device if lab.is_cuda else torch.device("cuda", torch.cuda.current_device())
    lab = lab.to(device=device, dtype=torch.int64)
    out = torch.zeros((lab.shape[0], n_class) + tuple(lab.shape[2:]), device=device, dtype=torch.float32)
    return out.scatter_(1, lab, 1.0)


def categorical_dice(prediction, truth, k, epsilon=1e-5):
    a = np.asarray(prediction) == k
    b = np.asarray(truth) == k
    return 2 * np.sum(a * b) / (np.sum(a) + np.sum(b) + epsilon)


def deformation_motion_loss(source_videos, motion_field):
    """OTA loss: warp every frame forward (motion channels 0,1) onto the next and every next frame
    backward (channels 2,3) onto the previous; MSE to the real frames + 0.005 * Huber smoothness of
    both fields, averaged over the T-1 frame pairs. source_videos (N,C,T,H,W), motion_field
    (N,4,T,H,W), both on the device."""
    mse = nn.MSELoss()
    mse_loss = 0
    smooth_loss = 0
    t = source_videos.shape[2]
    for index in range(t - 1):
        forward_motion = motion_field[:, :2, index, ...]
        backward_motion = motion_field[:, 2:, index + 1, ...]
        pred_forward = warp(source_videos[:, :, index, ...], forward_motion)
        pred_backward = warp(source_videos[:, :, index + 1, ...], backward_motion)
        mse_loss += mse(source_videos[:, :, index + 1, ...], pred_forward)
        mse_loss += mse(source_videos[:, :, index, ...], pred_backward)
        smooth_loss += huber_loss(forward_motion)
        smooth_loss += huber_loss(backward_motion)
    return (0.005 * smooth_loss + mse_loss) / 2 / (t - 1)


def motion_seg_loss(label_ed, label_es, ed_index, es_index, motion_output, seg_softmax, start=0, end=32,
                    seg_criterion=DiceLoss()):
    """SGS and OTS losses: the true ED and ES labels are warped (one-hot, bilinear) frame by frame
    forward to the end of the clip and backward to its start through the motion head's fields;
    each warped label is compared with the segmentation softmax of that frame (Dice), and the ED->ES
    / ES->ED warps with the true ES / ED labels. Returns (flow_loss, OTS_loss)."""
    dev = motion_output.device
    one_ed = convert_to_1hot(label_ed, 2, dev)
    one_es = convert_to_1hot(label_es, 2, dev)
    ots = DiceLoss()
    loss_forward = 0
    ots_loss = 0

    flow_source = one_ed
    for frame_index in range(ed_index, end - 1):
        next_label = warp(flow_source, motion_output[:, :2, frame_index, ...])
        if frame_index == (es_index - 1):
            ots_loss += ots(next_label, one_es)
        else:
            loss_forward += seg_criterion(seg_softmax[:, :, frame_index + 1, ...], next_label)
        flow_source = next_label

    flow_source = one_es
    for frame_index in range(es_index, end - 1):
        next_label = warp(flow_source, motion_output[:, :2, frame_index, ...])
        loss_forward += seg_criterion(seg_softmax[:, :, frame_index + 1, ...], next_label)
        flow_source = next_label

    flow_source = one_es
    loss_backward = 0
    for frame_index in range(es_index, start, -1):
        next_label = warp(flow_source, motion_output[:, 2:, frame_index, ...])
        if frame_index == ed_index + 1:
            ots_loss += ots(next_label, one_ed)
        else:
            loss_backward += seg_criterion(seg_softmax[:, :, frame_index - 1, ...], next_label)
        flow_source = next_label

    flow_source = one_ed
    for frame_index in range(ed_index, start, -1):
        next_label = warp(flow_source, motion_output[:, 2:, frame_index, ...])
        loss_backward += seg_criterion(seg_softmax[:, :, frame_index - 1, ...], next_label)
        flow_source = next_label

    flow_loss = (loss_forward + loss_backward) / ((motion_output.shape[2] - 2) * 2)
    ots_loss = ots_loss / 2
    return flow_loss, ots_loss

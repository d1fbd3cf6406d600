"""ORACLE (test infrastructure only -- never imported by the product path).

CPU restatement of the motion warp used by the reference's training losses and visualisation:
``generate_2dmotion_field`` (src/transform_utils.py:14-34) followed by
``F.grid_sample(img, grid, mode="bilinear", padding_mode="border", align_corners=False)``
(src/visualization_utils.py:128, src/clasfv_losses.py:45,87).

The reference hard-codes ``.cuda()`` (transform_utils.py:19-20); this restatement runs on torch CPU.
Grid: x = linspace(-1,1,W)[j] + motion[:,0], y = linspace(-1,1,H)[i] + motion[:,1] (the reference's
variable names grid_w/grid_h are swapped, the values are as stated).
"""
import torch
import torch.nn.functional as F


def motion_grid(motion):
    """motion: (N,2,H,W) -> grid (N,H,W,2)."""
    n, _, h, w = motion.shape
    gy, gx = torch.meshgrid(torch.linspace(-1, 1, h), torch.linspace(-1, 1, w), indexing="ij")
    x = gx[None] + motion[:, 0]
    y = gy[None] + motion[:, 1]
    return torch.stack((x, y), 3)


def warp(img, motion, mode="bilinear"):
    """img (N,C,H,W) float32, motion (N,2,H,W) float32 -> warped (N,C,H,W)."""
    img = torch.as_tensor(img).float()
    motion = torch.as_tensor(motion).float()
    return F.grid_sample(img, motion_grid(motion), mode=mode, padding_mode="border", align_corners=False)


def apply_sequence_deformation(img, motion, start, end, mode="bilinear", forward=True):
    """src/visualization_utils.py:107-130: recursive warp of one frame through motion[:, :, t]."""
    stepv = 1 if forward else -1
    out = img
    for t in range(start, end, stepv):
        m = motion[:, :2, t] if forward else motion[:, 2:, t]
        out = warp(out, m, mode)
    return out

"""Motion-field warp on the HIP engine (``clasfv_warp``).

Reference semantics: ``generate_2dmotion_field`` (src/transform_utils.py:14-34) builds the sampling
grid x = linspace(-1,1,W)[j] + motion[:,0], y = linspace(-1,1,H)[i] + motion[:,1], and
``F.grid_sample(img, grid, mode="bilinear", padding_mode="border", align_corners=False)`` samples it
(src/visualization_utils.py:128, src/clasfv_losses.py:45,87). The kernel fuses both: the grid is
never materialised. ``apply_sequence_deformation`` (src/visualization_utils.py:107-130) chains warps
through the motion head's per-frame fields.

``warp`` is differentiable: under autograd it runs through ``clasfv_warp_backward`` (gradients of
img and motion), which is what the training losses (src/clasfv_losses.py:29-136, ``losses.py``)
backpropagate through.
"""
import torch

from . import _lib


def _check(img, motion):
    if img.dim() != 4 or motion.dim() != 4 or motion.shape[1] != 2:
        raise ValueError("img (N,C,H,W) and motion (N,2,H,W) expected")
    n, c, h, w = img.shape
    if tuple(motion.shape) != (n, 2, h, w):
        raise ValueError(f"motion shape {tuple(motion.shape)} does not match image {tuple(img.shape)}")
    if motion.stride(3) != 1 or motion.stride(2) != w:
        motion = motion.contiguous()
    return img.contiguous(), motion


def _warp_forward(img, motion, out=None):
    img, motion = _check(img, motion)
    n, c, h, w = img.shape
    if out is None:
        out = torch.empty_like(img)
    lib = _lib.load()
    _lib.check(lib.clasfv_warp(_lib.ptr(img), n, c, h, w, _lib.ptr(motion), motion.stride(0), motion.stride(1),
                               _lib.ptr(out), _lib.stream_ptr(device=img.device)), "clasfv_warp")
    return out


class _Warp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, motion):
        img, motion = _check(img, motion)
        ctx.save_for_backward(img, motion)
        return _warp_forward(img, motion)

    @staticmethod
    def backward(ctx, grad_out):
        img, motion = ctx.saved_tensors
        n, c, h, w = img.shape
        gimg = torch.zeros_like(img) if ctx.needs_input_grad[0] else None
        gmot = torch.empty((n, 2, h, w), device=img.device, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        if gimg is None and gmot is None:
            return None, None
        grad_out = grad_out.contiguous()
        lib = _lib.load()
        nul = _lib.ctypes.c_void_p(0)
        _lib.check(lib.clasfv_warp_backward(_lib.ptr(grad_out), _lib.ptr(img), n, c, h, w, _lib.ptr(motion),
                                            motion.stride(0), motion.stride(1),
                                            _lib.ptr(gimg) if gimg is not None else nul,
                                            _lib.ptr(gmot) if gmot is not None else nul,
                                            _lib.stream_ptr(device=img.device)),
                   "clasfv_warp_backward")
        return gimg, gmot


def warp(img, motion, out=None):
    """img (N,C,H,W) float32 on the device, motion (N,2,H,W) (any strides on N and the channel
    dim; H,W contiguous) -> warped (N,C,H,W) = grid_sample(img, generate_2dmotion_field(img, motion),
    bilinear, border, align_corners=False). Differentiable in img and motion."""
    if torch.is_grad_enabled() and (img.requires_grad or motion.requires_grad):
        if out is not None:
            raise ValueError("out= is not supported under autograd")
        return _Warp.apply(img, motion)
    return _warp_forward(img, motion, out)


def generate_2dmotion_field(x, offset):
    """Reference-compatible grid (N,H,W,2) for callers that use F.grid_sample themselves."""
    n, _, h, w = x.shape
    gy, gx = torch.meshgrid(torch.linspace(-1, 1, h), torch.linspace(-1, 1, w), indexing="ij")
    gx, gy = gx.to(offset.device), gy.to(offset.device)
    return torch.stack((gx[None] + offset[:, 0], gy[None] + offset[:, 1]), 3)


def apply_sequence_deformation(img, motion, start_index, end_index, forward=True):
    """Recursively warp one frame img (N,C,H,W) through motion (N,4,T,H,W) frames
    start_index..end_index (exclusive), forward fields (channels 0,1) or backward (2,3)."""
    stepv = 1 if forward else -1
    cur = img.contiguous()
    ch = slice(0, 2) if forward else slice(2, 4)
    for t in range(start_index, end_index, stepv):
        cur = warp(cur, motion[:, ch, t])
    return cur

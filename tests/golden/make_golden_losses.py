"""Generate tests/golden/losses.npz by running the REFERENCE's training losses and warp backward.

Imports /root/reference/src/clasfv_losses.py (deformation_motion_loss, motion_seg_loss) and
src/transform_utils.generate_2dmotion_field with the stubs of make_golden.py, on torch CPU
(``torch.Tensor.cuda`` patched to the identity: the reference hard-codes .cuda()). Records the loss
values and the autograd gradients w.r.t. every differentiable input, plus the gradients of one
plain warp (generate_2dmotion_field + F.grid_sample(border, align_corners=False)). Inputs are
regenerated from the seeds in tests (``loss_inputs``). Run: ``python tests/golden/make_golden_losses.py``.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.dont_write_bytecode = True


def loss_inputs(T=6, H=32, W=40, seed=17):
    """Seeded inputs shared by this script and tests/test_gpu.py."""
    rng = np.random.Generator(np.random.PCG64(seed))
    video = rng.uniform(0, 1, (1, 3, T, H, W)).astype(np.float32)
    motion = np.tanh(rng.normal(0, 0.15, (1, 4, T, H, W))).astype(np.float32)
    logits = rng.normal(0, 1, (1, 2, T, H, W)).astype(np.float32)
    yy, xx = np.mgrid[0:H, 0:W]
    ed = ((((yy - H / 2) / 10.0) ** 2 + ((xx - W / 2) / 7.0) ** 2) <= 1).astype(np.int64)[None, None]
    es = ((((yy - H / 2) / 7.0) ** 2 + ((xx - W / 2) / 5.0) ** 2) <= 1).astype(np.int64)[None, None]
    warp_img = rng.uniform(0, 1, (2, 3, H, W)).astype(np.float32)
    warp_motion = np.tanh(rng.normal(0, 0.3, (2, 2, H, W))).astype(np.float32)
    warp_gout = rng.normal(0, 1, (2, 3, H, W)).astype(np.float32)
    return dict(video=video, motion=motion, logits=logits, ed=ed, es=es, ed_index=1, es_index=4,
                warp_img=warp_img, warp_motion=warp_motion, warp_gout=warp_gout)


# extra motion_seg_loss cases (ed_index, es_index, start, end): ES before ED, and a window that
# starts after the seed frames (the reference's forward loops ignore `start`, its backward loops `end`)
SGS_CASES = [(4, 1, 0, 6), (1, 4, 2, 6), (0, 3, 1, 5), (3, 2, 2, 4)]


def main():
    from tests.golden.make_golden import REF, install_stubs
    install_stubs()
    sys.path.insert(0, REF)
    torch.Tensor.cuda = lambda self, *a, **k: self
    from src.clasfv_losses import deformation_motion_loss, motion_seg_loss
    from src.transform_utils import generate_2dmotion_field
    d = loss_inputs()
    out = {}
    video = torch.from_numpy(d["video"]).requires_grad_()
    motion = torch.from_numpy(d["motion"]).requires_grad_()
    loss = deformation_motion_loss(video, motion)
    loss.backward()
    out["ota_loss"] = np.float64(loss.item())
    out["ota_grad_video"] = video.grad.numpy()
    out["ota_grad_motion"] = motion.grad.numpy()

    motion = torch.from_numpy(d["motion"]).requires_grad_()
    logits = torch.from_numpy(d["logits"]).requires_grad_()
    seg_softmax = F.softmax(logits, dim=1)
    flow, ots = motion_seg_loss(d["ed"], d["es"], d["ed_index"], d["es_index"], motion, seg_softmax,
                                start=0, end=d["video"].shape[2])
    (flow + ots).backward()
    out["sgs_flow_loss"] = np.float64(flow.item())
    out["sgs_ots_loss"] = np.float64(ots.item())
    out["sgs_grad_motion"] = motion.grad.numpy()
    out["sgs_grad_logits"] = logits.grad.numpy()

    for i, (ed_i, es_i, start, end) in enumerate(SGS_CASES):
        motion = torch.from_numpy(d["motion"]).requires_grad_()
        logits = torch.from_numpy(d["logits"]).requires_grad_()
        flow, ots = motion_seg_loss(d["ed"], d["es"], ed_i, es_i, motion, F.softmax(logits, dim=1), start=start, end=end)
        total = flow + ots
        if torch.is_tensor(total) and total.requires_grad:
            total.backward()
        out[f"sgs{i}_flow_loss"] = np.float64(float(flow))
        out[f"sgs{i}_ots_loss"] = np.float64(float(ots))
        out[f"sgs{i}_grad_motion"] = motion.grad.numpy() if motion.grad is not None else np.zeros_like(d["motion"])
        out[f"sgs{i}_grad_logits"] = logits.grad.numpy() if logits.grad is not None else np.zeros_like(d["logits"])

    img = torch.from_numpy(d["warp_img"]).requires_grad_()
    mot = torch.from_numpy(d["warp_motion"]).requires_grad_()
    grid = generate_2dmotion_field(img, mot)
    # the reference builds the grid as (offset_h, offset_w) stacked: x from channel 0, y from channel 1
    warped = F.grid_sample(img, grid, align_corners=False, padding_mode="border")
    warped.backward(torch.from_numpy(d["warp_gout"]))
    out["warp_out"] = warped.detach().numpy()
    out["warp_grad_img"] = img.grad.numpy()
    out["warp_grad_motion"] = mot.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "losses.npz"), **out)
    print({k: (np.shape(v), float(np.sum(v))) for k, v in out.items()})


if __name__ == "__main__":
    main()

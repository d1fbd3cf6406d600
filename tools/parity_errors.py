"""Measure the fp32 forward's max |error| on every shape the GPU parity tests check, so that the
test tolerances can sit just above the measured error (not orders of magnitude above it).

Run on the GPU box: python tools/parity_errors.py > gpurun_out/parity_errors.txt
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import fuse_ref, r2plus1d_ref  # noqa: E402


def main():
    import clasfv_amd.synthetic as S
    import clasfv_amd.weights as W
    from clasfv_amd.model import R2plus1D_18_MotionNet
    torch.set_num_threads(16)
    sd = W.synthetic_state_dict(W.DEFAULT_SEED)
    model = R2plus1D_18_MotionNet(pretrained=False)
    g = np.load(os.path.join(REPO, "tests", "golden", "model_forward.npz"))

    def rep(name, got, ref):
        got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
        d = np.abs(got - ref)
        print(f"{name:48s} max|d|={d.max():.3e}  p99.99={np.quantile(d, 0.9999):.3e}  max|ref|={np.abs(ref).max():.2f}",
              flush=True)

    seg, mot = model(torch.from_numpy(g["x_small"]))
    rep("small golden seg", seg.cpu().numpy(), g["seg_small"])
    rep("small golden mot", mot.cpu().numpy(), g["mot_small"])
    v = fuse_ref.zeroone_normalizer(S.echo_video(int(g["big_T"]), seed=int(g["big_video_seed"])))
    s = int(g["big_start"])
    seg, mot = model(torch.from_numpy(np.ascontiguousarray(v[None, :, s:s + 32])))
    idx = g["big_idx"]
    rep("full clip golden seg0", seg[0, 0].cpu().numpy().ravel()[idx], g["big_seg0"])
    rep("full clip golden seg1", seg[0, 1].cpu().numpy().ravel()[idx], g["big_seg1"])
    rep("full clip golden mot", mot[0].cpu().numpy().reshape(4, -1)[:, idx], g["big_mot"])
    for shape in [(2, 3, 16, 64, 48), (1, 3, 8, 16, 32), (3, 3, 24, 32, 32), (2, 3, 16, 64, 96), (1, 3, 8, 32, 48)]:
        x = np.random.default_rng(sum(shape)).uniform(0, 1, shape).astype(np.float32)
        seg, mot = model(torch.from_numpy(x))
        rs, rm = r2plus1d_ref.forward(sd, x)
        rep(f"oracle {shape} seg", seg.cpu().numpy(), rs.numpy())
        rep(f"oracle {shape} mot", mot.cpu().numpy(), rm.numpy())
    x = torch.from_numpy(np.random.default_rng(0).uniform(0, 1, (1, 3, 8, 32, 32)).astype(np.float32))
    seg, _ = model(x.cuda())
    rs, _ = r2plus1d_ref.forward(sd, x)
    rep("smoke 8x32x32 seg", seg.cpu().numpy(), rs.numpy())
    sd2 = W.synthetic_state_dict(99)
    model.load_state_dict(sd2)
    x = torch.rand(1, 3, 8, 32, 32, generator=torch.Generator().manual_seed(0))
    s2, _ = model(x)
    r2, _ = r2plus1d_ref.forward(sd2, x)
    rep("seed 99 8x32x32 seg", s2.cpu().numpy(), r2.numpy())
    model.load_state_dict(sd)
    x = np.random.default_rng(17).uniform(0, 1, (1, 3, 32, 112, 112)).astype(np.float32)
    t0 = time.time()
    seg, mot = model(torch.from_numpy(x))
    rs, rm = r2plus1d_ref.forward(sd, x)
    rep("oracle (1,3,32,112,112) seg", seg.cpu().numpy(), rs.numpy())
    rep("oracle (1,3,32,112,112) mot", mot.cpu().numpy(), rm.numpy())
    v = fuse_ref.zeroone_normalizer(S.echo_video(64, H=224, W=224, seed=21))
    x = np.ascontiguousarray(v[None])
    seg, mot = model(torch.from_numpy(x))
    rs, rm = r2plus1d_ref.forward_chunked(sd, x, frames_per_chunk=8)
    rep("config3 64x224x224 seg", seg.cpu().numpy(), rs.numpy())
    rep("config3 64x224x224 mot", mot.cpu().numpy(), rm.numpy())
    print(f"done in {time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()

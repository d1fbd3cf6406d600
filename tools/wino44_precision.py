"""Precision pre-check for a Winograd F(4x4,3x3) spatial kernel (CPU only, numpy/torch emulation).

Replaces the stride-1 1x3x3 convs on maps with H, W % 4 == 0 (layer1/layer2: the convs conv_wino_q
runs) by an fp32 emulation of F(2x2,3x3) (today's arithmetic) or F(4x4,3x3) (candidate), runs the
oracle forward on the north_star clip, and prints max |logit error| against a float64 forward.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import r2plus1d_ref  # noqa: E402

MATS = {
    2: (np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64),
        np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], np.float64),
        np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64)),
    4: (np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
                  [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], np.float64),
        np.array([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
                  [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], np.float64),
        np.array([[1, 1, 1, 1, 1, 0], [0, 1, -1, 2, -2, 0], [0, 1, 1, 4, 4, 0], [0, 1, -1, 8, -8, 1]], np.float64)),
}

MODE = {"m": 0}
_conv3d = F.conv3d


def wino(x, w, m):
    BT, G, AT = MATS[m]
    N, C, T, H, W = x.shape
    Co = w.shape[0]
    a = m + 2
    U = np.einsum("ij,ocjk,lk->ilco", G, w[:, :, 0].double().numpy(), G).astype(np.float32)  # (a,a,C,Co)
    xp = F.pad(x, (1, 1, 1, 1))
    th, tw = H // m, W // m
    d = xp.unfold(3, a, m).unfold(4, a, m)  # N,C,T,th,tw,a,a
    BTt = torch.from_numpy(BT.astype(np.float32))
    V = torch.einsum("ij,nctyxjk,lk->ilntyxc", BTt, d, BTt).reshape(a * a, -1, C)
    M = torch.bmm(V, torch.from_numpy(U).reshape(a * a, C, Co)).reshape(a, a, N, T, th, tw, Co)
    ATt = torch.from_numpy(AT.astype(np.float32))
    Y = torch.einsum("ij,jkntyxo,lk->ntyixlo", ATt, M, ATt)  # n t y i x l o
    return Y.reshape(N, T, H, W, Co).permute(0, 4, 1, 2, 3).contiguous()


def conv3d(x, w, b=None, stride=1, padding=0, *args):
    m = MODE["m"]
    if (m and x.dtype == torch.float32 and tuple(w.shape[2:]) == (1, 3, 3) and tuple(stride) == (1, 1, 1)
            and x.shape[3] % 4 == 0 and x.shape[4] % 4 == 0 and x.shape[3] >= 28):
        y = wino(x, w, m)
        return y if b is None else y + b.view(1, -1, 1, 1, 1)
    return _conv3d(x, w, b, stride, padding, *args)


def main():
    import clasfv_amd.synthetic as S
    import clasfv_amd.weights as Wt
    from oracle import fuse_ref
    torch.set_num_threads(8)
    F.conv3d = conv3d
    sd = Wt.echo_state_dict(Wt.DEFAULT_SEED) if hasattr(Wt, "echo_state_dict") else Wt.synthetic_state_dict(Wt.DEFAULT_SEED)
    for name, sdx in [("echo", sd), ("random", Wt.synthetic_state_dict(Wt.DEFAULT_SEED))]:
        v = fuse_ref.zeroone_normalizer(S.echo_video(40, seed=3))
        x = torch.from_numpy(np.ascontiguousarray(v[None, :, 0:32]))
        sd64 = {k: (torch.as_tensor(t).double() if torch.as_tensor(t).is_floating_point() else torch.as_tensor(t))
                for k, t in sdx.items()}
        MODE["m"] = 0
        s64, m64 = r2plus1d_ref.head(sd64, r2plus1d_ref.backbone(sd64, x.double()))
        for m in (0, 2, 4):
            MODE["m"] = m
            s, mo = r2plus1d_ref.forward(sdx, x)
            print(f"{name} F({m}x{m}) seg max|d|={float((s.double() - s64).abs().max()):.3e} "
                  f"mot max|d|={float((mo.double() - m64).abs().max()):.3e} max|seg|={float(s64.abs().max()):.2f}",
                  flush=True)


if __name__ == "__main__":
    main()

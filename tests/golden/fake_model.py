"""Test infrastructure: a cheap deterministic stand-in for the network, used to pin the clip
plumbing (src/fuse_utils.py:36-100) independently of the model. Only exact IEEE elementwise ops
(mul/add/sub/roll), so CPU and GPU evaluations agree bit for bit."""
import numpy as np
import torch

_WAVE = (0.15 * np.sin(np.arange(32) * 0.3) - 0.1).astype(np.float32)


def fake_model(x):
    x = torch.as_tensor(x).float()
    wave = torch.from_numpy(_WAVE).to(x.device)[None, :, None, None]
    s0 = 0.55 - x[:, 0]
    s1 = (0.6 * x[:, 1] + wave) + 0.2 * torch.roll(x[:, 2], 3, dims=2)
    seg = torch.stack([s0, s1], 1)
    return seg, torch.zeros((x.shape[0], 4) + tuple(x.shape[2:]), device=x.device)

"""Run the forward several times / with different batch compositions and report bitwise diffs."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from clasfv_amd.model import R2plus1D_18_MotionNet

m = R2plus1D_18_MotionNet(pretrained=False)
rng = np.random.default_rng(0)
x = torch.from_numpy(rng.uniform(0, 1, (28, 3, 32, 112, 112)).astype(np.float32)).cuda()
ref_s, ref_m = m(x)
ref_s, ref_m = ref_s.clone(), ref_m.clone()
for it in range(5):
    s, mo = m(x)
    print("repeat", it, "seg diff elems", int((s != ref_s).sum()), "mot diff", int((mo != ref_m).sum()), flush=True)
for lo, hi in [(0, 6), (6, 15), (15, 28), (0, 1), (27, 28)]:
    s, mo = m(x[lo:hi])
    print("sub", lo, hi, "seg diff", int((s != ref_s[lo:hi]).sum()), "max", float((s - ref_s[lo:hi]).abs().max()), flush=True)

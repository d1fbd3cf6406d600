"""Per-launch HIP-event timing overhead: 30-clip fp32 forwards timed with the engine's kernel timing
on and off (wall clock over 20 forwards after warm-up). usage (GPU box): python tools/timing_overhead.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clasfv_amd.model import R2plus1D_18_MotionNet  # noqa: E402

m = R2plus1D_18_MotionNet(pretrained=False, dtype="fp32", device="cuda:0")
x = torch.rand(30, 3, 32, 112, 112, device="cuda:0")
for _ in range(3):
    m(x)
torch.cuda.synchronize()
for rnd in range(3):
    for on in (True, False):
        m.engine.set_kernel_timing(on)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            m(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20 * 1e3
        if on:
            m.engine.kernel_timing()
        m.engine.set_kernel_timing(False)
        print(f"round {rnd} timing {'on ' if on else 'off'}: {dt:.3f} ms per 30-clip forward", flush=True)

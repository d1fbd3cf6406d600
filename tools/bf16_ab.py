"""config[4] precision A/B (GPU box): Dice delta and logit error of the bf16 forward against the fp32
forward on an echo-style clip, for every combination of the fp32-MFMA fallbacks of the bf16 stem,
decoder and patch convs (each switch is read once per process: one subprocess per combination)."""
import itertools
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import json, sys, numpy as np, torch
sys.path.insert(0, %r)
import clasfv_amd.synthetic as S
from clasfv_amd.model import R2plus1D_18_MotionNet
from clasfv_amd.echo import categorical_dice
from oracle import fuse_ref
v = fuse_ref.zeroone_normalizer(S.echo_video(64, seed=3))
out = {}
for s0 in (10, 30):
    x = torch.from_numpy(np.ascontiguousarray(v[None, :, s0:s0 + 32]))
    s32, _ = R2plus1D_18_MotionNet(pretrained=False)(x)
    s16, _ = R2plus1D_18_MotionNet(pretrained=False, dtype="bf16")(x)
    a = (s16[:, 1] > s16[:, 0]).cpu().numpy(); b = (s32[:, 1] > s32[:, 0]).cpu().numpy()
    out[s0] = [1 - categorical_dice(a, b, 1), float((s16 - s32).abs().median())]
print(json.dumps(out))
""" % REPO
SW = ["CLASFV_NO_STEM_BF16", "CLASFV_NO_DECODER_BF16", "CLASFV_NO_PATCH_BF16"]
for bits in itertools.product([0, 1], repeat=3):
    env = dict(os.environ, **{k: "1" for k, b in zip(SW, bits) if b})
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    tag = "+".join(k[10:] for k, b in zip(SW, bits) if b) or "default"
    print(tag, r.stdout.strip() if r.returncode == 0 else r.stderr[-500:], flush=True)

"""Generate tests/golden/preprocess.npz: the reference CLI's frame preprocessing run verbatim.

motion_segment.py:96-106 is module-level script code, so its four statements are replayed here on
synthetic cv2-layout frames (T,H,W,3) uint8 -- transpose + astype(float32), torch.Tensor(...).unsqueeze(0),
F.interpolate(size=(T,112,112), mode="trilinear", align_corners=True), squeeze().numpy() -- followed
by the reference's own ``zeroone_normalizer`` (src/echonet_dataset.py:38-50, imported with the stubs
of make_golden.py). Run in the build container: ``python tests/golden/make_golden_preprocess.py``.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.dont_write_bytecode = True

CASES = [  # (T, Hs, Ws, seed): downscale, upscale, identity size
    (12, 150, 200, 13),
    (9, 64, 80, 14),
    (10, 112, 112, 15),
]


def main():
    from tests.golden.make_golden import REF, install_stubs
    install_stubs()
    sys.path.insert(0, REF)
    from src.echonet_dataset import zeroone_normalizer
    import clasfv_amd.synthetic as S
    out = {}
    for i, (T, Hs, Ws, seed) in enumerate(CASES):
        video = S.echo_video_uint8(T, Hs, Ws, seed=seed)
        video = video.transpose((3, 0, 1, 2)).astype(np.float32)          # motion_segment.py:96
        video = torch.Tensor(video).unsqueeze(0)                         # :100
        video = F.interpolate(video, size=(video.shape[2], 112, 112), mode="trilinear", align_corners=True)
        video = video.squeeze().numpy()                                  # :104
        resized = video.copy()
        video = zeroone_normalizer(video)                                # :106
        out[f"case{i}"] = np.array([T, Hs, Ws, seed])
        out[f"resized{i}_sample"] = resized[:, ::2, ::3, ::5]
        out[f"resized{i}_sum"] = resized.astype(np.float64).sum((1, 2, 3))
        out[f"norm{i}_sample"] = video[:, ::2, ::3, ::5]
        out[f"norm{i}_sum"] = video.astype(np.float64).sum((1, 2, 3))
    np.savez_compressed(os.path.join(HERE, "preprocess.npz"), **out)
    print("wrote preprocess.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()

"""Generate tests/golden/northstar_c1.npz (and northstar_c1_random.npz): the CPU reference path at
BASELINE config[1].

One 200-frame synthetic EchoNet-style video (synthetic.echo_video(200, seed=0), zero-one normalised),
5 temporally shifted passes with step 1 (30 clips of 32 frames) -- exactly bench.py's per-GPU
workload -- with one of two seeded weight recipes:
  echo    (northstar_c1.npz)        weights.echo_state_dict(DEFAULT_SEED): the segmentation follows
          the synthetic LV, so the EFs are physiological (~77 %); the LV decision runs through the
          stem, layer1 and the decoder (layer2-4 reach the logits at ~1e-2 of the margin);
  random  (northstar_c1_random.npz) weights.synthetic_state_dict(DEFAULT_SEED): every layer at full
          gain, so every conv of the encoder moves the fused masks (EFs degenerate);
  deep    (northstar_c1_deep.npz, round 6) weights.deep_state_dict(DEFAULT_SEED): the echo
          segmentation routed through layer2-4 at full gain (about 60 % of the band's intensity input
          passes through them), so bf16 rounding anywhere in the encoder reaches masks with
          physiological EFs.
Everything is
computed by the oracle (tests-only infrastructure): the torch-CPU restatement of the reference model
(oracle/r2plus1d_ref.py, pinned to the reference module by tests/golden/model_forward.npz) and the
numpy restatement of src/fuse_utils.py (oracle/fuse_ref.py, pinned by tests/golden/plumbing.npz).

Stored (bit-packed masks):
  passes          the 5 per-pass label videos (pass k has 200 - k frames), concatenated
  fused_<method>  the fused (200,112,112) masks for majority, simple and staple
  ef_<method>     compute_ef_using_putative_clips of each fused mask (EF list and ED/ES pairs)
  logit_margin_*  |l1 - l0| statistics, to tell how close the fused masks are to argmax ties

Run in the build container: python tests/golden/make_golden_northstar.py [echo|random] (about a
minute each).
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import fuse_ref, r2plus1d_ref  # noqa: E402

T, F, STEP, SEED = 200, 5, 1, 0
RECIPE = sys.argv[1] if len(sys.argv) > 1 else "echo"
OUT = {"echo": "northstar_c1.npz", "random": "northstar_c1_random.npz", "deep": "northstar_c1_deep.npz"}[RECIPE]
METHODS = ("majority", "simple", "staple")


def main():
    import clasfv_amd.synthetic as S
    import clasfv_amd.weights as W
    from clasfv_amd.echo import compute_ef_using_putative_clips
    torch.set_num_threads(os.cpu_count() or 8)
    sd = W.recipe_state_dict(RECIPE, W.DEFAULT_SEED)
    model = r2plus1d_ref.OracleModel(sd)
    video = fuse_ref.zeroone_normalizer(S.echo_video(T, seed=SEED))
    k = fuse_ref.clamp_num_clips(T, F, STEP)
    t0 = time.time()
    margins = []

    def logged(x):
        seg, mot = model(x)
        margins.append(np.abs(seg[:, 1] - seg[:, 0]).numpy().ravel())
        return seg, mot

    passes = [fuse_ref.pass_labels(video, logged, s, True, to_numpy=lambda t: t.numpy())
              for s in range(0, k * STEP, STEP)]
    print(f"{sum(len(range(0, fuse_ref.n_clip_frames(T - s), 32)) for s in range(k))} clip forwards "
          f"in {time.time() - t0:.1f} s")
    out = {"T": np.int64(T), "fuse": np.int64(F), "step": np.int64(STEP), "seed": np.int64(SEED),
           "weights_seed": np.int64(W.DEFAULT_SEED), "weights_recipe": np.array(RECIPE),
           "passes": np.packbits(np.concatenate([p.ravel() for p in passes]).astype(np.uint8)),
           "pass_frames": np.array([p.shape[0] for p in passes], np.int64)}
    m = np.concatenate(margins)
    out["logit_margin_quantiles"] = np.quantile(m, [1e-6, 1e-5, 1e-4, 1e-3, 0.5]).astype(np.float64)
    for meth in METHODS:
        fused = fuse_ref.fuse_frames(passes, T, STEP, meth)
        efs, pairs = compute_ef_using_putative_clips(fused, "northstar", return_edes=True)
        out[f"fused_{meth}"] = np.packbits(fused.astype(np.uint8).ravel())
        out[f"fused_{meth}_shape"] = np.array(fused.shape, np.int64)
        out[f"ef_{meth}"] = np.array(efs, np.float64)
        out[f"pairs_{meth}"] = np.array(pairs, np.int64).reshape(-1, 2)
        print(meth, "LV fraction", float(fused.mean()), "EF", np.round(efs, 3), "pairs", pairs)
    np.savez_compressed(os.path.join(HERE, OUT), **out)


if __name__ == "__main__":
    main()

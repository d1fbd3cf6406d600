"""Pin the oracle (CPU restatement) against golden vectors produced by the reference code itself
(tests/golden/make_golden.py). CPU only."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fuse_ref, r2plus1d_ref, warp_ref
from tests.conftest import golden, unpack_labels
from tests.golden.fake_model import fake_model


def _np_model(x):
    seg, mot = fake_model(torch.from_numpy(np.ascontiguousarray(x)))
    return seg.numpy(), mot.numpy()


def test_param_count_and_keys(synthetic_sd):
    import clasfv_amd.arch as A
    g = golden("model_forward.npz")
    assert int(g["nparams"]) == A.NUM_PARAMS_REFERENCE == A.count_parameters()
    assert list(g["keys"]) == list(A.state_dict_spec().keys()) == list(synthetic_sd.keys())


def test_oracle_forward_small_matches_reference(synthetic_sd):
    g = golden("model_forward.npz")
    seg, mot = r2plus1d_ref.forward(synthetic_sd, g["x_small"])
    np.testing.assert_allclose(seg.numpy(), g["seg_small"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(mot.numpy(), g["mot_small"], rtol=0, atol=1e-6)


def test_oracle_forward_full_clip_matches_reference(synthetic_sd):
    import clasfv_amd.synthetic as S
    g = golden("model_forward.npz")
    v = fuse_ref.zeroone_normalizer(S.echo_video(int(g["big_T"]), seed=int(g["big_video_seed"])))
    s = int(g["big_start"])
    x = np.ascontiguousarray(v[None, :, s:s + 32])
    seg, mot = r2plus1d_ref.forward(synthetic_sd, x)
    seg, mot = seg.numpy(), mot.numpy()
    lab = (seg[0, 1] > seg[0, 0]).ravel()
    ref = np.unpackbits(g["big_label_bits"])[: lab.size].astype(bool)
    assert (lab != ref).sum() <= 2
    idx = g["big_idx"]
    np.testing.assert_allclose(seg[0, 0].ravel()[idx], g["big_seg0"], atol=1e-4)
    np.testing.assert_allclose(seg[0, 1].ravel()[idx], g["big_seg1"], atol=1e-4)
    np.testing.assert_allclose(mot[0].reshape(4, -1)[:, idx], g["big_mot"], atol=1e-6)


@pytest.mark.parametrize("tin,tout", [(200, 192), (192, 200), (33, 32), (32, 33), (70, 64), (64, 70), (80, 64),
                                      (199, 192), (160, 199), (48, 64)])
def test_temporal_resample_bitexact_vs_torch(tin, tout):
    rng = np.random.default_rng(tin * 1000 + tout)
    x = rng.random((2, tin, 24, 20), dtype=np.float32)
    ref = F.interpolate(torch.from_numpy(x)[None], size=(tout, 24, 20), mode="trilinear", align_corners=False)[0]
    np.testing.assert_array_equal(fuse_ref.temporal_resample(x, tout), ref.numpy())


def test_plumbing_fusion_off_matches_reference():
    import clasfv_amd.synthetic as S
    g = golden("plumbing.npz")
    for T in (33, 48, 70, 80, 200):
        v = fuse_ref.zeroone_normalizer(S.echo_video(T, seed=T))
        out = fuse_ref.segment_a_video_with_fusion(v, _np_model, num_clips=1)
        ref = unpack_labels(g, f"off_T{T}")
        assert out.shape == ref.shape and out.dtype == np.int64
        np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("T,f,step", [(70, 5, 1), (200, 5, 1), (80, 3, 2), (48, 10, 1), (40, 5, 3)])
def test_plumbing_fusion_on_matches_reference(T, f, step):
    """Vote gathering / frame indexing of the reference with majority voting as fuse_images."""
    import clasfv_amd.synthetic as S
    g = golden("plumbing.npz")
    v = fuse_ref.zeroone_normalizer(S.echo_video(T, seed=100 + T))
    out = fuse_ref.segment_a_video_with_fusion(v, _np_model, step=step, num_clips=f, fuse_method="majority")
    np.testing.assert_array_equal(out, unpack_labels(g, f"on_T{T}_f{f}_s{step}"))
    k = fuse_ref.clamp_num_clips(T, f, step)
    votes = [sum(1 for idx in range(min(i, k)) if i - idx * step >= 0) for i in range(1, T) if step - 1 < i]
    ref_votes = g[f"votes_T{T}_f{f}_s{step}"]
    assert [v_ for v_ in votes if v_ > 1] == list(ref_votes)


def test_plumbing_quirks():
    import clasfv_amd.synthetic as S
    g = golden("plumbing.npz")
    assert str(g["err_T32"]) == "IndexError"
    with pytest.raises(IndexError):
        fuse_ref.segment_a_video_with_fusion(fuse_ref.zeroone_normalizer(S.echo_video(32, seed=32)), _np_model,
                                             num_clips=1)
    clips = fuse_ref.divide_to_consecutive_clips(fuse_ref.zeroone_normalizer(S.echo_video(80, seed=80)), interpolate_last=True)
    assert tuple(clips.shape) == tuple(g["clips80_shape"])
    np.testing.assert_allclose(clips.sum((1, 2, 3, 4)), g["clips80_sum"], rtol=1e-6)
    np.testing.assert_array_equal(clips[:, :, ::7, ::13, ::11], g["clips80_sample"])
    assert fuse_ref.n_clip_frames(80) == 64 and fuse_ref.n_clip_frames(48) == 64 and fuse_ref.n_clip_frames(47) == 32


def test_pipeline_real_model_T48(synthetic_sd):
    import clasfv_amd.synthetic as S
    g = golden("pipeline_model_T48.npz")
    v = fuse_ref.zeroone_normalizer(S.echo_video(48, seed=48))
    model = r2plus1d_ref.OracleModel(synthetic_sd)
    out = fuse_ref.segment_a_video_with_fusion(v, model, num_clips=1, to_numpy=lambda t: t.numpy())
    ref = np.unpackbits(g["labels"])[: out.size].reshape(out.shape)
    assert (out != ref).sum() <= 4


def test_normalizer_matches_reference():
    import clasfv_amd.synthetic as S
    g = golden("normalizer.npz")
    out = fuse_ref.zeroone_normalizer(S.echo_video(int(g["T"]), seed=int(g["seed"])))
    np.testing.assert_array_equal(out[:, ::3, ::5, ::7], g["out_sample"])
    np.testing.assert_allclose(out.astype(np.float64).sum((1, 2, 3)), g["out_sum"], rtol=1e-12)


def test_warp_oracle_matches_reference():
    g = golden("warp.npz")
    for name in ("zero", "plus5px", "minus5px_y", "random", "large"):
        img = g["img_r"] if name in ("random", "large") else g["img"]
        out = warp_ref.warp(torch.from_numpy(img), torch.from_numpy(g["flow_" + name])).numpy()
        np.testing.assert_allclose(out, g["out_" + name], atol=1e-6, err_msg=name)
    box = warp_ref.warp(torch.from_numpy(g["box"]), torch.zeros(1, 2, 112, 112)).numpy()
    np.testing.assert_allclose(box, g["box_zero"], atol=1e-6)
    # zero flow is not the identity (corner-aligned grid, align_corners=False sampling)
    assert np.abs(box - g["box"]).max() > 0.1


def test_simple_vote_properties():
    rng = np.random.default_rng(0)
    a = (rng.random((16, 16)) > 0.5).astype(np.uint8)
    # unanimous votes are returned unchanged; two identical + one different -> the majority
    np.testing.assert_array_equal(fuse_ref.simple_vote([a, a, a]), a)
    np.testing.assert_array_equal(fuse_ref.simple_vote([a, a, 1 - a]), a)
    np.testing.assert_array_equal(fuse_ref.majority_vote([a, 1 - a]), np.zeros_like(a))


def test_chunked_oracle_equals_as_written(synthetic_sd):
    """forward_chunked (used for 64x224x224 clips) is the same function as the as-written head."""
    rng = np.random.default_rng(12)
    x = rng.uniform(0, 1, (1, 3, 16, 48, 64)).astype(np.float32)
    s1, m1 = r2plus1d_ref.forward(synthetic_sd, x)
    s2, m2 = r2plus1d_ref.forward_chunked(synthetic_sd, x, frames_per_chunk=3)
    np.testing.assert_allclose(s2.numpy(), s1.numpy(), atol=2e-5)
    np.testing.assert_allclose(m2.numpy(), m1.numpy(), atol=1e-6)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_preprocess_oracle_matches_reference(case):
    """motion_segment.py:96-106 replayed on the reference (tests/golden/make_golden_preprocess.py):
    the numpy restatement of the trilinear resize is bit-exact, and with the normaliser too."""
    import clasfv_amd.synthetic as S
    g = golden("preprocess.npz")
    T, Hs, Ws, seed = (int(v) for v in g[f"case{case}"])
    r = fuse_ref.preprocess_frames(S.echo_video_uint8(T, Hs, Ws, seed=seed))
    np.testing.assert_array_equal(r[:, ::2, ::3, ::5], g[f"resized{case}_sample"])
    np.testing.assert_allclose(r.astype(np.float64).sum((1, 2, 3)), g[f"resized{case}_sum"], rtol=1e-12)
    n = fuse_ref.zeroone_normalizer(r)
    np.testing.assert_array_equal(n[:, ::2, ::3, ::5], g[f"norm{case}_sample"])
    np.testing.assert_allclose(n.astype(np.float64).sum((1, 2, 3)), g[f"norm{case}_sum"], rtol=1e-12)


@pytest.mark.parametrize("shape", [(3, 37, 53, 112, 112), (2, 600, 800, 112, 112), (2, 50, 60, 64, 96), (2, 1, 7, 5, 9)])
def test_preprocess_oracle_bitexact_vs_torch(shape):
    T, Hs, Ws, H, W = shape
    v = np.random.default_rng(sum(shape)).integers(0, 256, (T, Hs, Ws, 3), dtype=np.uint8)
    ref = F.interpolate(torch.from_numpy(v.transpose(3, 0, 1, 2).astype(np.float32))[None], size=(T, H, W),
                        mode="trilinear", align_corners=True)[0].numpy()
    np.testing.assert_array_equal(fuse_ref.preprocess_frames(v, H, W), ref)


def test_warp_backward_oracle_matches_reference():
    """torch-CPU grid_sample autograd (the oracle for clasfv_warp_backward) vs the reference golden."""
    from tests.golden.make_golden_losses import loss_inputs
    d, g = loss_inputs(), golden("losses.npz")
    img = torch.from_numpy(d["warp_img"]).requires_grad_()
    mot = torch.from_numpy(d["warp_motion"]).requires_grad_()
    out = warp_ref.warp(img, mot)
    out.backward(torch.from_numpy(d["warp_gout"]))
    np.testing.assert_array_equal(out.detach().numpy(), g["warp_out"])
    np.testing.assert_array_equal(mot.grad.numpy(), g["warp_grad_motion"])
    np.testing.assert_array_equal(img.grad.numpy(), g["warp_grad_img"])


def test_staple_restatement_known_answers():
    """STAPLE (parity unpinned: LabelFusion absent) -- properties of the published algorithm:
    unanimous raters are reproduced; a rater that disagrees with the others everywhere gets low
    sensitivity/specificity and is outvoted; the output is a binary uint8 image of the input shape."""
    from oracle import fuse_ref
    rng = np.random.default_rng(0)
    truth = rng.integers(0, 2, (40, 48)).astype(np.uint8)
    assert np.array_equal(fuse_ref.staple_vote([truth] * 3), truth)
    noisy = [truth.copy() for _ in range(4)]
    for v in noisy[:3]:  # three good raters with 3 % independent flips
        flip = rng.uniform(size=truth.shape) < 0.03
        v[flip] ^= 1
    noisy[3] = 1 - truth  # an adversarial rater
    out = fuse_ref.staple_vote(noisy)
    assert out.dtype == np.uint8 and out.shape == truth.shape
    assert (out != truth).mean() < 0.01
    assert np.array_equal(fuse_ref.staple_vote([np.zeros((5, 5), np.uint8)] * 2), np.zeros((5, 5), np.uint8))
    assert np.array_equal(fuse_ref.staple_vote([np.ones((5, 5), np.uint8)] * 2), np.ones((5, 5), np.uint8))


def test_northstar_fixture_is_physiological():
    """tests/golden/northstar_c1.npz (the CPU path on config[1] with the "echo" weights): the masks
    follow the synthetic LV, so the EFs are physiological and the ED/ES pairs are the video's cycles
    (period 50) -- the EF leg of the north_star bar is not degenerate."""
    g = golden("northstar_c1.npz")
    assert str(g["weights_recipe"]) == "echo"
    for m in ("majority", "simple", "staple"):
        efs = g[f"ef_{m}"]
        assert len(efs) == 4 and np.all((30 < efs) & (efs < 80)), efs
        assert g[f"pairs_{m}"].tolist() == [[0, 25], [50, 75], [100, 125], [150, 175]]


def test_deep_fixture_is_physiological_and_depends_on_layer2_4():
    """tests/golden/northstar_c1_deep.npz (round 6: the "deep" weights route the echo segmentation
    through layer2-4 at full gain): physiological EFs on the video's cycles, and the oracle's masks
    move when only the layer2-4 taps move (x 0.99: the size of accumulated bf16 rounding), which they
    never do with the echo weights -- so config[4]'s EF leg on this fixture sees bf16 arithmetic in
    every layer of the encoder."""
    import torch
    import clasfv_amd.synthetic as S
    import clasfv_amd.weights as W
    g = golden("northstar_c1_deep.npz")
    assert str(g["weights_recipe"]) == "deep"
    for m in ("majority", "simple", "staple"):
        efs = g[f"ef_{m}"]
        assert len(efs) == 4 and np.all((60 < efs) & (efs < 85)), efs
        assert np.all(np.abs(g[f"pairs_{m}"] - [[0, 25], [50, 75], [100, 125], [150, 175]]) <= 1)
    shp = tuple(g["fused_simple_shape"])
    fused = np.unpackbits(g["fused_simple"])[: int(np.prod(shp))].reshape(shp)
    assert fused[25::50].sum((1, 2)).min() > 200  # non-empty end-systolic masks
    v = fuse_ref.zeroone_normalizer(S.echo_video(32, seed=0))
    x = torch.from_numpy(np.ascontiguousarray(v[None]))
    flips = {}
    for rec in ("echo", "deep"):
        sd = W.recipe_state_dict(rec)
        with torch.no_grad():
            taps = r2plus1d_ref.backbone(sd, x)
            s0, _ = r2plus1d_ref.head(sd, taps)
            s1, _ = r2plus1d_ref.head(sd, taps[:2] + [t * 0.99 for t in taps[2:]])
        flips[rec] = int(((s0[0, 1] > s0[0, 0]) != (s1[0, 1] > s1[0, 0])).sum())
    assert flips["echo"] == 0 and flips["deep"] > 0, flips

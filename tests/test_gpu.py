"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the reference goldens.

Tolerances: the forward is fp32 with a different summation order than cuDNN/mkldnn (Winograd and
implicit GEMMs, folded BatchNorm, decoder commuted to project-then-interpolate), so raw logits are
compared with an absolute tolerance and the derived masks with the north_star bar Dice delta <= 1e-3.
The logit tolerance sits a few times above the largest error measured on the box over every shape
tested here (profiles/r04pe_parity_errors.txt, on the round-4 kernels: seg <= 2.6e-5 at config[3]
64x224x224, <= 1.8e-5 at 32x112x112; motion <= 5.9e-7), so a kernel bug that moves one channel block
by 1e-4 fails.
Plumbing kernels (clip building, resample, argmax, voting, normaliser) are compared bit for bit.
"""
import os

import numpy as np
import pytest
import torch

from oracle import fuse_ref, r2plus1d_ref, warp_ref
from tests.conftest import golden, unpack_labels
from tests.golden.fake_model import fake_model

pytestmark = pytest.mark.gpu

DICE_TOL = 1e-3
SEG_ATOL = 1e-4   # fp32 logits (measured max 2.6e-5, r04pe)
MOT_ATOL = 2e-6   # fp32 tanh motion (measured max 5.9e-7, r04pe)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dice_delta(a, b):
    from clasfv_amd.echo import categorical_dice
    return 1.0 - categorical_dice(np.asarray(a), np.asarray(b), 1)


@pytest.fixture(scope="module")
def model():
    from clasfv_amd.model import R2plus1D_18_MotionNet
    return R2plus1D_18_MotionNet(pretrained=False)


@pytest.fixture(scope="module")
def echo_model():
    """The bench's weights: the "echo" recipe, whose masks follow the synthetic LV."""
    from clasfv_amd.model import R2plus1D_18_MotionNet
    return R2plus1D_18_MotionNet(pretrained=False, weights="echo")


@pytest.fixture(scope="module")
def deep_model():
    """The "deep" recipe: the echo segmentation routed through layer2-4 at full gain."""
    from clasfv_amd.model import R2plus1D_18_MotionNet
    return R2plus1D_18_MotionNet(pretrained=False, weights="deep")


def test_native_library_is_loaded(model):
    import clasfv_amd._lib as L
    with open("/proc/self/maps") as f:
        assert L.lib_path() in f.read()


def test_forward_small_vs_reference_golden(model):
    g = golden("model_forward.npz")
    seg, mot = model(torch.from_numpy(g["x_small"]))
    seg, mot = seg.cpu().numpy(), mot.cpu().numpy()
    np.testing.assert_allclose(seg, g["seg_small"], rtol=0, atol=SEG_ATOL)
    np.testing.assert_allclose(mot, g["mot_small"], rtol=0, atol=MOT_ATOL)
    ref_lab = g["seg_small"][:, 1] > g["seg_small"][:, 0]
    assert dice_delta(seg[:, 1] > seg[:, 0], ref_lab) <= DICE_TOL


def test_forward_full_clip_vs_reference_golden(model):
    import clasfv_amd.synthetic as S
    g = golden("model_forward.npz")
    v = fuse_ref.zeroone_normalizer(S.echo_video(int(g["big_T"]), seed=int(g["big_video_seed"])))
    s = int(g["big_start"])
    seg, mot = model(torch.from_numpy(np.ascontiguousarray(v[None, :, s:s + 32])))
    seg, mot = seg.cpu().numpy(), mot.cpu().numpy()
    lab = (seg[0, 1] > seg[0, 0]).ravel()
    ref = np.unpackbits(g["big_label_bits"])[: lab.size].astype(bool)
    assert dice_delta(lab, ref) <= DICE_TOL
    assert (lab != ref).mean() <= 1e-4
    idx = g["big_idx"]
    np.testing.assert_allclose(seg[0, 0].ravel()[idx], g["big_seg0"], rtol=0, atol=SEG_ATOL)
    np.testing.assert_allclose(seg[0, 1].ravel()[idx], g["big_seg1"], rtol=0, atol=SEG_ATOL)
    np.testing.assert_allclose(mot[0].reshape(4, -1)[:, idx], g["big_mot"], rtol=0, atol=MOT_ATOL)
    np.testing.assert_allclose(seg.astype(np.float64).sum((0, 2, 3, 4)), g["big_seg_sum"], rtol=1e-6)


@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 48), (1, 3, 8, 16, 32), (3, 3, 24, 32, 32)])
def test_forward_vs_oracle_other_shapes(model, synthetic_sd, shape):
    rng = np.random.default_rng(sum(shape))
    x = rng.uniform(0, 1, shape).astype(np.float32)
    seg, mot = model(torch.from_numpy(x))
    rs, rm = r2plus1d_ref.forward(synthetic_sd, x)
    np.testing.assert_allclose(seg.cpu().numpy(), rs.numpy(), rtol=0, atol=SEG_ATOL)
    np.testing.assert_allclose(mot.cpu().numpy(), rm.numpy(), rtol=0, atol=MOT_ATOL)


def test_forward_batch_is_per_clip_exact(model):
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.uniform(0, 1, (4, 3, 32, 112, 112)).astype(np.float32)).cuda()
    seg, mot = model(x)
    for i in (0, 3):
        s1, m1 = model(x[i:i + 1])
        assert torch.equal(s1[0], seg[i]) and torch.equal(m1[0], mot[i])


@pytest.mark.parametrize("shape", [(3, 3, 32, 80, 80), (3, 3, 16, 48, 80)])
def test_forward_batch_is_per_clip_exact_ragged_tiles(model, shape):
    """Kernel choice and tile grouping depend on the per-clip shape only: at 80x80 clips layer2's
    20x20 maps have 5 tile columns, where a group shape chosen from the batch's tile rows used to
    switch F(4x4) on at N=3 and off at N=1 (different rounding per clip)."""
    rng = np.random.default_rng(sum(shape))
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    seg, mot = model(x)
    for i in range(shape[0]):
        s1, m1 = model(x[i:i + 1])
        assert torch.equal(s1[0], seg[i]) and torch.equal(m1[0], mot[i]), i


def test_forward_batch_is_per_clip_exact_winot_nt_switch(model):
    """conv_winot5's channel block (csrc/winograd_t.hip winot5_nt) is picked from the launch's last-wave
    fill, so it depends on the batch: at 32x64x64 clips layer3's temporal convs (T = 8, the TS = 2
    form, 8x8 maps, 256 channels) run NT = 2 at three waves per SIMD for one clip (8 blocks) and NT = 4
    for 100 clips (400 blocks: fill 0.78 against 0.49). Both forms issue the same products in the same
    order, so a clip's logits must not depend on the batch (the rule switches exactly at
    the TS = 2 instantiation)."""
    rng = np.random.default_rng(83)
    x = torch.from_numpy(rng.uniform(0, 1, (100, 3, 32, 64, 64)).astype(np.float32)).cuda()
    seg, mot = model(x)
    for i in (0, 57, 99):
        s1, m1 = model(x[i:i + 1])
        assert torch.equal(s1[0], seg[i]) and torch.equal(m1[0], mot[i]), i


def test_forwards_on_concurrent_streams_equal_serial(model):
    """One engine handle keeps a workspace per launch stream (csrc/engine.hip Ctx), so forwards issued
    on different streams without a host sync in between -- two or more videos in flight, bench.py
    --inflight -- run concurrently and each equals the serial result bit for bit; past four streams
    the least recently used workspace is taken over after a device sync."""
    rng = np.random.default_rng(91)
    xs = [torch.from_numpy(rng.uniform(0, 1, (2, 3, 32, 64, 64)).astype(np.float32)).cuda() for _ in range(6)]
    ref = [model(x) for x in xs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(6)]
    for rnd in range(2):  # round 2 reuses round 1's streams (their contexts; six streams > four contexts)
        got = []
        for x, s in zip(xs, streams):
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                got.append(model(x))
        torch.cuda.synchronize()
        for i, ((s0, m0), (s1, m1)) in enumerate(zip(ref, got)):
            assert torch.equal(s0, s1) and torch.equal(m0, m1), (rnd, i)


def test_segment_videos_two_streams_in_flight(echo_model):
    """bench.py --inflight 2: consecutive fusion steps of one device video on two streams give the
    serial step's masks."""
    from clasfv_amd import dist as D
    import clasfv_amd.synthetic as S
    v = torch.as_tensor(S.echo_video(120, seed=3)).cuda()

    def step():
        return D.segment_videos_sharded([v], echo_model, num_clips=5, step=1, fuse_method="simple")[0]

    ref = step()
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k in range(4):
        s = streams[k % 2]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            outs.append(step())
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)


@pytest.mark.parametrize("shape", [(2, 3, 32, 112, 112), (3, 3, 24, 80, 112)])
def test_bf16_forward_batch_is_per_clip_exact(shape):
    """config[4] engines: every kernel choice is a per-clip shape rule too (conv_patch32_bf16 is taken
    from the per-clip block count, not the batch's), so one clip alone and the same clip inside a
    batch get the same products in the same order -- bit-identical, with the 32x32x16 kernel running
    at N = 1 as well."""
    from clasfv_amd.model import R2plus1D_18_MotionNet
    rng = np.random.default_rng(sum(shape) + 1)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    m16 = R2plus1D_18_MotionNet(pretrained=False, dtype="bf16")
    seg, mot = m16(x)
    m16.engine.set_kernel_timing(True)
    s1, m1 = m16(x[:1])
    kt = m16.engine.kernel_timing(cap=32)
    m16.engine.set_kernel_timing(False)
    assert "conv_patch32_bf16" in kt
    assert torch.equal(s1[0], seg[0]) and torch.equal(m1[0], mot[0])
    for i in range(1, shape[0]):
        si, mi = m16(x[i:i + 1])
        assert torch.equal(si[0], seg[i]) and torch.equal(mi[0], mot[i]), i


def test_forward_rejects_bad_shapes(model):
    with pytest.raises(RuntimeError, match="shape"):
        model(torch.zeros(1, 3, 12, 112, 112))
    with pytest.raises(RuntimeError, match="shape"):
        model(torch.zeros(1, 3, 32, 100, 112))


def test_load_state_dict_module_prefix(model, synthetic_sd):
    import clasfv_amd.weights as W
    sd2 = W.synthetic_state_dict(99)
    model.load_state_dict({"module." + k: torch.from_numpy(np.asarray(v)) for k, v in sd2.items()})
    x = torch.rand(1, 3, 8, 32, 32)
    s2, _ = model(x)
    r2, _ = r2plus1d_ref.forward(sd2, x)
    np.testing.assert_allclose(s2.cpu().numpy(), r2.numpy(), rtol=0, atol=SEG_ATOL)
    model.load_state_dict(synthetic_sd)
    assert sum(p.numel() for p in model.parameters() if p.requires_grad) == 31_575_731


# ---- plumbing kernels ---------------------------------------------------------------------------

def _norm_video(T, seed):
    import clasfv_amd.synthetic as S
    return fuse_ref.zeroone_normalizer(S.echo_video(T, seed=seed))


@pytest.mark.parametrize("T", [33, 48, 70, 80, 200, 64])
def test_build_clips_bitexact(T):
    from clasfv_amd import fuse_utils as FU
    v = _norm_video(T, T)
    for interp in (True, False):
        if not interp and T % 32 and FU.n_clips(T) * 32 > T:
            continue
        got = FU.divide_to_consecutive_clips(v, interpolate_last=interp).cpu().numpy()
        ref = fuse_ref.divide_to_consecutive_clips(v, interpolate_last=interp)
        np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("T", [33, 48, 70, 80, 200])
def test_pipeline_fusion_off_vs_reference_golden(T):
    from clasfv_amd import fuse_utils as FU
    g = golden("plumbing.npz")
    out = FU.segment_a_video_with_fusion(_norm_video(T, T), fake_model, num_clips=1)
    ref = unpack_labels(g, f"off_T{T}")
    assert out.dtype == np.int64 and out.shape == ref.shape
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("T,f,step", [(70, 5, 1), (200, 5, 1), (80, 3, 2), (48, 10, 1), (40, 5, 3)])
def test_pipeline_majority_vs_reference_golden(T, f, step):
    from clasfv_amd import fuse_utils as FU
    g = golden("plumbing.npz")
    out = FU.segment_a_video_with_fusion(_norm_video(T, 100 + T), fake_model, step=step, num_clips=f,
                                         fuse_method="majority")
    np.testing.assert_array_equal(out, unpack_labels(g, f"on_T{T}_f{f}_s{step}"))


@pytest.mark.parametrize("T,f,step", [(70, 5, 1), (80, 3, 2), (48, 10, 1)])
def test_pipeline_simple_vs_oracle(T, f, step):
    """SIMPLE fusion: GPU kernel vs the oracle's restatement (parity with LabelFusion unpinned)."""
    from clasfv_amd import fuse_utils as FU

    def np_model(x):
        s, m = fake_model(torch.from_numpy(np.ascontiguousarray(x)))
        return s.numpy(), m.numpy()
    v = _norm_video(T, 100 + T)
    out = FU.segment_a_video_with_fusion(v, fake_model, step=step, num_clips=f, fuse_method="simple")
    ref = fuse_ref.segment_a_video_with_fusion(v, np_model, step=step, num_clips=f, fuse_method="simple")
    np.testing.assert_array_equal(out, ref)


def _noisy_passes(K, T, step, H=40, W=48, seed=0):
    """K pass label videos (pass k has T - k*step frames): a pulsing ellipse plus per-pass blotches, so
    SIMPLE sees disagreeing candidates and iterates."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    passes = []
    for k in range(K):
        n = T - k * step
        v = np.zeros((n, H, W), np.uint8)
        for f in range(n):
            t = f + k * step
            a, b = 8 + 4 * np.sin(t / 5.0), 10 + 3 * np.cos(t / 7.0)
            m = ((yy - H / 2) / a) ** 2 + ((xx - W / 2) / b) ** 2 <= 1
            for _ in range(int(rng.integers(0, 4))):
                cy, cx, r = rng.integers(0, H), rng.integers(0, W), rng.integers(2, 9)
                m ^= (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
            v[f] = m
        passes.append(v)
    return passes


@pytest.mark.parametrize("K,T,step", [(2, 20, 1), (5, 40, 1), (10, 60, 1), (16, 70, 1), (6, 50, 3), (17, 60, 1)])
def test_fuse_simple_kernels_vs_oracle(K, T, step):
    """SIMPLE fusion: the packed-mask kernel (K <= 16) and the generic kernel both equal the oracle's
    restatement frame by frame (parity with LabelFusion itself unpinned)."""
    from clasfv_amd import fuse_utils as FU
    passes = _noisy_passes(K, T, step, seed=K * 100 + T)
    labels = np.zeros((K, T) + passes[0].shape[1:], np.uint8)
    for k, p in enumerate(passes):
        labels[k, :p.shape[0]] = p
    lab = torch.from_numpy(labels).cuda()
    ref = fuse_ref.fuse_frames(passes, T, step, "simple")
    fast = FU.fuse_votes(lab, step, "simple").cpu().numpy()
    generic = FU.fuse_votes(lab, step, "simple", force_generic=True).cpu().numpy()
    np.testing.assert_array_equal(generic, ref)
    np.testing.assert_array_equal(fast, ref)


def test_pipeline_quirks():
    from clasfv_amd import fuse_utils as FU
    with pytest.raises(IndexError):
        FU.segment_a_video_with_fusion(_norm_video(32, 32), fake_model, num_clips=1)


def test_pipeline_real_model_T48_vs_reference_golden(model):
    from clasfv_amd import fuse_utils as FU
    g = golden("pipeline_model_T48.npz")
    out = FU.segment_a_video_with_fusion(_norm_video(48, 48), model, num_clips=1)
    ref = np.unpackbits(g["labels"])[: out.size].reshape(out.shape)
    assert dice_delta(out, ref) <= DICE_TOL


def test_normalizer_bitexact_vs_reference_golden():
    import clasfv_amd.synthetic as S
    from clasfv_amd.preprocess import zeroone_normalizer
    g = golden("normalizer.npz")
    out = zeroone_normalizer(S.echo_video(int(g["T"]), seed=int(g["seed"])))
    np.testing.assert_array_equal(out[:, ::3, ::5, ::7], g["out_sample"])
    np.testing.assert_allclose(out.astype(np.float64).sum((1, 2, 3)), g["out_sum"], rtol=1e-12)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_preprocess_video_bitexact_vs_reference_golden(case):
    """clasfv_preprocess_video + normaliser == the reference CLI's resize + zeroone_normalizer."""
    import clasfv_amd.synthetic as S
    from clasfv_amd.preprocess import preprocess_video
    g = golden("preprocess.npz")
    T, Hs, Ws, seed = (int(v) for v in g[f"case{case}"])
    frames = S.echo_video_uint8(T, Hs, Ws, seed=seed)
    r = preprocess_video(frames, normalize=False).cpu().numpy()
    np.testing.assert_array_equal(r[:, ::2, ::3, ::5], g[f"resized{case}_sample"])
    np.testing.assert_array_equal(r, fuse_ref.preprocess_frames(frames))
    n = preprocess_video(torch.from_numpy(frames).cuda()).cpu().numpy()
    np.testing.assert_array_equal(n[:, ::2, ::3, ::5], g[f"norm{case}_sample"])
    np.testing.assert_allclose(n.astype(np.float64).sum((1, 2, 3)), g[f"norm{case}_sum"], rtol=1e-12)


@pytest.mark.parametrize("shape", [(4, 600, 800, 112, 112), (3, 50, 60, 64, 96), (2, 1, 7, 5, 9), (200, 112, 112, 112, 112)])
def test_preprocess_video_bitexact_vs_oracle(shape):
    from clasfv_amd.preprocess import preprocess_video
    T, Hs, Ws, H, W = shape
    v = np.random.default_rng(sum(shape)).integers(0, 256, (T, Hs, Ws, 3), dtype=np.uint8)
    out = preprocess_video(v, H, W, normalize=False).cpu().numpy()
    np.testing.assert_array_equal(out, fuse_ref.preprocess_frames(v, H, W))


def test_warp_vs_reference_golden():
    from clasfv_amd.warp import warp
    g = golden("warp.npz")
    for name in ("zero", "plus5px", "minus5px_y", "random", "large"):
        img = g["img_r"] if name in ("random", "large") else g["img"]
        out = warp(torch.from_numpy(img).cuda(), torch.from_numpy(g["flow_" + name]).cuda()).cpu().numpy()
        np.testing.assert_array_equal(out, g["out_" + name], err_msg=name)  # bit-exact
    box = warp(torch.from_numpy(g["box"]).cuda(), torch.zeros(1, 2, 112, 112).cuda()).cpu().numpy()
    np.testing.assert_array_equal(box, g["box_zero"])


def test_warp_backward_vs_reference_golden():
    """clasfv_warp_backward: motion gradient bit-exact vs the reference's CPU grid_sample backward,
    image gradient to float rounding (atomic scatter order)."""
    from clasfv_amd.warp import warp
    from tests.golden.make_golden_losses import loss_inputs
    d, g = loss_inputs(), golden("losses.npz")
    img = torch.from_numpy(d["warp_img"]).cuda().requires_grad_()
    mot = torch.from_numpy(d["warp_motion"]).cuda().requires_grad_()
    out = warp(img, mot)
    out.backward(torch.from_numpy(d["warp_gout"]).cuda())
    np.testing.assert_array_equal(out.detach().cpu().numpy(), g["warp_out"])
    np.testing.assert_array_equal(mot.grad.cpu().numpy(), g["warp_grad_motion"])
    np.testing.assert_allclose(img.grad.cpu().numpy(), g["warp_grad_img"], rtol=1e-5, atol=1e-6)


def test_warp_backward_strided_motion_vs_oracle():
    from clasfv_amd.warp import warp
    rng = np.random.default_rng(5)
    img = rng.uniform(0, 1, (2, 2, 24, 36)).astype(np.float32)
    motion = np.tanh(rng.normal(0, 0.4, (2, 4, 3, 24, 36))).astype(np.float32)  # large: exercises clipping
    gout = rng.normal(0, 1, (2, 2, 24, 36)).astype(np.float32)
    mg = torch.from_numpy(motion).cuda().requires_grad_()
    ig = torch.from_numpy(img).cuda().requires_grad_()
    warp(ig, mg[:, 2:, 1]).backward(torch.from_numpy(gout).cuda())
    mc = torch.from_numpy(motion).requires_grad_()
    ic = torch.from_numpy(img).requires_grad_()
    warp_ref.warp(ic, mc[:, 2:, 1]).backward(torch.from_numpy(gout))
    np.testing.assert_array_equal(mg.grad.cpu().numpy(), mc.grad.numpy())
    np.testing.assert_allclose(ig.grad.cpu().numpy(), ic.grad.numpy(), rtol=1e-5, atol=1e-6)


def test_training_losses_vs_reference_golden():
    """deformation_motion_loss (OTA) and motion_seg_loss (SGS/OTS) through the HIP warp: loss values
    and autograd gradients vs the reference's CPU run (fp32; gradients summed over many warps, so
    compared to float rounding)."""
    import torch.nn.functional as F
    from clasfv_amd import losses as L
    from tests.golden.make_golden_losses import loss_inputs
    d, g = loss_inputs(), golden("losses.npz")
    video = torch.from_numpy(d["video"]).cuda().requires_grad_()
    motion = torch.from_numpy(d["motion"]).cuda().requires_grad_()
    loss = L.deformation_motion_loss(video, motion)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g["ota_loss"], rtol=1e-5)  # GPU vs CPU reduction order
    np.testing.assert_allclose(video.grad.cpu().numpy(), g["ota_grad_video"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(motion.grad.cpu().numpy(), g["ota_grad_motion"], rtol=1e-4, atol=1e-7)

    motion = torch.from_numpy(d["motion"]).cuda().requires_grad_()
    logits = torch.from_numpy(d["logits"]).cuda().requires_grad_()
    flow, ots = L.motion_seg_loss(d["ed"], d["es"], d["ed_index"], d["es_index"], motion, F.softmax(logits, dim=1),
                                  start=0, end=d["video"].shape[2])
    (flow + ots).backward()
    np.testing.assert_allclose(flow.item(), g["sgs_flow_loss"], rtol=1e-5)
    np.testing.assert_allclose(ots.item(), g["sgs_ots_loss"], rtol=1e-5)
    np.testing.assert_allclose(motion.grad.cpu().numpy(), g["sgs_grad_motion"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(logits.grad.cpu().numpy(), g["sgs_grad_logits"], rtol=1e-4, atol=1e-7)


def test_warp_strided_motion_slice_vs_oracle():
    from clasfv_amd.warp import warp
    rng = np.random.default_rng(3)
    img = torch.from_numpy(rng.uniform(0, 1, (2, 3, 40, 56)).astype(np.float32))
    motion = torch.from_numpy(np.tanh(rng.normal(0, 0.2, (2, 4, 5, 40, 56))).astype(np.float32))
    out = warp(img.cuda(), motion.cuda()[:, 2:, 3]).cpu()
    ref = warp_ref.warp(img, motion[:, 2:, 3])
    np.testing.assert_array_equal(out.numpy(), ref.numpy())


def test_cli_end_to_end(tmp_path):
    """motion_segment.py drop-in: pickles with the reference names, EF text, int64 masks."""
    import pickle
    import subprocess
    import sys
    import clasfv_amd.synthetic as S
    vid = tmp_path / "echo_case.npy"
    np.save(vid, S.echo_video_uint8(100, seed=4))
    r = subprocess.run([sys.executable, "motion_segment.py", "-p", str(vid), "--synthetic-weights", "1234", "-f", "2",
                        "-c", "binary,binary_video", "-o", str(tmp_path), "-v"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "R2+1D MotionNet has 31575731 parameters." in r.stdout
    assert "systoles" in r.stdout
    whole = pickle.load(open(tmp_path / "echo_case_whole_video_segmentation.pkl", "rb"))
    assert whole.shape == (100, 112, 112) and whole.dtype == np.int64


def test_forward_config3_64x224_vs_chunked_oracle(model, synthetic_sd):
    """BASELINE config[3]: one 64-frame 224x224 clip (the as-written concat would be 13 GB; the
    oracle evaluates the same head frame-chunk by frame-chunk)."""
    import clasfv_amd.synthetic as S
    v = fuse_ref.zeroone_normalizer(S.echo_video(64, H=224, W=224, seed=21))
    x = np.ascontiguousarray(v[None])
    seg, mot = model(torch.from_numpy(x))
    seg, mot = seg.cpu().numpy(), mot.cpu().numpy()
    torch.set_num_threads(16)
    rs, rm = r2plus1d_ref.forward_chunked(synthetic_sd, x, frames_per_chunk=8)
    rs, rm = rs.numpy(), rm.numpy()
    np.testing.assert_allclose(seg, rs, rtol=0, atol=SEG_ATOL)
    np.testing.assert_allclose(mot, rm, rtol=0, atol=MOT_ATOL)
    assert dice_delta(seg[:, 1] > seg[:, 0], rs[:, 1] > rs[:, 0]) <= DICE_TOL


def test_sharded_pipeline_world1_equals_per_video(model):
    from clasfv_amd import dist as D
    from clasfv_amd import fuse_utils as FU
    vids = [torch.from_numpy(_norm_video(T, 300 + T)).cuda() for T in (70, 96, 45)]
    got = D.segment_videos_sharded(vids, model, num_clips=3, step=1, fuse_method="simple")
    for i, v in enumerate(vids):
        ref = FU.segment_a_video_with_fusion_device(v, model, num_clips=3, step=1, fuse_method="simple")
        assert torch.equal(got[i], ref)


def _dist_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from clasfv_amd import dist as D
        from clasfv_amd.model import R2plus1D_18_MotionNet
        m = R2plus1D_18_MotionNet(pretrained=False)
        vids = [torch.from_numpy(_norm_video(T, 300 + T)).cuda() for T in (70, 96, 45)]
        out = D.segment_videos_sharded(vids, m, num_clips=3, step=1, fuse_method="simple", rank=rank, world=world)
        q.put((rank, {k: v.cpu().numpy() for k, v in out.items()}))
    finally:
        dist.destroy_process_group()


def test_sharded_pipeline_two_ranks_equals_one(model):
    """Clip-wise sharding over 2 ranks (gloo exchange, both ranks on the one GPU of the test box):
    every rank's fused videos are bit-identical to the 1-process result."""
    import socket
    import torch.multiprocessing as mp
    from clasfv_amd import fuse_utils as FU
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, out = q.get(timeout=300)
        res.update(out)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert sorted(res) == [0, 1, 2]
    for i, T in enumerate((70, 96, 45)):
        ref = FU.segment_a_video_with_fusion_device(torch.from_numpy(_norm_video(T, 300 + T)).cuda(), model,
                                                    num_clips=3, step=1, fuse_method="simple").cpu().numpy()
        np.testing.assert_array_equal(res[i], ref)


def test_wrappers_accept_non_contiguous_inputs(model):
    """Every ABI wrapper densifies its tensors: strided (e.g. transposed numpy) videos give the same
    clips and masks as contiguous ones."""
    from clasfv_amd import fuse_utils as FU
    v = _norm_video(70, 5)
    strided = torch.from_numpy(np.ascontiguousarray(v.transpose(1, 2, 3, 0))).permute(3, 0, 1, 2).cuda()
    assert not strided.is_contiguous()
    table, _ = FU.clip_table(70, 3, 1)
    a = FU.build_clips(strided, table)
    b = FU.build_clips(torch.from_numpy(v).cuda(), table)
    assert torch.equal(a, b)
    assert torch.equal(FU.segment_a_video_with_fusion_device(strided, fake_model, num_clips=3),
                       FU.segment_a_video_with_fusion_device(v, fake_model, num_clips=3))


def test_forward_bf16_vs_reference_golden_config4_tolerance(model):
    """BASELINE config[4]: bf16 activations/weights with fp32 accumulation, Dice tolerance 1e-2."""
    import clasfv_amd.synthetic as S
    from clasfv_amd.model import R2plus1D_18_MotionNet
    g = golden("model_forward.npz")
    v = fuse_ref.zeroone_normalizer(S.echo_video(int(g["big_T"]), seed=int(g["big_video_seed"])))
    s = int(g["big_start"])
    m16 = R2plus1D_18_MotionNet(pretrained=False, dtype="bf16")
    seg, mot = m16(torch.from_numpy(np.ascontiguousarray(v[None, :, s:s + 32])))
    seg = seg.cpu().numpy()
    lab = (seg[0, 1] > seg[0, 0]).ravel()
    ref = np.unpackbits(g["big_label_bits"])[: lab.size].astype(bool)
    assert dice_delta(lab, ref) <= 1e-2
    idx = g["big_idx"]
    err = np.abs(seg[0, 1].ravel()[idx] - g["big_seg1"])
    assert np.median(err) < 0.05 and err.max() < 0.5
    # switching back to fp32 restores the exact path
    m16.set_compute_dtype("fp32")
    s32, _ = m16(torch.from_numpy(np.ascontiguousarray(v[None, :, s:s + 32])))
    s_ref, _ = model(torch.from_numpy(np.ascontiguousarray(v[None, :, s:s + 32])))
    assert torch.equal(s32, s_ref)


@pytest.mark.parametrize("shape", [(1, 3, 32, 112, 112), (2, 3, 16, 64, 48)])
def test_bf16_patch_conv_matches_direct_conv(model, shape):
    """bf16 stride-1 1x3x3 and 3x1x1 convs: the patch-staged kernel (conv_patch.hip, chunk-major K
    order) against the direct LDS-DMA kernel (variant no_patch_bf16, tap-major K order). The two sum the
    same bf16 products in different fp32 orders, so bf16 activations may round differently: the
    patch path's error against the fp32 forward must be no larger than the direct path's, and on the
    echo-style clip both stay within the config[4] bar (Dice delta <= 1e-2). The (2,3,16,64,48) case
    has ragged maps (layer3 16x12, layer4 8x6: masked tiles)."""
    import clasfv_amd.synthetic as S
    from clasfv_amd.model import R2plus1D_18_MotionNet
    if shape[2:] == (32, 112, 112):
        v = fuse_ref.zeroone_normalizer(S.echo_video(64, seed=3))
        x = torch.from_numpy(np.ascontiguousarray(v[None, :, 10:42]))
    else:
        x = torch.from_numpy(np.random.default_rng(23).uniform(0, 1, shape).astype(np.float32))
    s32, _ = model(x)
    m16 = R2plus1D_18_MotionNet(pretrained=False, dtype="bf16")
    s_p, m_p = m16(x)
    m16.set_kernel_variants("no_patch_bf16")
    s_d, m_d = m16(x)
    m16.set_kernel_variants()
    assert torch.isfinite(s_p).all() and torch.isfinite(m_p).all()
    e_p, e_d = (s_p - s32).abs(), (s_d - s32).abs()
    assert float(e_p.median()) <= 1.5 * float(e_d.median()) + 1e-3, (float(e_p.median()), float(e_d.median()))
    assert float(e_p.max()) <= 2 * float(e_d.max()) + 1e-2, (float(e_p.max()), float(e_d.max()))
    lab32 = (s32[:, 1] > s32[:, 0]).cpu().numpy().ravel()
    lab_p = (s_p[:, 1] > s_p[:, 0]).cpu().numpy().ravel()
    assert (lab_p == lab32).mean() >= 0.99
    if shape[2:] == (32, 112, 112):
        assert lab32.sum() > 1000 and dice_delta(lab_p, lab32) <= 1e-2


@pytest.mark.parametrize("shape", [(1, 3, 32, 112, 112), (2, 3, 16, 64, 48), (3, 3, 8, 32, 80), (2, 3, 24, 48, 48)])
def test_bf16_twalk_matches_patch(model, shape):
    """Round 6: the bf16 engines' 64-channel temporal convs (stem and layer1, 5 launches) on the
    frame-walking conv_twalk_bf16 (csrc/twalk.hip) against conv_patch_bf16 (variant no_twalk). Both sum
    the same bf16 products in different fp32 orders (input frame / channel / tap vs chunk / tap), so bf16
    activations may round differently: the walking path's error against the fp32 forward must be no
    larger than the patch path's, and so must its mask disagreement. Shapes: 16-frame segments
    (T = 32, 16), 8-frame segments (T = 8, 24), ragged 32-pixel columns (64x48 -> 32x24 = 768 pixels,
    32x80 -> 16x40, 48x48 -> 24x24 = 576)."""
    import clasfv_amd.synthetic as S
    from clasfv_amd.model import R2plus1D_18_MotionNet
    if shape[2:] == (32, 112, 112):
        v = fuse_ref.zeroone_normalizer(S.echo_video(64, seed=3))
        x = torch.from_numpy(np.ascontiguousarray(v[None, :, 10:42]))
    else:
        x = torch.from_numpy(np.random.default_rng(31).uniform(0, 1, shape).astype(np.float32))
    s32, _ = model(x)
    m16 = R2plus1D_18_MotionNet(pretrained=False, dtype="bf16")
    m16.engine.set_kernel_timing(True)
    s_w, m_w = m16(x)
    kt = m16.engine.kernel_timing(cap=32)
    m16.engine.set_kernel_timing(False)
    assert kt["conv_twalk_bf16"]["launches"] == 5, kt.keys()  # stem temporal + layer1's four
    m16.set_kernel_variants("no_twalk")
    s_p, _ = m16(x)
    m16.set_kernel_variants()
    assert torch.isfinite(s_w).all() and torch.isfinite(m_w).all()
    e_w, e_p = (s_w - s32).abs(), (s_p - s32).abs()
    assert float(e_w.median()) <= 1.5 * float(e_p.median()) + 1e-3, (float(e_w.median()), float(e_p.median()))
    assert float(e_w.max()) <= 2 * float(e_p.max()) + 1e-2, (float(e_w.max()), float(e_p.max()))
    lab32 = (s32[:, 1] > s32[:, 0]).cpu().numpy()
    d_w = dice_delta((s_w[:, 1] > s_w[:, 0]).cpu().numpy(), lab32)
    d_p = dice_delta((s_p[:, 1] > s_p[:, 0]).cpu().numpy(), lab32)
    assert d_w <= max(1e-2, 1.5 * d_p), (d_w, d_p)


@pytest.mark.parametrize("variant", ["no_stem_bf16", "no_decoder_bf16"])
def test_bf16_stem_and_decoder_vs_fp32_mfma_forms(model, variant):
    """config[4]: the bf16 stem (conv.hip conv_stem_bf16: clip split into bf16 hi + lo, bf16 MFMAs) and
    the bf16 decoder (decoder.hip, comb_2 on split-bf16 MFMAs) against their fp32-MFMA forms (kernel
    variant). The default bf16 forward must stay within the config[4] bar of the fp32 forward, with an
    error no larger than a small margin over the fp32-MFMA form's."""
    import clasfv_amd.synthetic as S
    from clasfv_amd.model import R2plus1D_18_MotionNet
    v = fuse_ref.zeroone_normalizer(S.echo_video(64, seed=3))
    x = torch.from_numpy(np.ascontiguousarray(v[None, :, 10:42]))
    m16 = R2plus1D_18_MotionNet(pretrained=False, dtype="bf16")
    s_d, mo_d = m16(x)
    m16.set_kernel_variants(variant)
    s_f, mo_f = m16(x)
    m16.set_kernel_variants()
    assert not torch.equal(s_d, s_f)  # the variant really ran another kernel
    s32, m32 = model(x)
    e_d = torch.cat([(s_d - s32).abs().ravel(), (mo_d - m32).abs().ravel()]).cpu().numpy()
    e_f = torch.cat([(s_f - s32).abs().ravel(), (mo_f - m32).abs().ravel()]).cpu().numpy()
    assert torch.isfinite(s_d).all() and torch.isfinite(mo_d).all()
    assert np.median(e_d) <= 1.5 * np.median(e_f) + 1e-3, (np.median(e_d), np.median(e_f))
    lab = (s_d[:, 1] > s_d[:, 0]).cpu().numpy().ravel()
    lab32 = (s32[:, 1] > s32[:, 0]).cpu().numpy().ravel()
    assert lab32.sum() > 1000 and dice_delta(lab, lab32) <= 1e-2


@pytest.mark.parametrize("shape", [(1, 3, 32, 112, 112), (2, 3, 16, 64, 48)])
def test_winograd_path_matches_direct_conv(model, shape):
    """The fused Winograd kernels (default for stride-1 fp32 convs) against the direct implicit-GEMM
    kernel (variant no_winograd), and both against the CPU oracle."""
    from clasfv_amd.model import R2plus1D_18_MotionNet
    rng = np.random.default_rng(17)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32))
    s_w, m_w = model(x)
    direct = R2plus1D_18_MotionNet(pretrained=False)
    direct.set_kernel_variants("no_winograd")
    s_d, m_d = direct(x)
    assert not torch.equal(s_w, s_d)  # two different kernels really ran
    np.testing.assert_allclose(s_w.cpu().numpy(), s_d.cpu().numpy(), rtol=0, atol=SEG_ATOL)
    np.testing.assert_allclose(m_w.cpu().numpy(), m_d.cpu().numpy(), rtol=0, atol=MOT_ATOL)
    if shape[2] <= 16:
        from oracle import r2plus1d_ref as R
        import clasfv_amd.weights as W
        rs, rm = R.forward(W.synthetic_state_dict(W.DEFAULT_SEED), x.numpy())
        np.testing.assert_allclose(s_w.cpu().numpy(), rs.numpy(), rtol=0, atol=SEG_ATOL)
        np.testing.assert_allclose(s_d.cpu().numpy(), rs.numpy(), rtol=0, atol=SEG_ATOL)


@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 96), (1, 3, 32, 112, 112)])
def test_kernel_variants_bitexact(model, shape):
    """The patch-tiled spatial Winograd kernel (conv_wino_q) and the rolling-halo temporal one
    (conv_winot5) compute the same products in the same accumulation order as conv_wino / conv_winot:
    the forward must be bit-identical with them switched off (F(2x2,3x3) everywhere: variant
    no_wino4). Split-K (conv_winot5 / conv_dma on maps of <= 256 voxels per clip: layer4) sums the
    same products in another order: within 5e-5."""
    rng = np.random.default_rng(23)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    model.set_kernel_variants("no_wino4")
    s_split, m_split = model(x)
    model.set_kernel_variants("no_wino4", "no_split_k")
    s_new, m_new = model(x)
    model.set_kernel_variants("no_wino4", "no_wino_patch", "winot_reference", "no_split_k")
    s_old, m_old = model(x)
    model.set_kernel_variants()
    assert torch.equal(s_new, s_old) and torch.equal(m_new, m_old)
    # summation order only: a few ulps of the layer4 sums, grown through the decoder (logits ~5)
    assert (s_split - s_new).abs().max().item() <= 5e-5 and (m_split - m_new).abs().max().item() <= 5e-6


@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 96), (1, 3, 32, 112, 112), (3, 3, 24, 32, 32), (2, 3, 16, 64, 48)])
def test_wino4_matches_wino2(model, shape):
    """conv_wino4 (Winograd F(4x4,3x3), the default for the layer1/layer2 spatial convs) against
    conv_wino_q / conv_wino (F(2x2,3x3), variant no_wino4): different fp32 rounding of the same
    convolution, within the forward bar; the mask labels agree except where |l1 - l0| is at that
    rounding level. Shapes cover 14-, 12- and 16-tile groups and groups spanning two frames."""
    rng = np.random.default_rng(41)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    s4, m4 = model(x)
    model.set_kernel_variants("no_wino4")
    s2, m2 = model(x)
    model.set_kernel_variants()
    assert not torch.equal(s4, s2)  # the F(4x4) kernel really ran
    np.testing.assert_allclose(s4.cpu().numpy(), s2.cpu().numpy(), rtol=0, atol=SEG_ATOL)
    np.testing.assert_allclose(m4.cpu().numpy(), m2.cpu().numpy(), rtol=0, atol=MOT_ATOL)
    d = (s4[:, 1] - s4[:, 0]).cpu().numpy()
    flips = ((s4[:, 1] > s4[:, 0]) != (s2[:, 1] > s2[:, 0])).cpu().numpy()
    assert np.all(np.abs(d[flips]) <= 2 * SEG_ATOL)


@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 96), (1, 3, 32, 112, 112), (3, 3, 24, 32, 32), (2, 3, 16, 64, 48),
                                   (1, 3, 16, 112, 224)])
def test_wino4w_bitexact_vs_wino4(model, shape):
    """The wide-block F(4x4,3x3) kernels issue conv_wino4's products in conv_wino4's order, so the
    forward is bit-identical across all three, with each kernel really running: conv_wino4r (the
    default: 12 row waves per block, three per SIMD; winograd4w.hip), conv_wino4w (variant no_wino4r:
    4 quadrant waves, one per SIMD) and conv_wino4 (variant no_wino4w: 48-channel blocks). Wide blocks
    cover 144 / 288 / 576 channels as 144-channel blocks and 480 as 96; 240 stays on conv_wino4."""
    rng = np.random.default_rng(47)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    outs = []
    for variant, kernel in ((None, "conv_wino4r"), ("no_wino4r", "conv_wino4w"), ("no_wino4w", "conv_wino4")):
        if variant:
            model.set_kernel_variants(variant)
        model.engine.set_kernel_timing(True)
        outs.append(model(x))
        kt = model.engine.kernel_timing()
        model.engine.set_kernel_timing(False)
        model.set_kernel_variants()
        assert kernel in kt, (variant, sorted(kt))
        if kernel != "conv_wino4":
            assert "conv_wino4r" not in kt or "conv_wino4w" not in kt
    for s_v, m_v in outs[1:]:
        assert torch.equal(outs[0][0], s_v) and torch.equal(outs[0][1], m_v)


@pytest.mark.parametrize("shape", [(1, 3, 32, 112, 112), (2, 3, 16, 64, 48), (3, 3, 8, 32, 32)])
def test_proj_x3_bitexact_vs_dma_x3(model, shape):
    """The decoder's 128-deep tap projections (P01 = W0 f_stem + W1 f_layer1, P2) on the persistent
    conv_proj_x3 (conv.hip) against conv_dma_x3 (variant no_proj_x3): the same six split-bf16 products
    per 32-deep K block in the same order and the same epilogue, so the forward is bit-identical."""
    rng = np.random.default_rng(59)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    model.engine.set_kernel_timing(True)
    s_p, m_p = model(x)
    kt = model.engine.kernel_timing()
    model.engine.set_kernel_timing(False)
    assert kt["conv_proj_x3"]["launches"] == 2  # P01 and P2
    model.set_kernel_variants("no_proj_x3")
    s_d, m_d = model(x)
    model.set_kernel_variants()
    assert torch.equal(s_p, s_d) and torch.equal(m_p, m_d)


@pytest.mark.parametrize("shape", [(2, 3, 32, 112, 112), (3, 3, 24, 80, 112)])
def test_bf16_patch32_bitexact_vs_patch16(shape):
    """config[4]: the bf16 layer1 spatial convs (NB 5) and, since round 6, layer2's and layer3's
    stride-1 spatial convs (NB 4 / 3 / 5 / 3 for 256 / 288 / 480 / 576 channels) on conv_patch32_bf16 (v_mfma_f32_32x32x16_bf16,
    4-frame blocks, LDS-staged stores) against conv_patch_bf16 (16x16x32, 2-frame blocks; variant
    no_patch32): the same bf16 products summed in fp32 -- bit-identical outputs on the box (convbench
    CB_CHECK over 4.8e8 layer1 outputs, profiles/r04_patch32_bf16.txt; layer2/3: r06k), asserted here on
    the whole forward: 10 launches (layer1's four, layer2's and layer3's three; layer4's 7x7 maps give
    too few blocks per clip) at 32x112x112 and with 40x56 layer1 maps."""
    from clasfv_amd.model import R2plus1D_18_MotionNet
    rng = np.random.default_rng(53)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    m16 = R2plus1D_18_MotionNet(pretrained=False, dtype="bf16")
    m16.engine.set_kernel_timing(True)
    s_32, mo_32 = m16(x)
    kt = m16.engine.kernel_timing()
    m16.engine.set_kernel_timing(False)
    assert kt["conv_patch32_bf16"]["launches"] == 10, kt.keys()
    m16.set_kernel_variants("no_patch32")
    s_16, mo_16 = m16(x)
    m16.set_kernel_variants()
    assert torch.isfinite(s_32).all()
    assert torch.equal(s_32, s_16) and torch.equal(mo_32, mo_16)


@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 96), (1, 3, 8, 32, 48)])
def test_decoder_x3_matches_fp32_mfma(model, shape):
    """The fp32 engines' comb_2 on six split-bf16 products (hi/mid/lo pieces of both operands, fp32
    accumulation) against the fp32 MFMA comb_2 (variant no_decoder_x3): the same 64x64 product to
    fp32 rounding, so the outputs differ only at the accumulation-order level."""
    rng = np.random.default_rng(43)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    s3, m3 = model(x)
    model.set_kernel_variants("no_decoder_x3")
    s1, m1 = model(x)
    model.set_kernel_variants()
    assert not torch.equal(s3, s1)  # the split-bf16 comb_2 really ran
    np.testing.assert_allclose(s3.cpu().numpy(), s1.cpu().numpy(), rtol=0, atol=SEG_ATOL / 10)
    np.testing.assert_allclose(m3.cpu().numpy(), m1.cpu().numpy(), rtol=0, atol=MOT_ATOL / 4)


@pytest.mark.parametrize("dtype,variants", [
    ("fp32", "w4r_cached_stores"),
    ("bf16", "patch32_cached_stores"),
])
def test_store_cache_policy_variants_bitexact(dtype, variants):
    """Round 5's output-store cache policies (csrc: __builtin_nontemporal_store in conv_wino4r and
    conv_patch32_bf16, the product; their cached predecessors as variants): only the stores' cache
    hint differs, so the forward is bit-identical."""
    from clasfv_amd.model import R2plus1D_18_MotionNet
    rng = np.random.default_rng(67)
    x = torch.from_numpy(rng.uniform(0, 1, (2, 3, 32, 112, 112)).astype(np.float32)).cuda()
    m = R2plus1D_18_MotionNet(pretrained=False, dtype=dtype)
    s0, m0 = m(x)
    m.set_kernel_variants(*variants.split("+"))
    s1, m1 = m(x)
    m.set_kernel_variants()
    assert torch.isfinite(s0).all()
    assert torch.equal(s0, s1) and torch.equal(m0, m1)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 96), (2, 3, 32, 112, 112), (3, 3, 8, 32, 48)])
def test_buffer_dmas_bitexact(dtype, shape):
    """Round 5's buffer-offset LDS-DMAs (csrc/conv.hip BUF: per-row tap-validity bits and 32-bit byte
    offsets; out-of-range offsets read zeros) in conv_dma_x3 (fp32 engines) and conv_dma (bf16 engines:
    strided / 1x1x1 convs and the decoder projections) against the 64-bit pointer form (variant
    no_dma_buf): the same bytes land in LDS, so the forward is bit-identical -- padded taps, rows past
    M and the dual-input projections included."""
    from clasfv_amd.model import R2plus1D_18_MotionNet
    rng = np.random.default_rng(71)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    m = R2plus1D_18_MotionNet(pretrained=False, dtype=dtype)
    m.engine.set_kernel_timing(True)
    s0, m0 = m(x)
    kt = m.engine.kernel_timing()
    m.engine.set_kernel_timing(False)
    assert ("conv_dma_x3" in kt) if dtype == "fp32" else ("conv_dma" in kt or "conv_dma_w" in kt)
    m.set_kernel_variants("no_dma_buf")
    s1, m1 = m(x)
    m.set_kernel_variants()
    assert torch.isfinite(s0).all()
    assert torch.equal(s0, s1) and torch.equal(m0, m1)


@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 96), (2, 3, 32, 112, 112), (3, 3, 8, 32, 48)])
def test_bf16_dma_w_bitexact(shape):
    """The bf16 engines' direct convs on conv_dma_w (csrc/conv.hip: 128-B LDS rows, two 32-deep K steps
    per ring stage, every DMA row a whole line of a tap's channels) against conv_dma (64-B rows; variant
    no_dma_w): the same bf16 products accumulated in the same order, so the forward is bit-identical
    (convbench CB_CHECK on layer2 / layer3 strided convs: profiles/r05ao_conv_dma_w.txt)."""
    from clasfv_amd.model import R2plus1D_18_MotionNet
    rng = np.random.default_rng(73)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    m = R2plus1D_18_MotionNet(pretrained=False, dtype="bf16")
    m.engine.set_kernel_timing(True)
    s0, m0 = m(x)
    kt = m.engine.kernel_timing()
    m.engine.set_kernel_timing(False)
    assert "conv_dma_w" in kt
    m.set_kernel_variants("no_dma_w")
    s1, m1 = m(x)
    m.set_kernel_variants()
    assert torch.isfinite(s0).all()
    assert torch.equal(s0, s1) and torch.equal(m0, m1)


@pytest.mark.parametrize("variant", ["no_dma_x3", "no_stem_x3"])
@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 96), (1, 3, 32, 112, 112), (3, 3, 8, 32, 48)])
def test_x3_convs_match_fp32_mfma(model, shape, variant):
    """The fp32 engines' split-bf16 convs (six bf16 products of 3-piece operands per K block, fp32
    accumulation) against the same convs on fp32 MFMAs: conv_dma_x3 (strided / 1x1x1 convs, decoder
    projections) vs conv_dma (variant no_dma_x3), conv_stem_x3 vs conv_stem_f32 (no_stem_x3). The
    same GEMMs to fp32 rounding, so the forward stays within the fp32 bar and the mask labels agree
    except at that rounding level."""
    rng = np.random.default_rng(47)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    s3, m3 = model(x)
    model.set_kernel_variants(variant)
    model.engine.set_kernel_timing(True)
    s1, m1 = model(x)
    kt = model.engine.kernel_timing(cap=32)
    model.engine.set_kernel_timing(False)
    model.set_kernel_variants()
    # the variant really moves those GEMMs (the decoder projections included) onto f32 MFMAs
    gone = ("conv_dma_x3", "conv_proj_x3") if variant == "no_dma_x3" else ("conv_stem_x3",)
    assert not any(k in kt for k in gone), sorted(kt)
    assert not torch.equal(s3, s1)  # the split-bf16 GEMM really ran
    np.testing.assert_allclose(s3.cpu().numpy(), s1.cpu().numpy(), rtol=0, atol=SEG_ATOL)
    np.testing.assert_allclose(m3.cpu().numpy(), m1.cpu().numpy(), rtol=0, atol=MOT_ATOL)
    d = (s3[:, 1] - s3[:, 0]).cpu().numpy()
    flips = ((s3[:, 1] > s3[:, 0]) != (s1[:, 1] > s1[:, 0])).cpu().numpy()
    assert np.all(np.abs(d[flips]) <= 2 * SEG_ATOL)


@pytest.mark.parametrize("shape", [(2, 3, 16, 64, 96), (1, 3, 32, 112, 112), (1, 3, 8, 32, 48)])
def test_c8_blocked_mid_bitexact(model, shape):
    """The 8-channel-blocked mid tensors (stem and Conv2Plus1D spatial -> temporal Winograd) only
    change where values live in HBM: the forward is bit-identical to the channels-last one
    (variant no_c8)."""
    rng = np.random.default_rng(31)
    x = torch.from_numpy(rng.uniform(0, 1, shape).astype(np.float32)).cuda()
    s_b, m_b = model(x)
    model.set_kernel_variants("no_c8")
    s_c, m_c = model(x)
    model.set_kernel_variants()
    assert torch.equal(s_b, s_c) and torch.equal(m_b, m_c)


# ---- north_star bar on BASELINE config[1] (round 2) -----------------------------------------------

NORTHSTAR_FIXTURES = {"echo": "northstar_c1.npz", "random": "northstar_c1_random.npz", "deep": "northstar_c1_deep.npz"}


def _northstar(recipe="echo"):
    import clasfv_amd.synthetic as S
    g = golden(NORTHSTAR_FIXTURES[recipe])
    assert str(g["weights_recipe"]) == recipe
    video = fuse_ref.zeroone_normalizer(S.echo_video(int(g["T"]), seed=int(g["seed"])))
    return g, video


def _recipe_model(request, recipe):
    # echo: the bench's weights (masks follow the LV, physiological EFs; layer2-4 reach the LV margin
    # at ~1e-2 only). random: every layer at full gain, so every conv of the encoder moves the masks.
    # deep (round 6): the echo segmentation routed through layer2-4 at full gain.
    if recipe == "deep":
        return request.getfixturevalue("deep_model")
    return request.getfixturevalue("echo_model" if recipe == "echo" else "model")


@pytest.mark.parametrize("recipe", ["echo", "random", "deep"])
def test_northstar_config1_pass_labels_vs_cpu(request, recipe):
    """Config[1] (200 frames, 5 shifted passes, 30 clips) through the real HIP model: every pass's
    label video (clips built on the GPU, batched forward, softmax -> resample -> argmax) against the
    CPU reference path (oracle model + numpy plumbing, tests/golden/make_golden_northstar.py)."""
    from clasfv_amd import fuse_utils as FU
    model = _recipe_model(request, recipe)
    g, video = _northstar(recipe)
    T, F, step = int(g["T"]), int(g["fuse"]), int(g["step"])
    v = torch.from_numpy(video).cuda()
    k = FU.clamp_num_clips(T, F, step)
    table, clip0 = FU.clip_table(T, k, step)
    labels = FU.pass_labels(FU.run_model(model, FU.build_clips(v, table)), clip0, T, step).cpu().numpy()
    frames = g["pass_frames"]
    ref_all = np.unpackbits(g["passes"])[: int(frames.sum()) * 112 * 112]
    at = 0
    for j, n in enumerate(frames):
        ref = ref_all[at: at + n * 112 * 112].reshape(n, 112, 112)
        at += n * 112 * 112
        got = labels[j, :n]
        assert dice_delta(got, ref) <= DICE_TOL, j
        assert (got != ref).mean() <= 1e-4, j


@pytest.mark.parametrize("recipe", ["echo", "random", "deep"])
@pytest.mark.parametrize("method", ["majority", "simple", "staple"])
def test_northstar_config1_fused_masks_and_ef_vs_cpu(request, recipe, method):
    """north_star bar (BASELINE.json): fused masks Dice delta <= 1e-3 and EF within 1e-3 of the CPU
    reference path, on config[1] with the real HIP model, through the drop-in
    segment_a_video_with_fusion (src/fuse_utils.py:36-100) and compute_ef_using_putative_clips
    (src/fuse_utils.py:105-148), for both weight recipes. The EF bar is 1e-3 for the echo recipe
    (physiological EFs); the random recipe's EFs sit near 100 % (ES volume ~0), where one pixel moves
    the EF by ~1e-3, so its EF bar is 1e-2 and that recipe is judged by Dice delta <= 1e-3 and
    identical ED/ES pairs. SIMPLE / STAPLE fusion: the CPU side is the oracle restatement
    (LabelFusion absent: parity with LabelFusion itself unpinned)."""
    from clasfv_amd import fuse_utils as FU
    from clasfv_amd.echo import compute_ef_using_putative_clips
    model = _recipe_model(request, recipe)
    g, video = _northstar(recipe)
    out = FU.segment_a_video_with_fusion(video, model, num_clips=int(g["fuse"]), step=int(g["step"]),
                                         fuse_method=method)
    shp = tuple(g[f"fused_{method}_shape"])
    ref = np.unpackbits(g[f"fused_{method}"])[: int(np.prod(shp))].reshape(shp).astype(np.int64)
    assert out.dtype == np.int64 and out.shape == ref.shape
    assert dice_delta(out, ref) <= DICE_TOL
    efs, pairs = compute_ef_using_putative_clips(out, "gpu", return_edes=True)
    assert np.array(pairs, np.int64).reshape(-1, 2).tolist() == g[f"pairs_{method}"].tolist()
    # random recipe: EFs ~100 % (ES volume ~0), where a one-pixel change moves the EF by ~1e-3
    np.testing.assert_allclose(np.array(efs, np.float64), g[f"ef_{method}"], rtol=0,
                               atol=1e-2 if recipe == "random" else 1e-3, equal_nan=True)
    if recipe != "random":  # physiological: the masks follow the LV
        assert np.all((30 < g[f"ef_{method}"]) & (g[f"ef_{method}"] < 80))


@pytest.mark.parametrize("K,T,step", [(3, 30, 1), (5, 40, 1), (17, 60, 1), (6, 50, 3), (40, 80, 1)])
def test_fuse_staple_vs_oracle(K, T, step):
    """STAPLE fusion kernel vs the oracle restatement (same iteration; float64 reductions in a
    different order, so a pixel whose posterior is within rounding of 0.5 could differ)."""
    from clasfv_amd import fuse_utils as FU
    passes = _noisy_passes(K, T, step, seed=K * 7 + T)
    labels = np.zeros((K, T) + passes[0].shape[1:], np.uint8)
    for k, p in enumerate(passes):
        labels[k, :p.shape[0]] = p
    got = FU.fuse_votes(torch.from_numpy(labels).cuda(), step, "staple").cpu().numpy()
    ref = fuse_ref.fuse_frames(passes, T, step, "staple")
    assert got.shape == ref.shape
    assert (got != ref).mean() <= 1e-5


@pytest.mark.parametrize("method", ["simple", "majority"])
def test_fuse_40_passes(method):
    """The reference accepts any num_clips (-f 40): K up to 64 passes."""
    from clasfv_amd import fuse_utils as FU
    K, T, step = 40, 70, 1
    passes = _noisy_passes(K, T, step, seed=404)
    labels = np.zeros((K, T) + passes[0].shape[1:], np.uint8)
    for k, p in enumerate(passes):
        labels[k, :p.shape[0]] = p
    got = FU.fuse_votes(torch.from_numpy(labels).cuda(), step, method).cpu().numpy()
    np.testing.assert_array_equal(got, fuse_ref.fuse_frames(passes, T, step, method))


def test_pipeline_f40_runs_like_reference():
    from clasfv_amd import fuse_utils as FU
    v = _norm_video(120, 9)
    for meth in ("majority", "simple"):
        def np_model(x):
            s, m = fake_model(torch.from_numpy(np.ascontiguousarray(x)))
            return s.numpy(), m.numpy()
        out = FU.segment_a_video_with_fusion(v, fake_model, num_clips=40, fuse_method=meth)
        ref = fuse_ref.segment_a_video_with_fusion(v, np_model, num_clips=40, fuse_method=meth)
        np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("T,step", [(70, 1), (96, 2), (200, 1)])
def test_pass_labels_from_margins_bitexact(T, step):
    """The multi-GPU exchange payload: labels from the logit margin l1 - l0 equal labels from both
    logit planes bit for bit (including resampled passes and near-tie logits)."""
    from clasfv_amd import fuse_utils as FU
    k = FU.clamp_num_clips(T, 4, step)
    table, clip0 = FU.clip_table(T, k, step)
    rng = np.random.default_rng(T)
    lg = rng.normal(0, 2, (len(table), 2, 32, 40, 48)).astype(np.float32)
    lg[:, 1, :, :4] = lg[:, 0, :, :4]                                   # exact ties
    lg[:, 1, :, 4:8] = np.nextafter(lg[:, 0, :, 4:8], np.float32(np.inf))  # 1-ulp margins
    logits = torch.from_numpy(lg).cuda()
    a = FU.pass_labels(logits, clip0, T, step)
    m = FU.logit_margin(logits)
    assert torch.equal(m, logits[:, 1] - logits[:, 0])
    b = FU.pass_labels(m, clip0, T, step, margin=True)
    for j in range(k):  # pass j has T - j*step frames (the rest of its row is unused)
        assert torch.equal(a[j, :T - j * step], b[j, :T - j * step]), j


def test_cli_default_device_cpu_matches_cuda(tmp_path):
    """Reference default -d cpu: host video and outputs, engine on GPU 0, same masks as -d cuda."""
    import pickle
    import subprocess
    import sys
    import clasfv_amd.synthetic as S
    vid = tmp_path / "echo_dev.npy"
    np.save(vid, S.echo_video_uint8(90, seed=6))
    outs = {}
    for dev in (None, "cuda"):
        d = tmp_path / (dev or "default")
        d.mkdir()
        cmd = [sys.executable, "motion_segment.py", "-p", str(vid), "--synthetic-weights", "1234", "-f", "3",
               "-c", "binary_video", "-o", str(d)] + (["-d", dev] if dev else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        if dev is None:
            assert "engine runs on GPU 0" in r.stderr
        outs[dev] = pickle.load(open(d / "echo_dev_whole_video_segmentation.pkl", "rb"))
    assert outs[None].dtype == np.int64 and np.array_equal(outs[None], outs["cuda"])


def test_normalizer_workspace_per_call_streams():
    """The normaliser's partials live in a caller-owned workspace (no shared static buffer): two
    videos normalised on two streams give the single-stream results."""
    from clasfv_amd.preprocess import zeroone_normalize_
    import clasfv_amd.synthetic as S
    a = torch.from_numpy(S.echo_video(64, seed=1)).cuda()
    b = torch.from_numpy(S.echo_video(64, seed=2)).cuda() * 0.5 + 3
    ra, rb = zeroone_normalize_(a.clone()), zeroone_normalize_(b.clone())
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        xa = zeroone_normalize_(a.clone())
    with torch.cuda.stream(s2):
        xb = zeroone_normalize_(b.clone())
    torch.cuda.synchronize()
    assert torch.equal(xa, ra) and torch.equal(xb, rb)


def test_video_stream_matches_per_video_pipeline(model):
    """Pipelined multi-video front end (pinned H2D on a copy stream, device preprocessing, no host
    sync between videos) == the drop-in per-video path on the same frames."""
    import clasfv_amd.synthetic as S
    from clasfv_amd import fuse_utils as FU
    from clasfv_amd.preprocess import preprocess_video
    from clasfv_amd.stream import VideoStream
    vids = [S.echo_video_uint8(T, seed=40 + T) for T in (70, 100, 45, 64)]
    vids.append(S.echo_video_uint8(50, 96, 128, seed=7))  # resized to 112x112 on the device
    got = VideoStream(model, num_clips=3, fuse_method="simple").run(vids)
    for v, g in zip(vids, got):
        ref = FU.segment_a_video_with_fusion(preprocess_video(v), model, num_clips=3, fuse_method="simple")
        assert g.dtype == np.int64
        np.testing.assert_array_equal(g, ref)


# ---- round 3: config[4] on the north_star video, CLI vs the CPU path, non-strict plumbing -------

@pytest.mark.parametrize("recipe", ["echo", "random", "deep"])
def test_northstar_config4_bf16_fused_masks_vs_cpu(recipe):
    """BASELINE config[4] bar on the config[1] video: the bf16 engine's fused masks (SIMPLE, 5 passes)
    against the CPU reference path's fp32 masks: Dice delta <= 1e-2 and EF close. Both weight recipes:
    with the echo weights layer2-4 reach the LV margin at ~1e-2 only, so the random recipe (every layer
    at full gain) is the case where bf16 rounding in layer2-4 can move masks. echo: same ED/ES pairs,
    every EF within 1 point. random: the ES masks are near-empty (EFs ~100 %, SURVEY-style degenerate
    systoles), so the ES frame is a near-tie among almost-empty frames (measured: 31 vs 33 in one
    systole) -- that recipe is judged by Dice and the mean EF within 1 point."""
    from clasfv_amd import fuse_utils as FU
    from clasfv_amd.echo import compute_ef_using_putative_clips
    from clasfv_amd.model import R2plus1D_18_MotionNet
    g, video = _northstar(recipe)
    m16 = R2plus1D_18_MotionNet(pretrained=False, weights=recipe, dtype="bf16")
    out = FU.segment_a_video_with_fusion(video, m16, num_clips=int(g["fuse"]), step=int(g["step"]),
                                         fuse_method="simple")
    shp = tuple(g["fused_simple_shape"])
    ref = np.unpackbits(g["fused_simple"])[: int(np.prod(shp))].reshape(shp).astype(np.int64)
    d = dice_delta(out, ref)
    efs, pairs = compute_ef_using_putative_clips(out, "bf16", return_edes=True)
    print(f"config[4] {recipe}: Dice delta {d:.3e}, EFs {np.round(efs, 3).tolist()} vs "
          f"{np.round(g['ef_simple'], 3).tolist()}, pairs {np.array(pairs).reshape(-1, 2).tolist()}")
    assert d <= 1e-2, d
    if recipe == "echo":
        assert np.array(pairs, np.int64).reshape(-1, 2).tolist() == g["pairs_simple"].tolist()
        np.testing.assert_allclose(np.array(efs, np.float64), g["ef_simple"], rtol=0, atol=1.0)
    elif recipe == "deep":
        # deep (round 6): the band's intensity is 30 % layer2-4 taps at full gain (a 1 % change of those
        # taps flips ~18 mask pixels per clip on the CPU path, none with the echo weights), so here bf16
        # rounding anywhere in the encoder reaches masks with physiological EFs (~78.5 %): the same
        # systoles with each ED / ES frame within one frame (the LV area plateaus at ED, so bf16 can move
        # find_peaks' pick to a neighbouring frame: measured 149 vs 150 once), every EF within 1 point
        got_p, ref_p = np.array(pairs, np.int64).reshape(-1, 2), g["pairs_simple"]
        assert got_p.shape == ref_p.shape and np.abs(got_p - ref_p).max() <= 1, (got_p.tolist(), ref_p.tolist())
        np.testing.assert_allclose(np.array(efs, np.float64), g["ef_simple"], rtol=0, atol=1.0)
    else:
        # (an ES frame whose mask is empty in both the ED and ES frame gives EF = 0/0: measured once)
        e_g, e_c = np.array(efs, np.float64), np.array(g["ef_simple"], np.float64)
        both = np.isfinite(e_g) & np.isfinite(e_c)
        assert len(e_g) == len(e_c) and both.sum() >= len(e_c) - 1
        assert abs(float(np.mean(e_g[both])) - float(np.mean(e_c[both]))) <= 1.0


@pytest.mark.timeout(300)
def test_cli_outputs_vs_oracle_cpu_path(tmp_path):
    """motion_segment.py (-d cpu default, -f 2, -v, pickles) against the CPU reference path on the
    same .npy video: the oracle's preprocessing (motion_segment.py:96-106), segment_a_video_with_fusion
    (src/fuse_utils.py:36-100, oracle model + numpy plumbing) and compute_ef_using_putative_clips.
    The ED/ES pickles and the whole-video pickle match the CPU masks (Dice delta <= 1e-3), and the
    -v text (systole count, ED/ES frames, EFs to 2 decimals) is the CPU path's text."""
    import pickle
    import subprocess
    import sys
    import clasfv_amd.synthetic as S
    import clasfv_amd.weights as W
    from clasfv_amd.echo import compute_ef_using_putative_clips
    frames = S.echo_video_uint8(100, seed=4)
    vid = tmp_path / "echo_case.npy"
    np.save(vid, frames)
    r = subprocess.run([sys.executable, "motion_segment.py", "-p", str(vid), "--synthetic-weights", "1234", "-f", "2",
                        "-c", "binary,binary_video", "-o", str(tmp_path), "-v"], capture_output=True, text=True,
                       timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "R2+1D MotionNet has 31575731 parameters." in r.stdout
    torch.set_num_threads(16)
    video = fuse_ref.zeroone_normalizer(fuse_ref.preprocess_frames(frames))
    cpu_model = r2plus1d_ref.OracleModel(W.echo_state_dict(1234))
    ref = fuse_ref.segment_a_video_with_fusion(video, cpu_model, num_clips=2, fuse_method="simple",
                                               to_numpy=lambda t: t.numpy())
    efs, pairs = compute_ef_using_putative_clips(ref, str(vid), return_edes=True)
    whole = pickle.load(open(tmp_path / "echo_case_whole_video_segmentation.pkl", "rb"))
    assert whole.dtype == np.int64 and whole.shape == ref.shape
    assert dice_delta(whole, ref) <= DICE_TOL
    assert len(pairs) >= 1 and all(30 < e < 80 for e in efs)
    for ed, es in pairs:
        for kind, idx in (("ED", ed), ("ES", es)):
            m = pickle.load(open(tmp_path / f"echo_case_{kind}_Frame_{idx}_segmentation.pkl", "rb"))
            assert m.dtype == np.int64 and m.shape == (112, 112)
            assert dice_delta(m, ref[idx]) <= 1e-2
    lines = ["Identified {:d} systoles".format(len(efs))]
    if efs:
        lines.append("")
        lines.append("Ejection fractions measured at each systole are:")
        for i, (ed, es) in enumerate(pairs):
            lines.append("Systole #{:d}: ED {:d} & ES {:d} length={:d}".format(i + 1, ed, es, es - ed))
            lines.append("EF: {:.2f}".format(efs[i]))
            lines.append("")
        lines.append("The average ejection fraction is {:.2f}".format(np.mean(efs)))
    got = r.stdout[r.stdout.index("Identified"):].rstrip("\n").split("\n")
    assert got == lines, (got, lines)


def test_non_strict_plumbing_single_clip_and_step_frames():
    """strict_reference=False: T = 32 yields the single pass's masks instead of the
    reference's IndexError (src/fuse_utils.py:38-42,82), and step > 1 keeps frames 1..step-1 with
    their single pass-0 vote (:85) -- every other frame equals the strict output."""
    from clasfv_amd import fuse_utils as FU

    def np_model(x):
        s, m = fake_model(torch.from_numpy(np.ascontiguousarray(x)))
        return s.numpy(), m.numpy()
    v32 = _norm_video(32, 32)
    with pytest.raises(IndexError):
        FU.segment_a_video_with_fusion(v32, fake_model, num_clips=1)
    out = FU.segment_a_video_with_fusion(v32, fake_model, num_clips=1, strict_reference=False)
    np.testing.assert_array_equal(out, fuse_ref.pass_labels(v32, np_model, 0))
    for T, f, step in ((80, 3, 2), (40, 5, 3), (70, 4, 1)):
        v = _norm_video(T, 100 + T)
        strict = FU.segment_a_video_with_fusion(v, fake_model, step=step, num_clips=f, fuse_method="majority")
        loose = FU.segment_a_video_with_fusion(v, fake_model, step=step, num_clips=f, fuse_method="majority",
                                               strict_reference=False)
        assert strict.shape[0] == T - (step - 1) and loose.shape[0] == T
        np.testing.assert_array_equal(loose[0], strict[0])
        np.testing.assert_array_equal(loose[step:], strict[1:])
        np.testing.assert_array_equal(loose[1:step], fuse_ref.pass_labels(v, np_model, 0)[1:step])


@pytest.mark.parametrize("K,T,step", [(2, 20, 1), (4, 40, 1), (6, 50, 3), (5, 30, 1)])
def test_fuse_itkvoting_vs_oracle(K, T, step):
    """itkvoting: itk::LabelVotingImageFilter's rule (ties -> undecided label 2), restated in the oracle
    (parity with SimpleITK itself unpinned: it is absent); majority keeps ties -> 0."""
    from clasfv_amd import fuse_utils as FU
    passes = _noisy_passes(K, T, step, seed=K * 11 + T)
    labels = np.zeros((K, T) + passes[0].shape[1:], np.uint8)
    for k, p in enumerate(passes):
        labels[k, :p.shape[0]] = p
    lab = torch.from_numpy(labels).cuda()
    got = FU.fuse_votes(lab, step, "itkvoting").cpu().numpy()
    np.testing.assert_array_equal(got, fuse_ref.fuse_frames(passes, T, step, "itkvoting"))
    if K % 2 == 0:
        assert (got == 2).any()  # even vote counts produce ties
    np.testing.assert_array_equal(FU.fuse_votes(lab, step, "majority").cpu().numpy(),
                                  fuse_ref.fuse_frames(passes, T, step, "majority"))


@pytest.mark.parametrize("case", [0, 1, 2, 3])
def test_motion_seg_loss_windows_vs_reference_golden(case):
    """motion_seg_loss with ES before ED and with windows that start after the seed frames: the
    reference's forward chains ignore `start`, its backward chains `end` (src/clasfv_losses.py:83-130);
    loss values and gradients vs the reference's CPU run (tests/golden/make_golden_losses.py)."""
    import torch.nn.functional as F
    from clasfv_amd import losses as L
    from tests.golden.make_golden_losses import SGS_CASES, loss_inputs
    d, g = loss_inputs(), golden("losses.npz")
    ed_i, es_i, start, end = SGS_CASES[case]
    motion = torch.from_numpy(d["motion"]).cuda().requires_grad_()
    logits = torch.from_numpy(d["logits"]).cuda().requires_grad_()
    flow, ots = L.motion_seg_loss(d["ed"], d["es"], ed_i, es_i, motion, F.softmax(logits, dim=1), start=start,
                                  end=end)
    np.testing.assert_allclose(float(flow), g[f"sgs{case}_flow_loss"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(float(ots), g[f"sgs{case}_ots_loss"], rtol=1e-5, atol=1e-7)
    total = flow + ots
    if torch.is_tensor(total) and total.requires_grad:
        total.backward()
    gm = motion.grad.cpu().numpy() if motion.grad is not None else np.zeros_like(d["motion"])
    gl = logits.grad.cpu().numpy() if logits.grad is not None else np.zeros_like(d["logits"])
    np.testing.assert_allclose(gm, g[f"sgs{case}_grad_motion"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(gl, g[f"sgs{case}_grad_logits"], rtol=1e-4, atol=1e-7)


def test_video_stream_under_a_non_default_stream(model):
    """VideoStream.run orders its compute on the stream current at the call: results
    under `with torch.cuda.stream(s)` equal the per-video path, and the pinned ring is reused."""
    import clasfv_amd.synthetic as S
    from clasfv_amd import fuse_utils as FU
    from clasfv_amd.preprocess import preprocess_video
    from clasfv_amd.stream import VideoStream
    vids = [S.echo_video_uint8(T, seed=60 + T) for T in (64, 90, 50)]
    vs = VideoStream(model, num_clips=2, fuse_method="majority")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        got = vs.run(vids)
        again = vs.run(vids[::-1])
    for v, g_, a in zip(vids, got, again[::-1]):
        ref = FU.segment_a_video_with_fusion(preprocess_video(v), model, num_clips=2, fuse_method="majority")
        np.testing.assert_array_equal(g_, ref)
        np.testing.assert_array_equal(a, ref)
    assert all(b is not None for b in vs._ring)


# ---- round 3: config[2] (64 videos, clips sharded over ranks) ------------------------------------

C2_VIDEOS, C2_FRAMES = 64, 200


def _c2_worker(rank, world, port, q):
    import hashlib
    import os
    import torch.distributed as dist
    import clasfv_amd.synthetic as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from clasfv_amd import dist as D
        from clasfv_amd.model import R2plus1D_18_MotionNet
        from clasfv_amd.preprocess import zeroone_normalize_
        m = R2plus1D_18_MotionNet(pretrained=False, weights="echo")
        lengths = [C2_FRAMES] * C2_VIDEOS
        need = D.videos_needed(lengths, 1, 1, rank, world)
        vids = [None] * C2_VIDEOS
        for v in need:
            vids[v] = zeroone_normalize_(torch.from_numpy(S.echo_video(C2_FRAMES, seed=v)).cuda())
        out = D.segment_videos_sharded(vids, m, num_clips=1, step=1, fuse_method="simple", rank=rank, world=world,
                                       lengths=lengths)
        q.put((rank, len(need), {k: hashlib.sha1(v.cpu().numpy().tobytes()).hexdigest() for k, v in out.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_config2_64_videos_over_8_ranks_equals_one_rank(echo_model):
    """BASELINE config[2] plan (64 x 200-frame videos, f = 1: 384 clips) over its 8 ranks (gloo, all
    sharing the one GPU of the box): every video is fused on exactly one rank, no clip crosses ranks
    (rows_exchanged == 0: the owner mapping is block-aligned), each rank holds only its 8 videos, and
    every fused mask is bit-identical to the 1-rank result."""
    import hashlib
    import socket
    import torch.multiprocessing as mp
    import clasfv_amd.synthetic as S
    from clasfv_amd import dist as D
    from clasfv_amd.preprocess import zeroone_normalize_
    world = 8
    lengths = [C2_FRAMES] * C2_VIDEOS
    assert D.exchange_stats(lengths, 1, 1, world) == (0, 0)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, held = {}, {}
    for _ in range(world):
        r, n_need, out = q.get(timeout=600)
        held[r] = n_need
        assert not set(out) & set(got)
        got.update(out)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert sorted(got) == list(range(C2_VIDEOS)) and all(n == C2_VIDEOS // world for n in held.values())
    vids = [zeroone_normalize_(torch.from_numpy(S.echo_video(C2_FRAMES, seed=v)).cuda()) for v in range(C2_VIDEOS)]
    ref = D.segment_videos_sharded(vids, echo_model, num_clips=1, step=1, fuse_method="simple")
    for v in range(C2_VIDEOS):
        assert got[v] == hashlib.sha1(ref[v].cpu().numpy().tobytes()).hexdigest(), v


def _c2r_worker(rank, world, port, q, lengths):
    import hashlib
    import os
    import torch.distributed as dist
    import clasfv_amd.synthetic as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from clasfv_amd import dist as D
        from clasfv_amd.model import R2plus1D_18_MotionNet
        from clasfv_amd.preprocess import zeroone_normalize_
        m = R2plus1D_18_MotionNet(pretrained=False, weights="echo")
        need = D.videos_needed(lengths, 1, 1, rank, world)
        vids = [None] * len(lengths)
        for v in need:
            vids[v] = zeroone_normalize_(torch.from_numpy(S.echo_video(lengths[v], seed=v)).cuda())
        evs = []
        out = D.segment_videos_sharded(vids, m, num_clips=1, step=1, fuse_method="simple", rank=rank, world=world,
                                       lengths=lengths, exchange_events=evs)
        torch.cuda.synchronize()
        q.put((rank, len(evs), {k: hashlib.sha1(v.cpu().numpy().tobytes()).hexdigest() for k, v in out.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_config2_ragged_over_8_ranks_exchanges_and_equals_one_rank(echo_model):
    """config[2] with ragged EchoNet-like lengths (16 seeded videos of 100-300 frames, f = 1) over 8
    ranks (gloo, all on the box's one GPU): videos straddle the clip blocks, so the owner all_to_all
    really moves logit margins (rows_exchanged > 0, every rank records the exchange), and every fused
    mask is bit-identical to the 1-rank result."""
    import hashlib
    import socket
    import torch.multiprocessing as mp
    import clasfv_amd.synthetic as S
    from clasfv_amd import dist as D
    from clasfv_amd.preprocess import zeroone_normalize_
    world = 8
    lengths = S.echonet_like_lengths(16, seed=7)
    rows, nbytes = D.exchange_stats(lengths, 1, 1, world)
    assert rows > 0 and nbytes == rows * 32 * 112 * 112 * 4
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c2r_worker, args=(r, world, port, q, lengths)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, n_ev, out = q.get(timeout=600)
        assert n_ev == 1, (r, n_ev)
        assert not set(out) & set(got)
        got.update(out)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert sorted(got) == list(range(len(lengths)))
    vids = [zeroone_normalize_(torch.from_numpy(S.echo_video(t, seed=v)).cuda()) for v, t in enumerate(lengths)]
    ref = D.segment_videos_sharded(vids, echo_model, num_clips=1, step=1, fuse_method="simple")
    for v in range(len(lengths)):
        assert got[v] == hashlib.sha1(ref[v].cpu().numpy().tobytes()).hexdigest(), v


@pytest.mark.timeout(400)
def test_bench_c1_line_parity_with_steps_in_flight():
    """The default bench line at N = 1 keeps two steps in flight, and every parity object it reports --
    fp32 and bf16, against the echo / random / deep CPU fixtures -- is within its bar (the recipe
    checks run one-stream steps after a device sync: a step in flight on the other stream once
    handed its masks to the host before they were written)."""
    import json
    import subprocess
    import sys
    cmd = [sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--extra-c3", "0", "--extra-stream", "0",
           "--cpu-baseline", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["config"]["steps_in_flight"] == 2
    b = line["bf16"]
    checks = {"fp32": line["parity"], "fp32 random": line["parity_random_weights"], "fp32 deep": line["parity_deep_weights"],
              "bf16": b["parity_vs_cpu"], "bf16 random": b["parity_vs_cpu_random_weights"],
              "bf16 deep": b["parity_vs_cpu_deep_weights"]}
    for name, p in checks.items():
        assert p is not None and p["within_bar"], (name, p)
    assert line["parity_deep_weights"]["ed_es_pairs_equal"] and line["parity_deep_weights"]["ef_delta_max_per_systole"] <= 1e-3


@pytest.mark.timeout(400)
@pytest.mark.parametrize("workload", ["c1", "c2", "c2r"])
def test_bench_self_launches_ranks(workload):
    """`bench.py --gpus 2` without a launcher starts the 2 rank processes itself (here over gloo, both
    on the one GPU) and rank 0 prints one JSON line with n_gpus == 2; under a launcher WORLD_SIZE must
    equal --gpus."""
    import json
    import subprocess
    import sys
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1",
           "--extra-bf16", "0", "--extra-c3", "0", "--extra-stream", "0", "--cpu-baseline", "0",
           "--workload", workload[:2]]
    if workload == "c2":
        cmd += ["--c2-videos", "8", "--c2-extra-fuse", "0"]
    if workload == "c2r":  # ragged lengths: the owner exchange runs and is timed
        cmd += ["--c2-videos", "8", "--c2-extra-fuse", "0", "--c2-lengths", "ragged"]
    if workload == "c1":  # the c1 line's ragged config[2] extra, kept small here
        cmd += ["--c2-videos", "8"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    if workload == "c2":
        assert line["scaling"] == "strong" and line["rows_exchanged_per_step"] == 0
        assert [p["clips"] for p in line["per_rank"]] == [24, 24]
    elif workload == "c2r":
        assert line["scaling"] == "strong" and line["rows_exchanged_per_step"] > 0
        assert line["bytes_exchanged_per_step"] == line["rows_exchanged_per_step"] * 32 * 112 * 112 * 4
        assert line["exchange_ms_per_step"] > 0 and line["exchange_transfer_ms"] > 0
    else:
        assert line["config"]["clips_per_step"] == 60
        c2r = line["c2_ragged"]
        assert c2r["rows_exchanged_per_step"] > 0 and c2r["exchange_ms_per_step"] > 0
        assert c2r["exchange_transfer_ms"] > 0


# ---- round 4: RCCL on the leased GPU, config[0] through the CLI ------------------------------------

RCCL_LENGTHS = (70, 48, 90)


def _rccl_worker(port, q):
    """One rank of a world-size-1 RCCL ("nccl") group, created the way bench.py creates it: the
    collectives of the multi-GPU path (all_gather_into_tensor in all_gather_clips, all_to_all_single
    in exchange_to_owners) forced to run on device tensors."""
    import hashlib
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    try:
        from clasfv_amd import dist as D
        from clasfv_amd.model import R2plus1D_18_MotionNet
        from clasfv_amd.preprocess import zeroone_normalize_
        import clasfv_amd.synthetic as S
        backend = dist.get_backend()
        x = torch.arange(5 * 7, dtype=torch.float32, device=dev).reshape(5, 7)
        g = D.all_gather_clips(x, 5, 0, 1, force=True)
        owners = [0] * 5
        e = D.exchange_to_owners(x, owners, 0, 1, force=True)
        m = R2plus1D_18_MotionNet(pretrained=False)
        vids = [zeroone_normalize_(torch.from_numpy(S.echo_video(T, seed=T)).to(dev)) for T in RCCL_LENGTHS]
        forced = D.segment_videos_sharded(vids, m, num_clips=3, step=1, fuse_method="simple", force_exchange=True)
        plain = D.segment_videos_sharded(vids, m, num_clips=3, step=1, fuse_method="simple")
        torch.cuda.synchronize()
        q.put({"backend": backend, "gather_ok": bool(torch.equal(g, x)), "a2a_ok": bool(torch.equal(e, x)),
               "gather_dev": str(g.device), "forced": {k: hashlib.sha1(v.cpu().numpy().tobytes()).hexdigest()
                                                       for k, v in forced.items()},
               "plain": {k: hashlib.sha1(v.cpu().numpy().tobytes()).hexdigest() for k, v in plain.items()}})
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_world1_collectives_and_forced_exchange():
    """RCCL runs on the one leased GPU: a world-size-1 "nccl" process group (bench.py's
    init_process_group call, replacing the reference's nn.DataParallel, motion_segment.py:69) drives
    all_gather_into_tensor and all_to_all_single on device tensors (identity at one rank), and a
    sharded pass whose logit margins are forced through the all_to_all fuses bit-identically to the
    unexchanged logits."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(port, q))
    p.start()
    r = q.get(timeout=280)
    p.join(60)
    assert p.exitcode == 0
    assert r["backend"] == "nccl" and r["gather_dev"].startswith("cuda")
    assert r["gather_ok"] and r["a2a_ok"]
    assert sorted(r["forced"]) == list(range(len(RCCL_LENGTHS))) and r["forced"] == r["plain"]


@pytest.mark.timeout(300)
def test_cli_config0_single_clip_non_strict_vs_cpu(tmp_path):
    """BASELINE config[0] through the real CLI with the HIP model: one 32-frame 112x112 clip, fusion
    off (-f 1). The reference crashes there (num_clips clamps to 0, IndexError at
    src/fuse_utils.py:38-42,82) and so does the default (strict) CLI; --no-strict-reference yields the
    single pass's masks, which match the oracle CPU path's single-pass masks (Dice delta <= 1e-3)."""
    import pickle
    import subprocess
    import sys
    import clasfv_amd.synthetic as S
    import clasfv_amd.weights as W
    frames = S.echo_video_uint8(32, seed=7)
    vid = tmp_path / "one_clip.npy"
    np.save(vid, frames)
    base = [sys.executable, "motion_segment.py", "-p", str(vid), "--synthetic-weights", "1234", "-f", "1",
            "-c", "binary_video", "-o", str(tmp_path)]
    strict = subprocess.run(base, capture_output=True, text=True, timeout=280, cwd=REPO)
    assert strict.returncode != 0 and "IndexError" in strict.stderr, strict.stderr[-2000:]
    r = subprocess.run(base + ["--no-strict-reference"], capture_output=True, text=True, timeout=280, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    got = pickle.load(open(tmp_path / "one_clip_whole_video_segmentation.pkl", "rb"))
    torch.set_num_threads(16)
    video = fuse_ref.zeroone_normalizer(fuse_ref.preprocess_frames(frames))
    cpu_model = r2plus1d_ref.OracleModel(W.echo_state_dict(1234))
    ref = fuse_ref.pass_labels(video, cpu_model, 0, True, to_numpy=lambda t: t.numpy())
    assert got.dtype == np.int64 and got.shape == ref.shape == (32, 112, 112)
    assert dice_delta(got, ref) <= DICE_TOL

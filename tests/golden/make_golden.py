"""Generate tests/golden/*.npz by running the REFERENCE's own code.

Run in the build container only (``python tests/golden/make_golden.py``): it imports
``/root/reference/src/...`` with inert stubs for third-party modules that are absent from the image
(torchvision -> tests/golden/tv_stub.py restatement, SimpleITK -> identity array/image shim,
LabelFusion.fuse_images -> majority-vote stub that also records the votes it receives, echonet /
skimage / IPython / h5py -> empty modules). Nothing from the reference is written to the repo except
these input/output vectors. The EF fixtures need scikit-image and are produced by
``make_golden_ef.py`` under /opt/conda/bin/python3.9.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

VOTE_LOG = []


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def _majority_fuse(images, method, class_list=None):
    v = np.stack([np.asarray(i) for i in images])
    VOTE_LOG.append(len(images))
    counts = np.stack([(v == c).sum(0) for c in class_list])
    return np.asarray(class_list)[np.argmax(counts, 0)].astype(np.uint8)


class _Numpy119:
    """numpy namespace whose ``array`` builds an object array from ragged nested lists instead of
    raising (numpy 1.19 behaviour, relied on at src/fuse_utils.py:50 when shifted passes have
    different clip counts)."""

    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def array(x, *a, **k):
        try:
            return np.array(x, *a, **k)
        except ValueError:
            out = np.empty(len(x), dtype=object)
            for i, e in enumerate(x):
                out[i] = e
            return out


def install_stubs():
    from tests.golden import tv_stub
    tv_stub.install()
    _stub("SimpleITK", GetImageFromArray=lambda a, isVector=False: np.asarray(a), GetArrayFromImage=lambda a: np.asarray(a))
    _stub("LabelFusion")
    _stub("LabelFusion.wrapper", fuse_images=_majority_fuse)
    _stub("echonet")
    _stub("echonet.datasets", Echo=None)
    _stub("skimage")
    _stub("skimage.transform", resize=None, rescale=None, rotate=None)
    _stub("skimage.segmentation", find_boundaries=None)
    _stub("IPython")
    _stub("IPython.display", HTML=None)
    _stub("h5py")
    _stub("cv2", NORM_MINMAX=32)
    sys.path.insert(0, REF)


def main():
    install_stubs()
    torch.set_num_threads(8)
    from src.model.R2plus1D_18_MotionNet import R2plus1D_18_MotionNet
    from src import fuse_utils
    from src.echonet_dataset import zeroone_normalizer
    from src import transform_utils
    import clasfv_amd.weights as W
    import clasfv_amd.synthetic as S
    from tests.golden.fake_model import fake_model

    torch.Tensor.cuda = lambda self, *a, **k: self  # reference hard-codes .cuda() in the warp grid
    fuse_utils.np = _Numpy119()  # pinned numpy 1.19.2 (requirements.txt:109) builds ragged object arrays

    # ---- model forward through the reference module ------------------------------------------
    sd = W.synthetic_state_dict(W.DEFAULT_SEED)
    net = R2plus1D_18_MotionNet(pretrained=False)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    net.eval()
    nparams = sum(p.numel() for p in net.parameters() if p.requires_grad)
    keys = list(net.state_dict().keys())

    def norm_video(T, seed):
        return zeroone_normalizer(S.echo_video(T, seed=seed))

    rng = np.random.Generator(np.random.PCG64(7))
    x_small = rng.uniform(0, 1, (1, 3, 8, 32, 32)).astype(np.float32)
    with torch.no_grad():
        seg_s, mot_s = net(torch.from_numpy(x_small))
    vid = norm_video(64, seed=3)
    x_big = np.ascontiguousarray(vid[None, :, 16:48])
    with torch.no_grad():
        seg_b, mot_b = net(torch.from_numpy(x_big))
    seg_b = seg_b.numpy()
    mot_b = mot_b.numpy()
    lab_b = (seg_b[0, 1] > seg_b[0, 0])
    idx = rng.integers(0, seg_b[0, 0].size, 4096)
    np.savez_compressed(
        os.path.join(HERE, "model_forward.npz"),
        seed=W.DEFAULT_SEED, nparams=nparams, keys=np.array(keys),
        x_small=x_small, seg_small=seg_s.numpy(), mot_small=mot_s.numpy(),
        big_video_seed=3, big_T=64, big_start=16,
        big_label_bits=np.packbits(lab_b.ravel()), big_idx=idx,
        big_seg0=seg_b[0, 0].ravel()[idx], big_seg1=seg_b[0, 1].ravel()[idx],
        big_mot=mot_b[0].reshape(4, -1)[:, idx],
        big_seg_sum=seg_b.astype(np.float64).sum((0, 2, 3, 4)), big_mot_sum=mot_b.astype(np.float64).sum((0, 2, 3, 4)),
        big_seg_abs=np.abs(seg_b).astype(np.float64).sum())
    print("model_forward.npz", nparams, len(keys))

    # ---- plumbing (fusion off / on) with the deterministic fake model --------------------------
    cases = {}
    for T in (33, 48, 70, 80, 200):
        v = norm_video(T, seed=T)
        out = fuse_utils.segment_a_video_with_fusion(v, fake_model, interpolate_last=True, step=1, num_clips=1)
        cases[f"off_T{T}"] = out
    for T, f, step in ((70, 5, 1), (200, 5, 1), (80, 3, 2), (48, 10, 1), (40, 5, 3)):
        v = norm_video(T, seed=100 + T)
        VOTE_LOG.clear()
        out = fuse_utils.segment_a_video_with_fusion(v, fake_model, interpolate_last=True, step=step, num_clips=f,
                                                     fuse_method="simple", class_list=[0, 1])
        cases[f"on_T{T}_f{f}_s{step}"] = out
        cases[f"votes_T{T}_f{f}_s{step}"] = np.array(VOTE_LOG, np.int64)
    try:
        fuse_utils.segment_a_video_with_fusion(norm_video(32, 32), fake_model, num_clips=1)
        err32 = ""
    except Exception as e:  # the reference crashes at T=32 (K clamps to 0)
        err32 = type(e).__name__
    clips80 = fuse_utils.divide_to_consecutive_clips(norm_video(80, 80), interpolate_last=True)
    clips_ni = fuse_utils.divide_to_consecutive_clips(norm_video(64, 64), interpolate_last=False)
    packed = {k: (np.packbits(v.astype(bool)) if k.startswith(("off", "on")) else v) for k, v in cases.items()}
    shapes = {k + "_shape": np.array(v.shape) for k, v in cases.items()}
    dtypes = {k + "_dtype": np.array(str(v.dtype)) for k, v in cases.items()}
    np.savez_compressed(os.path.join(HERE, "plumbing.npz"), err_T32=np.array(err32), clips80_shape=np.array(clips80.shape),
                        clips80_dtype=np.array(str(clips80.dtype)), clips80_sum=clips80.sum((1, 2, 3, 4)),
                        clips80_sample=clips80[:, :, ::7, ::13, ::11].astype(np.float32),
                        clips64_sum=clips_ni.sum((1, 2, 3, 4)), **packed, **shapes, **dtypes)
    print("plumbing.npz", err32, {k: v.shape for k, v in cases.items()})

    # ---- plumbing with the real (reference) model, fusion off, T=48 ----------------------------
    v48 = norm_video(48, seed=48)

    def ref_model(x):
        with torch.no_grad():
            return net(x)
    lab48 = fuse_utils.segment_a_video_with_fusion(v48, ref_model, interpolate_last=True, step=1, num_clips=1)
    np.savez_compressed(os.path.join(HERE, "pipeline_model_T48.npz"), labels=np.packbits(lab48.astype(bool)),
                        shape=np.array(lab48.shape), dtype=np.array(str(lab48.dtype)), video_seed=48)
    print("pipeline_model_T48.npz", lab48.shape, lab48.mean())

    # ---- normaliser -------------------------------------------------------------------------------
    raw = S.echo_video(40, seed=5)
    nv = zeroone_normalizer(raw.copy())
    np.savez_compressed(os.path.join(HERE, "normalizer.npz"), T=40, seed=5, out_sample=nv[:, ::3, ::5, ::7],
                        out_sum=nv.astype(np.float64).sum((1, 2, 3)))

    # ---- motion warp: generate_2dmotion_field + grid_sample(border, align_corners=False) --------
    import torch.nn.functional as F
    wr = np.random.Generator(np.random.PCG64(11))
    img = np.ascontiguousarray(zeroone_normalizer(S.echo_video(4, seed=9))[:2, 1:3].transpose(1, 0, 2, 3))  # (2,2,112,112)
    box = np.zeros((1, 1, 112, 112), np.float32)
    box[..., 40:70, 50:60] = 1.0
    img_r = wr.uniform(0, 1, (1, 3, 48, 64)).astype(np.float32)  # non-square: catches H/W swaps
    flows = {
        "zero": (img, np.zeros((2, 2, 112, 112), np.float32)),
        "plus5px": (img, np.concatenate([np.full((2, 1, 112, 112), 10.0 / 112, np.float32),
                                         np.zeros((2, 1, 112, 112), np.float32)], 1)),
        "minus5px_y": (img, np.concatenate([np.zeros((2, 1, 112, 112), np.float32),
                                            np.full((2, 1, 112, 112), -10.0 / 112, np.float32)], 1)),
        "random": (img_r, np.tanh(wr.normal(0, 0.3, (1, 2, 48, 64))).astype(np.float32)),
        "large": (img_r, np.tanh(wr.normal(0, 3.0, (1, 2, 48, 64))).astype(np.float32)),
    }
    wout = {}
    for name, (im, fl) in flows.items():
        grid = transform_utils.generate_2dmotion_field(torch.from_numpy(im), torch.from_numpy(fl))
        wout["out_" + name] = F.grid_sample(torch.from_numpy(im), grid, align_corners=False,
                                            padding_mode="border").numpy()
        wout["flow_" + name] = fl
    gridb = transform_utils.generate_2dmotion_field(torch.from_numpy(box), torch.zeros(1, 2, 112, 112))
    wout["box_zero"] = F.grid_sample(torch.from_numpy(box), gridb, align_corners=False, padding_mode="border").numpy()
    np.savez_compressed(os.path.join(HERE, "warp.npz"), img=img, img_r=img_r, box=box, **wout)
    print("warp.npz", list(wout))


if __name__ == "__main__":
    main()

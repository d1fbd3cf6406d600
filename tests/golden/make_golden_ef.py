"""Generate tests/golden/ef.npz by running the REFERENCE's EF code
(``src/fuse_utils.compute_ef_using_putative_clips`` -> ``src/echonet_dataset.EDESpairs`` ->
``src/utils/echo_utils.get2dPucks`` with scikit-image ``find_boundaries``).

Run in the build container with the interpreter that has scikit-image:
``/opt/conda/bin/python3.9 tests/golden/make_golden_ef.py``. torch / SimpleITK / LabelFusion /
echonet are absent there and replaced by inert stubs (they are imported but not used on this path).
"""
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def _load_synthetic():
    p = os.path.join(REPO, "fully-automated-multi-heartbeat-echocardiography-video-segmentation-and-motion-tracking_amd",
                     "synthetic.py")
    spec = importlib.util.spec_from_file_location("synthetic_standalone", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def main():
    class _Obj(object):
        pass
    _stub("torch", Tensor=None)
    _stub("torch.nn")
    _stub("torch.nn.functional")
    _stub("torch.utils")
    _stub("torch.utils.data", Dataset=_Obj, DataLoader=None, Subset=None)
    sys.modules["torch"].nn = sys.modules["torch.nn"]
    sys.modules["torch.nn"].functional = sys.modules["torch.nn.functional"]
    _stub("SimpleITK")
    _stub("LabelFusion")
    _stub("LabelFusion.wrapper", fuse_images=None)
    _stub("echonet")
    _stub("echonet.datasets", Echo=None)
    _stub("h5py")
    sys.path.insert(0, "/root/reference")
    from src.fuse_utils import compute_ef_using_putative_clips
    from src.utils.echo_utils import get2dPucks

    S = _load_synthetic()
    rng = np.random.Generator(np.random.PCG64(21))
    videos = {}
    videos["ellipse200"] = S.ellipse_masks(200)
    v = S.ellipse_masks(200).copy()
    flips = rng.uniform(0, 1, v.shape) < 0.01
    v[flips] = 1 - v[flips]
    videos["noisy200"] = v
    videos["ellipse150_p37"] = S.ellipse_masks(150, period=37)
    v = S.ellipse_masks(120, period=45).copy()
    v[60:63] = 0
    videos["gap120"] = v
    videos["const64"] = np.repeat(S.ellipse_masks(1), 64, axis=0)
    v = S.ellipse_masks(160, period=40).copy()
    v[:, :, 70:] = 0  # truncated (non-convex after cut) LV
    v[::9, 10:14, 10:14] = 1  # small second component on some frames
    videos["twocomp160"] = v

    out = {}
    for name, m in videos.items():
        efs, pairs = compute_ef_using_putative_clips(m, test_pat_index=name, return_edes=True)
        out[name + "_bits"] = np.packbits(m.astype(bool))
        out[name + "_shape"] = np.array(m.shape)
        out[name + "_efs"] = np.array(efs, np.float64)
        out[name + "_pairs"] = np.array(pairs, np.int64).reshape(-1, 2)
        print(name, pairs, np.round(efs, 6))
    # get2dPucks on individual frames (Simpson's method of disks, 10 pucks)
    frames = [videos["ellipse200"][0], videos["ellipse200"][25], videos["noisy200"][13], videos["twocomp160"][9],
              videos["twocomp160"][20], np.zeros((112, 112), np.int64)]
    Ls, Rs = [], []
    for f in frames:
        L, R = get2dPucks((f == 1).astype("int"), (1.0, 1.0))
        Ls.append(L)
        Rs.append(R)
    out["pucks_frames"] = np.packbits(np.stack(frames).astype(bool))
    out["pucks_L"] = np.array(Ls, np.float64)
    out["pucks_R"] = np.stack(Rs).astype(np.float64)
    np.savez_compressed(os.path.join(HERE, "ef.npz"), names=np.array(list(videos)), **out)


if __name__ == "__main__":
    main()

"""Ejection fraction from fused LV masks (host side; per-video 1-D/2-D work, not data parallel).

Restates, with numpy + scipy only:
* ``compute_ef_using_putative_clips``  src/fuse_utils.py:105-148 (area curve -> percentiles ->
  scipy.signal.find_peaks for systole/diastole -> ED/ES pairs -> Simpson's method of disks)
* ``EDESpairs``                        src/echonet_dataset.py:159-172
* ``get2dPucks``                       src/utils/echo_utils.py:259-385 (principal axes via eig(cov),
  boundary = skimage ``find_boundaries(mode='thick')`` = grey dilation != grey erosion with the
  4-connected cross and reflect borders, 10 half-open bins along the major axis, radius = median
  |minor projection|; an empty bin gives NaN like the reference)
Pinned by tests/golden/ef.npz, produced by the reference code itself.
"""
import numpy as np
from scipy import ndimage
from scipy.signal import find_peaks

_CROSS = ndimage.generate_binary_structure(2, 1)


def find_boundaries_thick(label_img):
    img = np.asarray(label_img)
    if img.dtype == bool:
        img = img.astype(np.uint8)
    return ndimage.grey_dilation(img, footprint=_CROSS) != ndimage.grey_erosion(img, footprint=_CROSS)


def get2dPucks(abin, apix, npucks=10):
    """Length of the structure along its major axis and the npucks disk radii about it."""
    if ~np.any(abin):
        return 1.0, np.zeros((npucks,))
    x, y = np.where(abin > 0)
    X = np.stack([x, y])
    if X.shape[1] < 1:
        return (0.0, np.zeros((npucks,)))
    X = np.multiply(X, np.array(apix)[:, None])
    try:
        val, vec = np.linalg.eig(np.cov(X, rowvar=True))
    except Exception:
        return (0.0, np.zeros((npucks,)))
    order = np.argsort(val)[-1::-1]
    vec = vec[:, order]
    if vec[0, 0] < 0:
        vec[:, 0] = -1.0 * vec[:, 0]
    if vec[1, 1] < 0:
        vec[:, 1] = -1.0 * vec[:, 1]
    mu = np.expand_dims(np.mean(X, axis=1), axis=1)
    B = find_boundaries_thick(abin)
    Xb = np.stack(np.where(B))
    Xb = np.multiply(Xb, np.array(apix)[:, None])
    proj = np.dot((Xb - mu).T, vec)
    L_min, L_max = np.min(proj, axis=0), np.max(proj, axis=0)
    L = L_max - L_min
    edges = np.linspace(L_min[0], L_max[0], npucks + 1)
    R = []
    with np.errstate(invalid="ignore"):
        for i in range(len(edges) - 1):
            which = np.logical_and(proj[:, 0] >= edges[i], proj[:, 0] < edges[i + 1])
            # the reference's `len(which) == 0` guard never fires: an empty bin's median is NaN
            r = np.median(np.abs(proj[:, 1][which])) if which.any() else np.nan
            R.append(r)
    return L[0], np.array(R)


def EDESpairs(diastole, systole):
    diastole = np.sort(np.array(diastole))
    systole = np.sort(np.array(systole))
    clips = []
    inds = np.searchsorted(diastole, systole, side="left")
    for i, sf in enumerate(systole):
        if inds[i] == 0:
            continue
        best_df = diastole[inds[i] - 1]
        if len(clips) == 0 or best_df != clips[-1][0]:
            clips.append((best_df, sf))
    return clips


def compute_ef_using_putative_clips(fused_segmentations, test_pat_index, return_edes=False):
    seg = np.asarray(fused_segmentations)
    size = np.sum(seg, axis=(1, 2)).ravel()
    _05cut, _85cut, _95cut = np.percentile(size, [5, 85, 95])
    trim_range = _95cut - _05cut
    systole = find_peaks(-size, distance=20, prominence=(0.50 * trim_range))[0]
    diastole = find_peaks(size, distance=20, prominence=(0.50 * trim_range))[0]
    diastole = [x for x in diastole if size[x] >= _85cut]
    if np.mean(size[:3]) >= _85cut:
        diastole = [0] + diastole
    diastole = np.array(diastole)
    clip_pairs = EDESpairs(diastole, systole)
    frames = seg.reshape(-1, seg.shape[-2], seg.shape[-1])
    efs = []
    for ed, es in clip_pairs:
        l_ed, r_ed = get2dPucks((frames[ed] == 1).astype("int"), (1.0, 1.0))
        l_es, r_es = get2dPucks((frames[es] == 1).astype("int"), (1.0, 1.0))
        with np.errstate(invalid="ignore", divide="ignore"):
            edv = np.sum(((np.pi * r_ed * r_ed) * l_ed / len(r_ed)))
            esv = np.sum(((np.pi * r_es * r_es) * l_es / len(r_es)))
            ef = (edv - esv) / edv * 100
        if ef < 0:
            print("Negative EF at patient: " + str(test_pat_index))
            continue
        efs.append(ef)
    if return_edes:
        return efs, clip_pairs
    return efs


def categorical_dice(prediction, truth, k, epsilon=1e-5):
    """src/clasfv_losses.py:60-68 -- the Dice metric used for parity."""
    A = (np.asarray(prediction) == k)
    B = (np.asarray(truth) == k)
    return 2 * np.sum(A * B) / (np.sum(A) + np.sum(B) + epsilon)

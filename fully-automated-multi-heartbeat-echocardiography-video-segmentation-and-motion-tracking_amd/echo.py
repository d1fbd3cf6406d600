"""Ejection fraction from fused LV masks (host side: per-video 1-D / 2-D work, not data parallel).

Behaviour (not code) of the reference's EF stage, re-derived from SURVEY.md section 3.4:

* ``compute_ef_using_putative_clips(fused_segmentations, test_pat_index, return_edes=False)``
  (src/fuse_utils.py:105-148): LV area per frame -> 5/85/95th percentiles -> end-systoles are the
  area minima and end-diastoles the area maxima found by ``scipy.signal.find_peaks`` (distance 20,
  prominence half the 5-95 range), diastoles kept only when their area reaches the 85th percentile,
  frame 0 added as a diastole when the first three frames are that large -> each systole is paired
  with the latest diastole before it (``EDESpairs``, src/echonet_dataset.py:159-172) -> volumes by
  Simpson's monoplane method of disks -> EF = (EDV - ESV) / EDV * 100; negative EFs are reported and
  dropped.
* ``get2dPucks(abin, apix, npucks=10)`` (src/utils/echo_utils.py:259-385): the mask's principal axes
  (eigenvectors of the pixel-coordinate covariance, major axis first, each axis oriented so its own
  coordinate is non-negative), the mask's thick boundary (a pixel whose 4-neighbourhood, edges
  replicated, is mixed), the boundary's extent L along the major axis cut into ``npucks`` half-open
  slabs, and per slab the median distance of its boundary pixels from the major axis (NaN for an
  empty slab, as the reference); an empty mask gives (1.0, zeros), a mask whose covariance has no
  eigen-decomposition (one pixel) (0.0, zeros).
* ``compute_ef_batch``: the same for many videos on a thread pool (numpy / scipy release the GIL in
  their kernels), for the batched multi-video path.

Pinned by tests/golden/ef.npz, which the reference code itself produced (tests/golden/make_golden_ef.py).
"""
import warnings
from concurrent.futures import ThreadPoolExecutor

import numpy as np
from scipy.signal import find_peaks


def thick_boundary(mask):
    """Boolean map of the pixels whose 4-neighbourhood (edge pixels replicated) holds both values."""
    m = np.asarray(mask) != 0
    pad = np.pad(m, 1, mode="edge")
    stack = np.stack([pad[1:-1, 1:-1], pad[:-2, 1:-1], pad[2:, 1:-1], pad[1:-1, :-2], pad[1:-1, 2:]])
    return stack.any(axis=0) & ~stack.all(axis=0)


def get2dPucks(abin, apix, npucks=10):
    """(length along the major axis, npucks disk radii) of a binary mask; ``apix`` = pixel spacing
    per image axis. An empty mask gives (1.0, zeros) as in the reference."""
    mask = np.asarray(abin) > 0
    if not mask.any():
        return 1.0, np.zeros((npucks,))
    spacing = np.asarray(apix, dtype=np.float64).reshape(2, 1)
    pts = np.stack(np.nonzero(mask)) * spacing            # (2, n) pixel coordinates
    with np.errstate(invalid="ignore", divide="ignore"), warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)  # one-pixel masks: "Degrees of freedom <= 0"
        cov = np.cov(pts, rowvar=True)
    try:  # a one-pixel mask has an undefined (NaN) covariance: (0.0, zeros) as the reference
        evals, evecs = np.linalg.eig(cov)
    except np.linalg.LinAlgError:
        return 0.0, np.zeros((npucks,))
    axes = evecs[:, np.argsort(evals)[::-1]]            # major axis first
    axes = axes * np.where(np.diag(axes) < 0, -1.0, 1.0)  # axis i points along +coordinate i
    centre = pts.mean(axis=1, keepdims=True)
    rim = np.stack(np.nonzero(thick_boundary(mask))) * spacing
    coords = np.dot((rim - centre).T, axes)             # (n_rim, 2): (along, across) the major axis
    lo, hi = coords.min(axis=0), coords.max(axis=0)
    cuts = np.linspace(lo[0], hi[0], npucks + 1)
    slab = np.digitize(coords[:, 0], cuts, right=False) - 1  # cuts[i] <= x < cuts[i+1] -> i
    dist = np.abs(coords[:, 1])
    radii = np.array([np.median(dist[slab == i]) if np.any(slab == i) else np.nan for i in range(npucks)])
    return (hi - lo)[0], radii


def EDESpairs(diastole, systole):
    """[(ED, ES)]: every systole with the latest diastole strictly before it; a diastole already
    paired with an earlier systole is not paired again."""
    ed = np.sort(np.asarray(diastole))
    es = np.sort(np.asarray(systole))
    prev = np.searchsorted(ed, es, side="left") - 1
    pairs, last = [], -1
    for j, s in zip(prev, es):
        if j >= 0 and j != last:
            pairs.append((ed[j], s))
            last = j
    return pairs


def _disk_volume(length, radii):
    """Simpson's monoplane method: sum of npucks cylinders of height length / npucks."""
    return np.sum(np.pi * radii * radii * length / len(radii))


def compute_ef_using_putative_clips(fused_segmentations, test_pat_index, return_edes=False):
    seg = np.asarray(fused_segmentations)
    area = seg.sum(axis=(1, 2)).ravel()
    p5, p85, p95 = np.percentile(area, [5, 85, 95])
    prom = 0.50 * (p95 - p5)
    es = find_peaks(-area, distance=20, prominence=prom)[0]
    ed = [int(i) for i in find_peaks(area, distance=20, prominence=prom)[0] if area[i] >= p85]
    if np.mean(area[:3]) >= p85:
        ed.insert(0, 0)
    pairs = EDESpairs(np.array(ed), es)
    frames = seg.reshape(-1, seg.shape[-2], seg.shape[-1])
    efs = []
    for d, s in pairs:
        with np.errstate(invalid="ignore", divide="ignore"):
            edv = _disk_volume(*get2dPucks((frames[d] == 1).astype(int), (1.0, 1.0)))
            esv = _disk_volume(*get2dPucks((frames[s] == 1).astype(int), (1.0, 1.0)))
            ef = (edv - esv) / edv * 100
        if ef < 0:
            print("Negative EF at patient: " + str(test_pat_index))
            continue
        efs.append(ef)
    return (efs, pairs) if return_edes else efs


def compute_ef_batch(segmentations, names=None, return_edes=False, workers=8):
    """compute_ef_using_putative_clips over many fused mask videos on a thread pool."""
    names = list(names) if names is not None else list(range(len(segmentations)))
    with ThreadPoolExecutor(max(1, workers)) as ex:
        return list(ex.map(lambda a: compute_ef_using_putative_clips(a[0], a[1], return_edes),
                           zip(segmentations, names)))


def categorical_dice(prediction, truth, k, epsilon=1e-5):
    """Dice of class k (src/clasfv_losses.py:60-68), the parity metric: 2|A & B| / (|A| + |B| + eps)."""
    a = np.asarray(prediction) == k
    b = np.asarray(truth) == k
    return 2 * np.count_nonzero(a & b) / (np.count_nonzero(a) + np.count_nonzero(b) + epsilon)

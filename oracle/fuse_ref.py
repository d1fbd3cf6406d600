"""ORACLE (test infrastructure only -- never imported by the product path).

numpy restatement of the reference clip plumbing and label fusion, ``src/fuse_utils.py``:

* ``temporal_resample``      -- ``F.interpolate(..., size=(T_out, 112, 112), mode="trilinear",
                                align_corners=False)`` with H, W unchanged (fuse_utils.py:22-23, :75-76),
                                i.e. PyTorch's ``area_pixel_compute_source_index`` +
                                ``guard_index_and_lambda`` along time, evaluated in float32.
* ``divide_to_consecutive_clips``  (fuse_utils.py:16-33)
* ``segment_a_video_with_fusion``  (fuse_utils.py:36-100), including its quirks: banker's rounding
  of the clip count, the K clamp (:38-42), the IndexError when K == 0 (:82), and frames 1..step-1
  being dropped for step > 1 (:85).
* ``majority_vote`` / ``simple_vote`` -- the per-frame fusion rule. ``fuse_images`` lives in the
  unpinned, absent LabelFusion package: majority voting (ties -> lower label) is pinned only by the
  golden fixtures produced with the same rule as a stub; SIMPLE (Langerak et al. 2010, BraTS-toolkit
  form) and STAPLE (Warfield et al. 2004, ITK form) are restatements of the published algorithms and
  are **parity unpinned**.
"""
import numpy as np


def temporal_source_index(t_in, t_out):
    """(i0, i1, l0, l1) float32 lambdas for align_corners=False linear resampling t_in -> t_out."""
    dst = np.arange(t_out)
    if t_in == t_out:
        z = np.zeros(t_out, np.float32)
        return dst.copy(), dst.copy(), z + np.float32(1), z
    scale = np.float32(np.float32(t_in) / np.float32(t_out))
    # torch's CPU kernel is built with FMA contraction: src = fma(scale, dst + 0.5, -0.5)
    # (bit-exactness against F.interpolate is checked in tests/test_oracle.py)
    src = _fma(np.full(t_out, scale, np.float32), dst.astype(np.float32) + np.float32(0.5),
               np.full(t_out, -0.5, np.float32))
    src = np.maximum(src, np.float32(0)).astype(np.float32)
    i0 = np.minimum(np.floor(src).astype(np.int64), t_in - 1)
    l1 = np.clip(src - i0.astype(np.float32), np.float32(0), np.float32(1)).astype(np.float32)
    i1 = i0 + (i0 < t_in - 1)
    l0 = (np.float32(1) - l1).astype(np.float32)
    return i0, i1, l0, l1


def temporal_resample(x, t_out, axis=1):
    """Linear resampling along ``axis`` (float32 in/out), as trilinear with H, W unchanged."""
    x = np.asarray(x, np.float32)
    t_in = x.shape[axis]
    i0, i1, l0, l1 = temporal_source_index(t_in, t_out)
    a = np.take(x, i0, axis=axis)
    b = np.take(x, i1, axis=axis)
    shp = [1] * x.ndim
    shp[axis] = t_out
    l0 = np.broadcast_to(l0.reshape(shp), a.shape)
    l1 = np.broadcast_to(l1.reshape(shp), a.shape)
    # Interpolate<1>::eval: t * wts + t2 * wts2, contracted to fma(t, wts, t2 * wts2)
    return _fma(a, l0, (b * l1).astype(np.float32))


def _ac_true_index(n_in, n_out):
    """align_corners=True linear weights: scale = (float)(in-1)/(out-1), src = scale*dst (float32)."""
    scale = np.float32(np.float32(n_in - 1) / np.float32(n_out - 1)) if n_out > 1 else np.float32(0)
    src = (scale * np.arange(n_out).astype(np.float32)).astype(np.float32)
    i0 = np.minimum(src.astype(np.int64), n_in - 1)
    l1 = np.clip(src - i0.astype(np.float32), np.float32(0), np.float32(1)).astype(np.float32)
    return i0, i0 + (i0 < n_in - 1), (np.float32(1) - l1).astype(np.float32), l1


def preprocess_frames(frames, height=112, width=112):
    """motion_segment.py:96-104: (T,Hs,Ws,3) uint8 -> (3,T,Hs,Ws) float32 -> F.interpolate(size=(T,
    height, width), mode="trilinear", align_corners=True). The temporal level is the identity (T kept);
    W then H are combined as fma(x0, l0, x1*l1) (PyTorch's CPU Interpolate<>::eval, bit-exact).
    Not normalised (zeroone_normalizer follows in the reference)."""
    x = np.asarray(frames).transpose(3, 0, 1, 2).astype(np.float32)
    h0, h1, lh0, lh1 = _ac_true_index(x.shape[2], height)
    w0, w1, lw0, lw1 = _ac_true_index(x.shape[3], width)
    rows0, rows1 = x[:, :, h0], x[:, :, h1]
    lw0, lw1 = lw0[None, None, None, :], lw1[None, None, None, :]
    top = _fma(rows0[..., w0], lw0, (rows0[..., w1] * lw1).astype(np.float32))
    bot = _fma(rows1[..., w0], lw0, (rows1[..., w1] * lw1).astype(np.float32))
    return _fma(top, lh0[None, None, :, None], (bot * lh1[None, None, :, None]).astype(np.float32))


def _fma(x, y, z):
    """float32 fused multiply-add emulated in float64 (exact product, one final rounding)."""
    return (np.asarray(x, np.float64) * np.asarray(y, np.float64) + np.asarray(z, np.float64)).astype(np.float32)


def n_clip_frames(t, clip_length=32):
    return int(np.round(t / clip_length) * clip_length)  # np.round: half to even


def divide_to_consecutive_clips(video, clip_length=32, interpolate_last=False):
    """(3,T,H,W) -> (n,3,clip_length,H,W) float32 (the reference returns the same values as float64)."""
    t = video.shape[1]
    src = video
    if t % clip_length != 0 and interpolate_last:
        src = temporal_resample(video, n_clip_frames(t, clip_length), axis=1)
    clips = []
    for start in range(0, n_clip_frames(t, clip_length), clip_length):
        c = src[:, start:start + clip_length]
        if c.shape[1] != clip_length:
            raise ValueError("all the input array dimensions except for the concatenation axis must match exactly")
        clips.append(c)
    if not clips:
        return np.empty((0, 3, clip_length) + video.shape[2:], np.float32)
    return np.stack(clips).astype(np.float32)


def softmax2(logits):
    """softmax over axis 1 of (n,2,...) float32."""
    m = np.maximum(logits[:, 0:1], logits[:, 1:2])
    e = np.exp(logits - m)
    return (e / e.sum(axis=1, keepdims=True)).astype(np.float32)


def clamp_num_clips(t, num_clips, step):
    if t < 32 + num_clips * step:
        num_clips = (t - 32) // step
    if num_clips < 0:
        num_clips = 1
    return num_clips


def pass_labels(video, model, shift, interpolate_last=True, to_numpy=None):
    """Labels (T-shift, H, W) of one temporally shifted pass (fuse_utils.py:45-80)."""
    clips = divide_to_consecutive_clips(video[:, shift:], interpolate_last=interpolate_last)
    probs = []
    for c in clips:
        seg, _ = model(c[None])
        seg = to_numpy(seg) if to_numpy else np.asarray(seg)
        probs.append(softmax2(seg.astype(np.float32)))
    h, w = video.shape[2:]
    if probs:
        p = np.concatenate(probs).transpose(1, 0, 2, 3, 4).reshape(2, -1, h, w)
    else:
        p = np.zeros((2, 0, h, w), np.float32)
    tk = video.shape[1] - shift
    if interpolate_last and tk % 32 != 0:
        p = temporal_resample(p, tk, axis=1)
    return (p[1] > p[0]).astype(np.int64)  # np.argmax over 2 classes: ties -> 0


def majority_vote(votes, class_list=(0, 1)):
    """Per-pixel plurality over a list of label images; ties -> lowest label."""
    v = np.stack(votes)
    counts = np.stack([(v == c).sum(0) for c in class_list])
    return np.asarray(class_list)[np.argmax(counts, axis=0)].astype(np.uint8)


def itk_voting(votes, class_list=(0, 1)):
    """itk::LabelVotingImageFilter with the default undecided label (max input label + 1): plurality,
    a tie of the top counts -> undecided. PARITY UNPINNED (SimpleITK / LabelFusion absent)."""
    v = np.stack(votes).astype(np.int64)
    counts = np.stack([(v == c).sum(0) for c in class_list])
    top = counts.max(0)
    winners = (counts == top[None]).sum(0)
    undecided = int(v.max()) + 1
    out = np.asarray(class_list)[np.argmax(counts, axis=0)]
    return np.where(winners > 1, undecided, out).astype(np.uint8)


def _dice(a, b):
    s = a.sum() + b.sum()
    return 1.0 if s == 0 else 2.0 * float((a & b).sum()) / float(s)


def simple_vote(votes, class_list=(0, 1), t=0.05, stop=25, iterations=25):
    """SIMPLE (selective and iterative method for performance level estimation), BraTS-toolkit form:
    per label (descending), weighted majority of binarised candidates with weights (dice+1)^2 against
    the running estimate, candidates below t*max(weight) dropped, stop when the estimate's voxel
    count changes by < ``stop``. PARITY UNPINNED (LabelFusion source absent)."""
    result = np.zeros(votes[0].shape, np.uint8)
    for lab in sorted(class_list, reverse=True):
        cands = [(v == lab) for v in votes]
        w = [1.0] * len(cands)
        est = _weighted_mv(cands, w)
        conv = int(est.sum())
        for _ in range(iterations):
            w = [(_dice(c, est) + 1.0) ** 2 for c in cands]
            mx = max(w)
            keep = [i for i in range(len(cands)) if w[i] > t * mx]
            cands = [cands[i] for i in keep]
            w = [w[i] for i in keep]
            est = _weighted_mv(cands, w)
            if abs(conv - int(est.sum())) < stop:
                break
            conv = int(est.sum())
        result[est] = lab
    return result


def staple_vote(votes, class_list=(0, 1), max_iter=100, tol=1e-7, init=0.99999):
    """Binary STAPLE (Warfield, Zou & Wells 2004), in the form of ITK's STAPLEImageFilter: rater j's
    decision D_j = (vote == 1); prior f = mean of all decisions; sensitivity p_j / specificity q_j
    start at ``init``; E step W = f*P1 / (f*P1 + (1-f)*P0), P1 = prod_j (p_j if D_j else 1-p_j),
    P0 = prod_j (1-q_j if D_j else q_j) (products in rater order, float64); M step p_j = sum W D_j /
    sum W, q_j = sum (1-W)(1-D_j) / sum (1-W) (a zero denominator keeps the old value); stop when no
    p_j, q_j moves by more than ``tol`` or after ``max_iter`` iterations; label 1 where W > 0.5.
    ``fuse_images(..., "staple")`` of LabelFusion (src/fuse_utils.py:95) is absent: PARITY UNPINNED;
    this is the restatement the GPU kernel (plumbing.hip fuse_staple_kernel) is checked against."""
    d = np.stack([np.asarray(v) == 1 for v in votes]).reshape(len(votes), -1)
    nv, npx = d.shape
    f = d.sum() / float(nv * npx)
    p = np.full(nv, init)
    q = np.full(nv, init)

    def e_step(p, q):
        a = np.full(npx, f)
        b = np.full(npx, 1.0 - f)
        for j in range(nv):
            a = a * np.where(d[j], p[j], 1.0 - p[j])
            b = b * np.where(d[j], 1.0 - q[j], q[j])
        s = a + b
        with np.errstate(invalid="ignore", divide="ignore"):
            return np.where(s > 0, a / s, f)

    for _ in range(max_iter):
        w = e_step(p, q)
        sw = w.sum()
        sn = npx - sw
        np_ = np.array([(w * d[j]).sum() / sw if sw > 0 else p[j] for j in range(nv)])
        nq_ = np.array([((1.0 - w) * ~d[j]).sum() / sn if sn > 0 else q[j] for j in range(nv)])
        done = np.all(np.abs(np_ - p) <= tol) and np.all(np.abs(nq_ - q) <= tol)
        p, q = np_, nq_
        if done:
            break
    return (e_step(p, q) > 0.5).astype(np.uint8).reshape(np.asarray(votes[0]).shape)


def _weighted_mv(cands, w):
    on = np.zeros(cands[0].shape, np.float64)
    off = np.zeros(cands[0].shape, np.float64)
    for c, wi in zip(cands, w):
        on += c * wi
        off += (~c) * wi
    return on > off


FUSERS = {"majority": majority_vote, "majorityvoting": majority_vote, "mv": majority_vote,
          "itkvoting": itk_voting, "voting": itk_voting, "simple": simple_vote, "staple": staple_vote}


def fuse_frames(passes, t, step, fuse_method="simple", class_list=(0, 1)):
    """Per-frame fusion loop (fuse_utils.py:82-100). ``passes[k]`` is (T-k*step, H, W)."""
    if len(passes) == 0:
        raise IndexError("list index out of range")
    fuse = FUSERS[fuse_method.lower()]
    fused = [passes[0][0]]
    for i in range(1, t):
        if step - 1 < i:
            votes = []
            for idx in range(min(i, len(passes))):
                if i - idx * step < 0:
                    break
                votes.append(passes[idx][i - idx * step].astype(np.uint8))
            if len(votes) <= 1:
                fused.append(votes[0])
            else:
                fused.append(fuse(votes, class_list).astype(np.uint8))
    return np.array(fused).astype(np.int64)


def segment_a_video_with_fusion(video, model, interpolate_last=True, step=1, num_clips=10, fuse_method="simple",
                                class_list=(0, 1), to_numpy=None):
    t = video.shape[1]
    k = clamp_num_clips(t, num_clips, step)
    passes = [pass_labels(video, model, s, interpolate_last, to_numpy) for s in range(0, k * step, step)]
    return fuse_frames(passes, t, step, fuse_method, class_list)


def zeroone_normalizer(video):
    """src/echonet_dataset.py:38-50, float32 in place semantics."""
    v = np.array(video, np.float32, copy=True)
    shp = v.shape
    v = v.reshape(3, -1)
    v -= v.min(axis=1).reshape(3, 1)
    v /= v.max(axis=1).reshape(3, 1)
    return v.reshape(shp)

"""Seeded synthetic weights for ``R2plus1D_18_MotionNet`` and checkpoint I/O.

No trained weights exist offline (README.md:14 points at Google Drive) and ``pretrained=True``
(src/model/R2plus1D_18_MotionNet.py:13) would download Kinetics weights, so benchmarks and parity
tests use a deterministic numpy PCG64 stream. Same seed -> bit-identical tensors on every host,
so only the seed needs to travel.

Checkpoints in the reference format ``{"model": state_dict}`` with ``module.``-prefixed keys
(motion_segment.py:69-72) are read with ``torch.load(..., weights_only=True)``.
"""
from collections import OrderedDict

import numpy as np

from .arch import state_dict_spec, strip_module_prefix

DEFAULT_SEED = 1234
# Segmentation-head bias offset for class 1 (LV). Chosen so that a random-weight network on the
# synthetic EchoNet-style video labels a non-trivial fraction of voxels as LV, which keeps the Dice
# parity metric meaningful (class-1 share measured in tests/test_host_logic.py).
SEG_BIAS_LV = -2.4


def synthetic_state_dict(seed=DEFAULT_SEED):
    """OrderedDict name -> numpy array, reference key names, float32 (int64 for num_batches_tracked)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = OrderedDict()
    for name, shape in state_dict_spec().items():
        if name.endswith("num_batches_tracked"):
            sd[name] = np.array(0, dtype=np.int64)
            continue
        n = int(np.prod(shape)) if shape else 1
        if name.endswith("running_mean"):
            a = rng.normal(0.0, 0.1, n)
        elif name.endswith("running_var"):
            a = rng.uniform(0.5, 2.0, n)
        elif len(shape) == 1 and ("batch_norm" in name or _is_bn(name)):
            a = rng.uniform(0.8, 1.2, n) if name.endswith(".weight") else rng.normal(0.0, 0.1, n)
        elif name.endswith(".bias"):
            a = rng.normal(0.0, 0.05, n)
        elif name == "motion_head.weight":
            a = rng.normal(0.0, np.sqrt(1e-5), n)  # reference init, R2plus1D_18_MotionNet.py:23
        else:
            fan_in = int(np.prod(shape[1:]))
            a = rng.normal(0.0, np.sqrt(2.0 / fan_in), n)
        sd[name] = a.astype(np.float32).reshape(shape)
    sd["segmentation_head.bias"] = sd["segmentation_head.bias"] + np.array([0.0, SEG_BIAS_LV], np.float32)
    return sd


# "echo" recipe constants (see echo_state_dict). Intensities are in zero-one-normalised units of the
# synthetic video (synthetic.py): outside the sector ~0.12, LV blood pool ~0.19-0.21, sector ~0.74.
ECHO = {
    "S0": 10.0,        # stem output scale of the designed channels
    "box": 5,          # stem intensity box (pixels, odd, <= 7)
    "haar": 7,         # stem Haar gradient window (pixels, odd, <= 7): wider than the box, so an edge
                       # is flagged before it raises the box mean
    "g": 0.0,          # layer1 residual-branch gain of the 3x3-box-smoothed channels (0: pass-through)
    "band": (0.168, 0.210, 0.252),  # LV band of the smoothed intensity (low, centre, high)
    "c": 100.0,        # comb_1 slope of the band ramps
    "eps": 0.5,        # comb_2 threshold of the band response
    "dark": 0.26,      # below this a band pixel may be the sector border's crossing, not blood pool
    "k": 50.0,         # slope of the dark / edge indicators (0 -> 1 over 1/k)
    "grad": 0.12,      # smoothed |gradient| (L1 of 4 Haar responses) of an edge
    "k_grad": 20.0,
    "A": 10.0,         # seg-head gain of the band response
    "A_edge": 100.0,   # seg-head weight of the dark-and-edge indicator (vetoes the band)
    "noise": 1e-4,     # scale of the random weights kept on every other input of a designed unit
}


def _identity_bn(sd, bn, rows, gamma=1.0):
    for r in rows:
        sd[bn + ".weight"][r] = gamma
        sd[bn + ".bias"][r] = 0.0
        sd[bn + ".running_mean"][r] = 0.0
        sd[bn + ".running_var"][r] = 1.0 - 1e-5  # var + eps == 1: the folded scale is gamma


def echo_state_dict(seed=DEFAULT_SEED, p=None):
    """Seeded weights whose segmentation follows the synthetic video's LV (physiological EFs).

    The "random" recipe (synthetic_state_dict) exercises every kernel but segments noise, so its
    fused masks give degenerate EFs (~100 %). This recipe keeps every weight of that recipe except a
    small designed path, so every conv still computes dense random channel mixes:

    * stem 1x7x7: channel 0 = box mean of the intensity over the central box x box window,
      channels 1-4 = rectified Haar gradients over a haar x haar window (+x, -x, +y, -y);
    * stem 3x1x1: channel 0 = mean of frames (t, t+1) of channel 0, channel 5 = relu of
      (mean of (t-1, t)) - (mean of (t, t+1)), so channel 0 + channel 5 = the larger of the two
      2-frame means -- right at both clip ends despite the zero temporal padding; channels 1-4 pass
      through (centre tap);
    * layer1 (both blocks): the 6 channels pass through the residual (branch gain g of a 3x3 box
      smoothing, 0 by default);
    * comb_1 (ReLU ramps of the intensity L = ch0 + ch5 and gradient magnitude G = ch1 + .. + ch4 of
      the layer1 tap): a triangle band response over L, and clamped indicators "L is dark" and
      "G is an edge";
    * comb_2: the band response above a threshold, and the AND of the two indicators;
    * seg head: logit1 - logit0 = A * band - A_edge * (dark AND edge) - 0.1.
    LV = smoothed intensity in the blood-pool band, except on strong edges (where the band crosses
    the bright sector's border: outside the sector the video is almost as dark as the LV).

    Every designed unit keeps the random recipe's weights on its other inputs, scaled by
    p["noise"], so the other taps (layer2-4) still reach the logits.
    """
    p = dict(ECHO, **(p or {}))
    sd = synthetic_state_dict(seed)
    R = "r2plus1d_model."
    S0, g = p["S0"], p["g"]
    nd = 6  # designed channels: intensity, +x, -x, +y, -y gradients, intensity end correction
    bs, hs = int(p["box"]), int(p["haar"])
    o, oh = (7 - bs) // 2, (7 - hs) // 2
    h2 = hs // 2
    # stem 1x7x7 (45, 3, 1, 7, 7)
    w = sd[R + "stem.0.weight"]
    w[:nd] = 0.0
    w[0, :, :, o:o + bs, o:o + bs] = S0 / (3 * bs * bs)
    haar = np.zeros((7, 7), np.float32)
    haar[oh:oh + hs, 4:4 + h2] = 1.0
    haar[oh:oh + hs, 3 - h2:3] = -1.0
    for k, h in ((1, haar), (2, -haar), (3, haar.T), (4, -haar.T)):
        w[k] = (S0 / (3 * hs * h2)) * h[None, None]
    _identity_bn(sd, R + "stem.1", range(nd))
    w = sd[R + "stem.3.weight"]  # (64, 45, 3, 1, 1): taps t-1, t, t+1
    w[:nd] = 0.0
    w[0, 0, :, 0, 0] = (0.0, 0.5, 0.5)
    w[5, 0, :, 0, 0] = (0.5, 0.0, -0.5)
    for k in range(1, 5):
        w[k, k, 1] = 1.0
    _identity_bn(sd, R + "stem.4", range(nd))
    box = np.full((3, 3), 1.0 / 9.0, np.float32)
    for b in range(2):
        pre = f"{R}layer1.{b}."
        for conv, bn, kind, gain in (("conv1.0.0", "conv1.0.1", "box", 1.0), ("conv1.0.3", "conv1.1", "tap", 1.0),
                                     ("conv2.0.0", "conv2.0.1", "box", 1.0), ("conv2.0.3", "conv2.1", "tap", g)):
            w = sd[pre + conv + ".weight"]
            w[:nd] = 0.0
            if g:
                for k in range(nd):
                    if kind == "box":
                        w[k, k, 0] = box
                    else:
                        w[k, k, 1] = 1.0
            _identity_bn(sd, pre + bn, range(nd), gamma=gain)
    # decoder: comb_1 (64, 1024) rows 0-6 read layer1 channels 0-5 (concat columns 64..69)
    lo, mid, hi = p["band"]
    unit = (1.0 + g) ** 2 * S0  # layer1 channel value per unit of normalised intensity
    L = [64, 69]
    G = [65, 66, 67, 68]
    w1 = sd["comb_1_layer.weight"].reshape(64, 1024)
    b1 = sd["comb_1_layer.bias"]
    nr = 7
    w1[:nr] *= p["noise"]
    for r, t in enumerate((lo, mid, hi)):  # r0 - 2 r1 + r2: triangle over [lo, hi]
        w1[r, L] = p["c"] / unit
        b1[r] = -p["c"] * t
    k = p["k"]
    for r, off in ((3, 0.0), (4, -1.0)):  # r3 - r4 = clamp(k (dark - L), 0, 1)
        w1[r, L] = -k / unit
        b1[r] = k * p["dark"] + off
    for r, off in ((5, 0.0), (6, -1.0)):  # r5 - r6 = clamp(k_grad (G - grad), 0, 1)
        w1[r, G] = p["k_grad"] / unit
        b1[r] = -p["k_grad"] * p["grad"] + off
    _identity_bn(sd, "comb_batch_norm_1", range(nr))
    w2 = sd["comb_2_layer.weight"].reshape(64, 64)
    b2 = sd["comb_2_layer.bias"]
    w2[:2] *= p["noise"]
    w2[0, :3] = (1.0, -2.0, 1.0)
    b2[0] = -p["eps"]
    w2[1, 3:7] = (1.0, -1.0, 1.0, -1.0)  # AND of the two indicators
    b2[1] = -1.0
    _identity_bn(sd, "comb_batch_norm_2", [0, 1])
    ws = sd["segmentation_head.weight"].reshape(2, 64)
    ws *= 10 * p["noise"]
    ws[1, 0] = p["A"]
    ws[1, 1] = -p["A_edge"]
    sd["segmentation_head.bias"][:] = (0.0, -0.1)
    return sd


# "deep" recipe constants (see deep_state_dict)
DEEP = {
    "g_deep": 1.0,                     # branch gain of the designed channels in layer2-4 (full gain)
    "alpha": (0.7, 0.2, 0.07, 0.03),   # share of the layer1..layer4 taps in the band's intensity
    "floor": 0.172,                    # layer1 intensity below which a pixel is never LV
    # echo constants changed for this recipe: the blurred deep taps raise the intensity at the centre
    # of the narrow end-systolic LV, so the band reaches higher (and the dark-and-edge veto with it)
    "echo": {"band": (0.168, 0.25, 0.34), "dark": 0.35},
}


def deep_state_dict(seed=DEFAULT_SEED, p=None):
    """The "echo" segmentation routed through the WHOLE encoder at full gain (round 6).

    In the echo recipe the LV decision reads only the layer1 tap, so layer2-4 reach the logits at
    ~1e-4 and a bf16 engine's rounding there never moves a mask. Here the 6 designed channels
    (intensity, 4 rectified gradients, intensity end correction) also run through every BasicBlock
    of layer2-4 at full gain: the residual carries them (the strided 1x1x1 downsample as an identity
    per channel) and the branch adds a 3x3 box smoothing of each (sp1 / sp2 box, tp1 / tp2 centre
    tap, BN gamma g_deep) -- real 9-tap accumulations in bf16 weights and activations. comb_1's band
    rows read the intensity as a mix of all four taps (alpha: layer1 .. layer4, each normalised by its
    tap's gain), so roughly 60 % of the band input has passed through layer2-4 and been trilinearly
    upsampled from 28^2, 14^2 and 7^2 maps. The edge veto keeps reading layer1's gradients. Every
    other weight is the echo recipe's (random full-gain channels everywhere else)."""
    q = dict(DEEP, **(p or {}))
    pe = dict(q["echo"], **(p or {}))
    sd = echo_state_dict(seed, pe)
    e = dict(ECHO, **pe)
    R = "r2plus1d_model."
    nd = 6
    g = q["g_deep"]
    box = np.full((3, 3), 1.0 / 9.0, np.float32)
    for li in (2, 3, 4):
        for b in range(2):
            pre = f"{R}layer{li}.{b}."
            for conv, bn, kind in (("conv1.0.0", "conv1.0.1", "box"), ("conv1.0.3", "conv1.1", "tap"),
                                   ("conv2.0.0", "conv2.0.1", "box"), ("conv2.0.3", "conv2.1", "tap")):
                w = sd[pre + conv + ".weight"]
                w[:nd] = 0.0
                for k in range(nd):
                    if kind == "box":
                        w[k, k, 0] = box
                    else:
                        w[k, k, 1] = 1.0
                # the branch gain once per half (conv1's BN after the temporal conv, conv2's likewise)
                _identity_bn(sd, pre + bn, range(nd), gamma=g if kind == "tap" and conv == "conv2.0.3" else 1.0)
            if b == 0:
                w = sd[pre + "downsample.0.weight"]
                w[:nd] = 0.0
                for k in range(nd):
                    w[k, k, 0, 0, 0] = 1.0
                _identity_bn(sd, pre + "downsample.1", range(nd))
    # per-tap gain of the designed intensity: layer1 (1 + g1)^2 S0, then (1 + g_deep) per block
    unit1 = (1.0 + e["g"]) ** 2 * e["S0"]
    units = [unit1 * (1.0 + g) ** (2 * i) for i in range(4)]
    col0 = (64, 128, 256, 512)  # concat column of each tap's channel 0 (layer1 .. layer4)
    w1 = sd["comb_1_layer.weight"].reshape(64, 1024)
    b1 = sd["comb_1_layer.bias"]
    lo, mid, hi = e["band"]
    for r, t in enumerate((lo, mid, hi)):
        w1[r, [64, 69]] = 0.0
        for a, u, c in zip(q["alpha"], units, col0):
            w1[r, [c, c + 5]] = a * e["c"] / u
        b1[r] = -e["c"] * t
    # "very dark" veto: the blurred deep taps put the band on the dark side of the sector's border,
    # beyond the reach of layer1's edge indicator; r7 - r8 = clamp(k (floor - L1), 0, 1) on layer1's
    # intensity (outside the sector ~0.12, blood pool ~0.19-0.21) drives comb_2 row 2 and the seg head
    k = e["k"]
    w1[7:9] *= e["noise"]
    for r, off in ((7, 0.0), (8, -1.0)):
        w1[r, [64, 69]] = -k / unit1
        b1[r] = k * q["floor"] + off
    _identity_bn(sd, "comb_batch_norm_1", [7, 8])
    w2 = sd["comb_2_layer.weight"].reshape(64, 64)
    b2 = sd["comb_2_layer.bias"]
    w2[2] *= e["noise"]
    w2[2, 7:9] = (1.0, -1.0)
    b2[2] = 0.0
    _identity_bn(sd, "comb_batch_norm_2", [2])
    sd["segmentation_head.weight"].reshape(2, 64)[1, 2] = -e["A_edge"]
    return sd


RECIPES = {"random": synthetic_state_dict, "echo": echo_state_dict, "deep": deep_state_dict}


def recipe_state_dict(recipe="random", seed=DEFAULT_SEED):
    if recipe not in RECIPES:
        raise ValueError(f"weights recipe must be one of {sorted(RECIPES)}")
    return RECIPES[recipe](seed)


def _is_bn(name):
    # backbone BN modules are the odd-indexed / ".1" entries named in arch.backbone_convs()
    from .arch import backbone_convs
    global _BN_NAMES
    try:
        bn_names = _BN_NAMES
    except NameError:
        bn_names = _BN_NAMES = {c.bn for _, c in backbone_convs()}
    return name.rsplit(".", 1)[0] in bn_names


def load_checkpoint(path):
    """Reference checkpoint -> OrderedDict of numpy arrays with the ``module.`` prefix stripped."""
    import torch
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict) and "model" in obj:
        obj = obj["model"]
    out = OrderedDict()
    for k, v in obj.items():
        out[strip_module_prefix(k)] = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
    return out


def save_checkpoint(path, state_dict, module_prefix=True):
    """Write ``{"model": state_dict}`` the way the reference training notebook does."""
    import torch
    sd = OrderedDict()
    for k, v in state_dict.items():
        sd[("module." if module_prefix else "") + k] = torch.from_numpy(np.array(v, copy=True))
    torch.save({"model": sd}, path)

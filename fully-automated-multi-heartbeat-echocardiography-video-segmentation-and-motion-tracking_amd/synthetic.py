"""Synthetic EchoNet-Dynamic-shaped inputs (the licensed dataset is not available offline).

Video recipe: three identical grayscale channels; background speckle U(0,1)*60,
a bright ultrasound sector (cone) and a dark LV ellipse whose semi-axes pulse with period 50 frames:
phi = (1 + cos(2*pi*t/50)) / 2, a = 22 + 10*phi (rows), b = 10 + 5*phi (cols), centred at (56, 56)
of a 112x112 frame. uint8, numpy PCG64 seeded per video.
"""
import numpy as np


def lv_phase(t, period=50):
    return 0.5 * (1.0 + np.cos(2.0 * np.pi * np.asarray(t, np.float64) / period))


def ellipse_masks(T, H=112, W=112, period=50):
    """(T,H,W) int64 LV masks of the pulsing ellipse (EF known-answer recipe)."""
    t = np.arange(T)[:, None, None]
    y = np.arange(H)[None, :, None]
    x = np.arange(W)[None, None, :]
    phi = lv_phase(t, period)
    a = 22.0 + 10.0 * phi
    b = 10.0 + 5.0 * phi
    cy, cx = (H / 2.0), (W / 2.0)
    return ((((y - cy) / a) ** 2 + ((x - cx) / b) ** 2) <= 1.0).astype(np.int64)


def echo_video_uint8(T=200, H=112, W=112, seed=0, period=50):
    """(T,H,W,3) uint8 RGB video, the layout cv2 decoding produces in motion_segment.py:86-94."""
    rng = np.random.Generator(np.random.PCG64(seed))
    speckle = rng.uniform(0.0, 1.0, (T, H, W)) * 60.0
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    apex_y, apex_x = 0.04 * H, W / 2.0
    r = np.hypot(yy - apex_y, xx - apex_x)
    ang = np.arctan2(xx - apex_x, yy - apex_y)
    cone = (np.abs(ang) < 0.75) & (r < 0.95 * H)
    img = speckle.copy()
    img[:, cone] += 110.0 + 60.0 * rng.uniform(0.0, 1.0, (T, int(cone.sum())))
    lv = ellipse_masks(T, H, W, period).astype(bool)
    img[lv] *= 0.25
    v = np.clip(img, 0, 255).astype(np.uint8)
    return np.repeat(v[..., None], 3, axis=-1)


def echo_video(T=200, H=112, W=112, seed=0, period=50):
    """(3,T,H,W) float32 video after the CLI's transpose (motion_segment.py:96), not normalised."""
    return np.ascontiguousarray(echo_video_uint8(T, H, W, seed, period).transpose(3, 0, 1, 2), dtype=np.float32)


def echonet_like_lengths(n, seed=2024, lo=100, hi=300):
    """Seeded ragged video lengths in [lo, hi] frames (EchoNet-Dynamic clips run ~100-300 frames at
    50 fps): the config[2] batch with lengths that make videos straddle the ranks' clip blocks, so the
    owner exchange (dist.exchange_to_owners) moves logit margins over RCCL."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return [int(t) for t in rng.integers(lo, hi + 1, size=n)]

"""ORACLE (test infrastructure only -- never imported by the product path).

CPU restatement of the CLAS-FV model forward, op-for-op as the reference writes it:

* backbone = torchvision 0.6.0 ``r2plus1d_18`` (VideoResNet / R2Plus1dStem / BasicBlock /
  Conv2Plus1D), called at src/model/R2plus1D_18_MotionNet.py:29-37. torchvision is absent from the
  image, so the definition is restated here (pinned by the parameter count 31,575,731 printed in
  …CLAS_FV_train_test.ipynb:180 and by tests/golden fixtures produced by the reference's own
  ``R2plus1D_18_MotionNet`` module).
* head = five trilinear ``align_corners=True`` upsamplings (:41-49), ``torch.cat`` (:52), 1x1x1 conv
  1024->64 + BN + ReLU (:55-57), 64->64 + BN + ReLU (:59-62), seg head (:65), motion head + tanh
  (:68-69) -- the as-written graph, including the 1.6 GB concat at 32x112x112.

Runs on torch CPU in fp32; also used as the CPU baseline ("port") in bench.py.
"""
import torch
import torch.nn.functional as F

_EPS = 1e-5


def _t(sd, name):
    v = sd[name]
    if not torch.is_tensor(v):
        v = torch.from_numpy(v)
    return v


def _conv_bn(sd, x, conv, bn, stride, pad, relu=True):
    x = F.conv3d(x, _t(sd, conv + ".weight"), None, stride, pad)
    x = F.batch_norm(x, _t(sd, bn + ".running_mean"), _t(sd, bn + ".running_var"), _t(sd, bn + ".weight"),
                     _t(sd, bn + ".bias"), False, 0.0, _EPS)
    return F.relu(x) if relu else x


def _block(sd, x, pre, stride, has_ds):
    # conv1 = Sequential(Conv2Plus1D(i, o, mid, stride), BN, ReLU)
    h = _conv_bn(sd, x, pre + "conv1.0.0", pre + "conv1.0.1", (1, stride, stride), (0, 1, 1))
    h = _conv_bn(sd, h, pre + "conv1.0.3", pre + "conv1.1", (stride, 1, 1), (1, 0, 0))
    # conv2 = Sequential(Conv2Plus1D(o, o, mid), BN)
    h = _conv_bn(sd, h, pre + "conv2.0.0", pre + "conv2.0.1", (1, 1, 1), (0, 1, 1))
    h = _conv_bn(sd, h, pre + "conv2.0.3", pre + "conv2.1", (1, 1, 1), (1, 0, 0), relu=False)
    res = _conv_bn(sd, x, pre + "downsample.0", pre + "downsample.1", (stride,) * 3, (0, 0, 0),
                   relu=False) if has_ds else x
    return F.relu(h + res)


def backbone(sd, x):
    """Returns the five decoder taps (stem, layer1, layer2, layer3, layer4)."""
    R = "r2plus1d_model."
    s = _conv_bn(sd, x, R + "stem.0", R + "stem.1", (1, 2, 2), (0, 3, 3))
    s = _conv_bn(sd, s, R + "stem.3", R + "stem.4", (1, 1, 1), (1, 0, 0))
    taps = [s]
    h = s
    for li, stride in enumerate([1, 2, 2, 2], start=1):
        h = _block(sd, h, f"{R}layer{li}.0.", stride, has_ds=(li > 1))
        h = _block(sd, h, f"{R}layer{li}.1.", 1, has_ds=False)
        taps.append(h)
    return taps


def head(sd, taps):
    scales = [(1, 2, 2), (1, 2, 2), (2, 4, 4), (4, 8, 8), (8, 16, 16)]
    ups = [F.interpolate(t, scale_factor=list(s), mode="trilinear", align_corners=True) for t, s in zip(taps, scales)]
    cat = torch.cat(ups, 1)
    h = F.conv3d(cat, _t(sd, "comb_1_layer.weight"), _t(sd, "comb_1_layer.bias"))
    del cat, ups
    h = F.relu(F.batch_norm(h, _t(sd, "comb_batch_norm_1.running_mean"), _t(sd, "comb_batch_norm_1.running_var"),
                            _t(sd, "comb_batch_norm_1.weight"), _t(sd, "comb_batch_norm_1.bias"), False, 0.0, _EPS))
    h = F.conv3d(h, _t(sd, "comb_2_layer.weight"), _t(sd, "comb_2_layer.bias"))
    h = F.relu(F.batch_norm(h, _t(sd, "comb_batch_norm_2.running_mean"), _t(sd, "comb_batch_norm_2.running_var"),
                            _t(sd, "comb_batch_norm_2.weight"), _t(sd, "comb_batch_norm_2.bias"), False, 0.0, _EPS))
    seg = F.conv3d(h, _t(sd, "segmentation_head.weight"), _t(sd, "segmentation_head.bias"))
    mot = torch.tanh(F.conv3d(h, _t(sd, "motion_head.weight"), _t(sd, "motion_head.bias")))
    return seg, mot


def _lerp_frames(t, t_out):
    """align_corners=True linear resampling of dim 2 to t_out frames."""
    t_in = t.shape[2]
    if t_in == t_out:
        return t
    scale = (t_in - 1) / (t_out - 1) if t_out > 1 else 0.0
    idx = torch.arange(t_out, dtype=torch.float32) * torch.tensor(scale, dtype=torch.float32)
    i0 = torch.clamp(idx.floor().long(), max=t_in - 1)
    lam = (idx - i0.float()).clamp(0, 1)
    i1 = torch.clamp(i0 + 1, max=t_in - 1)
    lam = lam.view(1, 1, -1, 1, 1)
    return t[:, :, i0] * (1 - lam) + t[:, :, i1] * lam


@torch.no_grad()
def forward_chunked(sd, x, frames_per_chunk=4):
    """Same function as ``forward`` for large clips (e.g. BASELINE config[3], 64x224x224, whose
    as-written concat is 13 GB): the five trilinear align_corners=True upsamplings are evaluated
    separably (time, then F.interpolate bilinear over H, W) for a few output frames at a time and
    the 1x1x1 head is applied per chunk. Equal to ``forward`` up to fp32 rounding."""
    if not torch.is_tensor(x):
        x = torch.from_numpy(x)
    x = x.float()
    taps = backbone(sd, x)
    n, _, t, h, w = x.shape
    segs, mots = [], []
    for t0 in range(0, t, frames_per_chunk):
        t1 = min(t, t0 + frames_per_chunk)
        ups = []
        for tap in taps:
            lt = _lerp_frames(tap, t)[:, :, t0:t1]
            c, k = lt.shape[1], lt.shape[2]
            sp = F.interpolate(lt.permute(0, 2, 1, 3, 4).reshape(n * k, c, lt.shape[3], lt.shape[4]), size=(h, w),
                               mode="bilinear", align_corners=True)
            ups.append(sp.reshape(n, k, c, h, w).permute(0, 2, 1, 3, 4))
        s_, m_ = head_from_cat(sd, torch.cat(ups, 1))
        segs.append(s_)
        mots.append(m_)
    return torch.cat(segs, 2), torch.cat(mots, 2)


def head_from_cat(sd, cat):
    h = F.conv3d(cat, _t(sd, "comb_1_layer.weight"), _t(sd, "comb_1_layer.bias"))
    h = F.relu(F.batch_norm(h, _t(sd, "comb_batch_norm_1.running_mean"), _t(sd, "comb_batch_norm_1.running_var"),
                            _t(sd, "comb_batch_norm_1.weight"), _t(sd, "comb_batch_norm_1.bias"), False, 0.0, _EPS))
    h = F.conv3d(h, _t(sd, "comb_2_layer.weight"), _t(sd, "comb_2_layer.bias"))
    h = F.relu(F.batch_norm(h, _t(sd, "comb_batch_norm_2.running_mean"), _t(sd, "comb_batch_norm_2.running_var"),
                            _t(sd, "comb_batch_norm_2.weight"), _t(sd, "comb_batch_norm_2.bias"), False, 0.0, _EPS))
    seg = F.conv3d(h, _t(sd, "segmentation_head.weight"), _t(sd, "segmentation_head.bias"))
    mot = torch.tanh(F.conv3d(h, _t(sd, "motion_head.weight"), _t(sd, "motion_head.bias")))
    return seg, mot


@torch.no_grad()
def forward(sd, x):
    """x: (N,3,T,H,W) float32 CPU tensor -> (seg_logits (N,2,T,H,W), motion (N,4,T,H,W))."""
    if not torch.is_tensor(x):
        x = torch.from_numpy(x)
    return head(sd, backbone(sd, x.float()))


class OracleModel:
    """Callable with the reference model's signature: model(clip) -> (seg, motion)."""

    def __init__(self, sd):
        self.sd = {k: _t(sd, k) for k in sd}
        self.calls = 0

    def __call__(self, x):
        self.calls += 1
        return forward(self.sd, x)

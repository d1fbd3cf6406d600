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

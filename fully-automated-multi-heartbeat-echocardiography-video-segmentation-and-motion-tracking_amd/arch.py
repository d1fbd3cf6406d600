"""Architecture of ``R2plus1D_18_MotionNet`` as data.

The reference builds the network from torchvision 0.6.0 ``r2plus1d_18`` (stem + layer1..4) plus the
CLAS-FV decoder head (``src/model/R2plus1D_18_MotionNet.py:11-24``). torchvision is not a dependency
here: this module restates the layer table once so that the synthetic-weight generator, the
checkpoint loader and the native library all agree on names, shapes and order.

State-dict names are the reference's own (``r2plus1d_model.stem.0.weight`` ... ``segmentation_head.bias``);
a ``module.`` prefix (``nn.DataParallel``, ``motion_segment.py:69``) is accepted by the loaders.
"""
from collections import OrderedDict

NUM_PARAMS_REFERENCE = 31_575_731  # printed by every reference notebook (…CLAS_FV_train_test.ipynb:180)


def midplanes(inplanes, planes):
    """torchvision 0.6.0 BasicBlock: mid = (i*o*3*3*3) // (i*3*3 + 3*o)."""
    return (inplanes * planes * 27) // (inplanes * 9 + 3 * planes)


class Conv:
    """One bias-free Conv3d of the backbone followed by BatchNorm3d (eval)."""

    def __init__(self, name, bn, cin, cout, k, s, p):
        self.name, self.bn = name, bn
        self.cin, self.cout = cin, cout
        self.k, self.s, self.p = tuple(k), tuple(s), tuple(p)

    def __repr__(self):
        return f"Conv({self.name}, {self.cin}->{self.cout}, k={self.k}, s={self.s}, p={self.p})"


def backbone_convs():
    """Ordered list of the 41 backbone convolutions (stem, 8 blocks, 3 downsamples).

    Returns list of (role, Conv) with role in {stem_s, stem_t, sp1, tp1, sp2, tp2, ds}; block
    boundaries are marked by role prefix order.
    """
    R = "r2plus1d_model."
    out = []
    out.append(("stem_s", Conv(R + "stem.0", R + "stem.1", 3, 45, (1, 7, 7), (1, 2, 2), (0, 3, 3))))
    out.append(("stem_t", Conv(R + "stem.3", R + "stem.4", 45, 64, (3, 1, 1), (1, 1, 1), (1, 0, 0))))
    inplanes = 64
    for li, (planes, stride) in enumerate([(64, 1), (128, 2), (256, 2), (512, 2)], start=1):
        for b in range(2):
            st = stride if b == 0 else 1
            mid = midplanes(inplanes if b == 0 else planes, planes)
            pre = f"{R}layer{li}.{b}."
            cin1 = inplanes if b == 0 else planes
            out.append(("sp1", Conv(pre + "conv1.0.0", pre + "conv1.0.1", cin1, mid, (1, 3, 3), (1, st, st), (0, 1, 1))))
            out.append(("tp1", Conv(pre + "conv1.0.3", pre + "conv1.1", mid, planes, (3, 1, 1), (st, 1, 1), (1, 0, 0))))
            out.append(("sp2", Conv(pre + "conv2.0.0", pre + "conv2.0.1", planes, mid, (1, 3, 3), (1, 1, 1), (0, 1, 1))))
            out.append(("tp2", Conv(pre + "conv2.0.3", pre + "conv2.1", mid, planes, (3, 1, 1), (1, 1, 1), (1, 0, 0))))
            if b == 0 and (stride != 1 or inplanes != planes):
                out.append(("ds", Conv(pre + "downsample.0", pre + "downsample.1", inplanes, planes, (1, 1, 1),
                                       (stride, stride, stride), (0, 0, 0))))
        inplanes = planes
    return out


def _bn_entries(prefix, c):
    return [(prefix + ".weight", (c,)), (prefix + ".bias", (c,)), (prefix + ".running_mean", (c,)),
            (prefix + ".running_var", (c,)), (prefix + ".num_batches_tracked", ())]


def state_dict_spec():
    """OrderedDict name -> shape in the reference module's registration order (242 entries)."""
    spec = OrderedDict()
    R = "r2plus1d_model."
    convs = backbone_convs()
    # registration order inside a BasicBlock: conv1 (0.0, 0.1, 0.3, 1), conv2 (...), downsample
    # -- the order produced by backbone_convs() already matches except that downsample comes last
    # within block 0, which it does.
    for role, c in convs:
        spec[c.name + ".weight"] = (c.cout, c.cin) + c.k
        for n, s in _bn_entries(c.bn, c.cout):
            spec[n] = s
    spec[R + "fc.weight"] = (400, 512)
    spec[R + "fc.bias"] = (400,)
    spec["comb_1_layer.weight"] = (64, 1024, 1, 1, 1)
    spec["comb_1_layer.bias"] = (64,)
    for n, s in _bn_entries("comb_batch_norm_1", 64):
        spec[n] = s
    spec["comb_2_layer.weight"] = (64, 64, 1, 1, 1)
    spec["comb_2_layer.bias"] = (64,)
    for n, s in _bn_entries("comb_batch_norm_2", 64):
        spec[n] = s
    spec["motion_head.weight"] = (4, 64, 1, 1, 1)
    spec["motion_head.bias"] = (4,)
    spec["segmentation_head.weight"] = (2, 64, 1, 1, 1)
    spec["segmentation_head.bias"] = (2,)
    return spec


def _reorder_block_entries(spec):
    return spec


def count_parameters(spec=None):
    """Trainable parameter count (excludes BN running stats / num_batches_tracked)."""
    spec = spec or state_dict_spec()
    n = 0
    for name, shape in spec.items():
        if name.endswith(("running_mean", "running_var", "num_batches_tracked")):
            continue
        k = 1
        for d in shape:
            k *= d
        n += k
    return n


def strip_module_prefix(name):
    return name[len("module."):] if name.startswith("module.") else name


# Decoder taps feeding comb_1_layer, in concat order (src/model/R2plus1D_18_MotionNet.py:52):
# (tap name, channels, temporal/spatial downsample factor relative to the input clip)
DECODER_TAPS = [("stem", 64, 1, 2), ("layer1", 64, 1, 2), ("layer2", 128, 2, 4), ("layer3", 256, 4, 8),
                ("layer4", 512, 8, 16)]
BN_EPS = 1e-5

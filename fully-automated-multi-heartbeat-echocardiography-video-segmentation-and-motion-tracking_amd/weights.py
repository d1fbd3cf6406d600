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

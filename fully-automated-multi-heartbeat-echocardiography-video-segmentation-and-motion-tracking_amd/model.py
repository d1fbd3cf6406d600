"""Drop-in ``R2plus1D_18_MotionNet`` backed by the HIP engine (libclasfv.so).

Mirrors src/model/R2plus1D_18_MotionNet.py:10-71: ``forward(x) -> (segmentation_logits, motion)``
with x (N,3,T,H,W) float32, seg (N,2,T,H,W) and motion (N,4,T,H,W) = tanh(...). The state dict has
the reference's 242 keys; ``load_state_dict`` accepts the ``module.``-prefixed keys that
``nn.DataParallel`` checkpoints carry (motion_segment.py:69-72).

Differences, all deliberate:
* ``pretrained=True`` cannot download Kinetics weights offline; the network starts from seeded
  synthetic weights (``weights="random"``: weights.synthetic_state_dict; ``weights="echo"``: the
  recipe whose masks follow the synthetic video's LV, weights.echo_state_dict) and a checkpoint is
  expected to be loaded.
* Inference only: forward runs under no autograd (the reference builds graphs it never uses,
  src/fuse_utils.py:59).
* Any H, W multiple of 16 and T multiple of 8 is accepted (the reference's concat needs the same).
"""
import ctypes
import warnings
from collections import OrderedDict

import numpy as np
import torch
from torch import nn

from . import _lib
from .arch import strip_module_prefix
from .weights import DEFAULT_SEED, recipe_state_dict


class Engine:
    """Owns one clasfv handle (weights + workspace) on one HIP device."""

    def __init__(self, device=None, dtype="fp32"):
        if not torch.cuda.is_available():
            raise RuntimeError("CLAS-FV engine requires a HIP (ROCm) GPU; none is visible")
        self.lib = _lib.load()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        h = ctypes.c_void_p()
        _lib.check(self.lib.clasfv_create(self.device.index, ctypes.byref(h)), "clasfv_create")
        self.h = h
        self.set_dtype(dtype)

    def set_dtype(self, dtype):
        """'fp32' (default, reference precision) or 'bf16' (BASELINE config[4]); re-load weights after."""
        if dtype not in _lib.DTYPES:
            raise ValueError(f"dtype must be one of {sorted(_lib.DTYPES)}")
        _lib.check(self.lib.clasfv_set_compute_dtype(self.h, _lib.DTYPES[dtype]), "clasfv_set_compute_dtype")
        self.dtype = "bf16" if _lib.DTYPES[dtype] == 1 else "fp32"

    def set_variants(self, *names):
        """Kernel variants for A/B tests (CLASFV_VARIANT_*; e.g. "no_winograd"); no names = the
        product kernels. Returns the previous names. Call load() afterwards if no_winograd changed."""
        flags = 0
        for n in names:
            if n not in _lib.VARIANTS:
                raise ValueError(f"unknown kernel variant {n!r}: {sorted(_lib.VARIANTS)}")
            flags |= _lib.VARIANTS[n]
        old = self.lib.clasfv_get_kernel_variants(self.h)
        _lib.check(self.lib.clasfv_set_kernel_variants(self.h, flags), "clasfv_set_kernel_variants")
        return tuple(n for n, b in _lib.VARIANTS.items() if old & b)

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.lib.clasfv_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def param_table(self):
        out = []
        name = ctypes.c_char_p()
        nd = ctypes.c_int()
        dims = (ctypes.c_int64 * 5)()
        for i in range(self.lib.clasfv_param_count(self.h)):
            _lib.check(self.lib.clasfv_param_info(self.h, i, ctypes.byref(name), ctypes.byref(nd), dims), "param_info")
            out.append((name.value.decode(), tuple(int(dims[d]) for d in range(nd.value))))
        return out

    def load(self, state):
        for k, v in state.items():
            a = np.ascontiguousarray(np.asarray(v.detach().cpu() if torch.is_tensor(v) else v), dtype=np.float32)
            _lib.check(self.lib.clasfv_load_param(self.h, k.encode(), a.ctypes.data_as(ctypes.c_void_p), a.size),
                       f"load {k}")
        _lib.check(self.lib.clasfv_finalize(self.h), "clasfv_finalize")

    def forward(self, x, seg, mot, stream=None):
        n, c, t, hh, ww = x.shape
        _lib.check(self.lib.clasfv_forward(self.h, _lib.ptr(x), n, t, hh, ww, _lib.ptr(seg), _lib.ptr(mot),
                                           _lib.stream_ptr(stream, self.device)), "clasfv_forward")

    def set_kernel_timing(self, enable=True):
        """Per-kernel HIP-event timing of every later forward (see clasfv_kernel_timing)."""
        _lib.check(self.lib.clasfv_set_kernel_timing(self.h, 1 if enable else 0), "clasfv_set_kernel_timing")

    def kernel_timing(self, cap=16):
        """{kernel: {"launches", "ms", "gflop", "xgflop"}} over the forwards since the last call (then
        cleared). gflop: algorithmic (direct-conv MACs x 2); xgflop: MFMA work actually issued."""
        names = (ctypes.c_char_p * cap)()
        launches = (ctypes.c_int * cap)()
        ms = (ctypes.c_double * cap)()
        gf = (ctypes.c_double * cap)()
        xg = (ctypes.c_double * cap)()
        n = self.lib.clasfv_kernel_timing(self.h, cap, names, launches, ms, gf, xg)
        if n < 0:
            _lib.check(n, "clasfv_kernel_timing")
        return {names[i].decode(): {"launches": int(launches[i]), "ms": float(ms[i]), "gflop": float(gf[i]),
                                    "xgflop": float(xg[i])} for i in range(n)}

    def workspace_bytes(self):
        return int(self.lib.clasfv_workspace_bytes(self.h))


class R2plus1D_18_MotionNet(nn.Module):
    """HIP-backed drop-in for the reference model (inference)."""

    def __init__(self, pretrained=True, output_channels=4, device=None, seed=DEFAULT_SEED, dtype="fp32",
                 weights="random"):
        super().__init__()
        if output_channels != 4:
            raise ValueError("the motion head has 4 channels [fwd x, fwd y, bwd x, bwd y]")
        if pretrained:
            warnings.warn("pretrained=True: Kinetics weights cannot be downloaded offline; using seeded synthetic "
                          "weights (load a checkpoint with load_state_dict)", stacklevel=2)
        self.engine = Engine(device, dtype)
        self._state = OrderedDict()
        self._params = None
        self._load(recipe_state_dict(weights, seed))

    def set_kernel_variants(self, *names):
        """A/B-test kernel variants (see Engine.set_variants); weights are re-uploaded so the
        choice of Winograd or direct weight images follows. Returns the previous variant names."""
        old = self.engine.set_variants(*names)
        self.engine.load(self._state)
        return old

    def set_compute_dtype(self, dtype):
        """Switch the encoder between exact fp32 and bf16 (fp32 accumulation) and re-upload weights."""
        self.engine.set_dtype(dtype)
        self.engine.load(self._state)
        return self

    # ---- state dict ------------------------------------------------------------------------------
    def _load(self, sd):
        table = self.engine.param_table()
        state = OrderedDict()
        for name, shape in table:
            if name not in sd:
                raise KeyError(f"missing key in state_dict: {name}")
            v = sd[name]
            t = v.detach().cpu() if torch.is_tensor(v) else torch.from_numpy(np.asarray(v))
            if tuple(t.shape) != shape:
                raise RuntimeError(f"size mismatch for {name}: {tuple(t.shape)} vs {shape}")
            state[name] = t.clone()
        self.engine.load(state)
        self._state = state
        self._params = None

    def load_state_dict(self, state_dict, strict=True):
        sd = OrderedDict((strip_module_prefix(k), v) for k, v in state_dict.items())
        expected = {n for n, _ in self.engine.param_table()}
        unexpected = [k for k in sd if k not in expected]
        missing = [k for k in expected if k not in sd]
        if strict and (unexpected or missing):
            raise RuntimeError(f"Error(s) in loading state_dict: missing={missing[:5]} unexpected={unexpected[:5]}")
        merged = OrderedDict(self._state)
        merged.update({k: v for k, v in sd.items() if k in expected})
        self._load(merged)
        return nn.modules.module._IncompatibleKeys(missing, unexpected)

    def state_dict(self, *args, **kwargs):
        return OrderedDict((k, v.clone()) for k, v in self._state.items())

    def parameters(self, recurse=True):
        if self._params is None:
            self._params = [nn.Parameter(v.float(), requires_grad=True) for k, v in self._state.items()
                            if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]
        return iter(self._params)

    # ---- forward ---------------------------------------------------------------------------------
    @torch.no_grad()
    def forward(self, x):
        x = torch.as_tensor(x)
        if x.dim() != 5 or x.shape[1] != 3:
            raise ValueError(f"expected (N,3,T,H,W), got {tuple(x.shape)}")
        x = x.to(self.engine.device, torch.float32).contiguous()
        n, _, t, h, w = x.shape
        seg = torch.empty((n, 2, t, h, w), device=x.device, dtype=torch.float32)
        mot = torch.empty((n, 4, t, h, w), device=x.device, dtype=torch.float32)
        self.engine.forward(x, seg, mot)
        return seg, mot

"""ctypes binding of ``libclasfv.so`` (C ABI declared in include/clasfv.h).

There is no CPU fallback: if the library is missing or a call fails, a RuntimeError is raised.
"""
import ctypes
import os

from .build import LIB_PATH

c_int, c_int64, c_void_p, c_char_p = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_char_p
_P = c_void_p

# name -> (restype, argtypes); mirrors include/clasfv.h
SIGNATURES = {
    "clasfv_last_error": (c_char_p, []),
    "clasfv_version": (c_int, []),
    "clasfv_source_hash": (c_char_p, []),
    "clasfv_create": (c_int, [c_int, ctypes.POINTER(c_void_p)]),
    "clasfv_destroy": (c_int, [_P]),
    "clasfv_param_count": (c_int, [_P]),
    "clasfv_param_info": (c_int, [_P, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int), ctypes.POINTER(c_int64)]),
    "clasfv_load_param": (c_int, [_P, c_char_p, _P, c_int64]),
    "clasfv_finalize": (c_int, [_P]),
    "clasfv_forward": (c_int, [_P, _P, c_int, c_int, c_int, c_int, _P, _P, _P]),
    "clasfv_workspace_bytes": (c_int64, [_P]),
    "clasfv_set_compute_dtype": (c_int, [_P, c_int]),
    "clasfv_get_compute_dtype": (c_int, [_P]),
    "clasfv_set_kernel_variants": (c_int, [_P, c_int]),
    "clasfv_get_kernel_variants": (c_int, [_P]),
    "clasfv_set_kernel_timing": (c_int, [_P, c_int]),
    "clasfv_kernel_timing": (c_int, [_P, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int),
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]),
    "clasfv_build_clips": (c_int, [_P, c_int, c_int, c_int, _P, c_int, c_int, _P, _P]),
    "clasfv_pass_labels": (c_int, [_P, c_int, _P, c_int, c_int, c_int, c_int, c_int, _P, _P]),
    "clasfv_pass_labels_margin": (c_int, [_P, c_int, _P, c_int, c_int, c_int, c_int, c_int, _P, _P]),
    "clasfv_logit_margin": (c_int, [_P, c_int, c_int, c_int, _P, _P]),
    "clasfv_fuse_votes": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, _P, _P]),
    "clasfv_warp": (c_int, [_P, c_int, c_int, c_int, c_int, _P, c_int64, c_int64, _P, _P]),
    "clasfv_zeroone_workspace_bytes": (c_int64, []),
    "clasfv_zeroone_normalize": (c_int, [_P, c_int64, _P, _P]),
    "clasfv_warp_backward": (c_int, [_P, _P, c_int, c_int, c_int, c_int, _P, c_int64, c_int64, _P, _P, _P]),
    "clasfv_preprocess_video": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, _P, _P]),
}

ABI_VERSION = 3  # CLASFV_ABI_VERSION of include/clasfv.h these signatures describe
FUSE_MAJORITY, FUSE_SIMPLE, FUSE_STAPLE, FUSE_ITKVOTING = 0, 1, 2, 3
FUSE_FORCE_GENERIC = 0x100
# CLASFV_VARIANT_* bits (include/clasfv.h)
VARIANTS = {"no_winograd": 1, "no_wino_patch": 2, "winot_reference": 4, "no_c8": 8, "no_stem_bf16": 16,
            "no_patch_bf16": 32, "no_decoder_bf16": 64, "winot_no_ts1": 128, "no_split_k": 256, "no_wino4": 512,
            "no_decoder_x3": 1024, "no_dma_x3": 2048, "no_stem_x3": 4096, "no_wino4w": 8192,
            "no_patch32": 16384, "no_proj_x3": 32768, "no_wino4r": 65536,
            "no_dma_buf": 262144, "w4r_cached_stores": 524288,
            "patch32_cached_stores": 4194304, "no_dma_w": 16777216, "no_twalk": 67108864}
DTYPES = {"fp32": 0, "float32": 0, "bf16": 1, "bfloat16": 1}
_lib = None


def lib_path():
    return LIB_PATH


def load():
    """Load and return the ctypes library. A library whose embedded source hash differs from the
    sources on disk (older than them, or built from other ones) is rebuilt before it is loaded --
    never used stale; without hipcc that rebuild raises."""
    global _lib
    if _lib is not None:
        return _lib
    from . import build as B
    want = B.source_hash()
    have = B.library_hash()
    if have != want:
        import sys
        print(f"clasfv: {LIB_PATH} {'missing' if have is None and not os.path.exists(LIB_PATH) else 'stale'} "
              f"(library source hash {have}, sources {want}): rebuilding", file=sys.stderr)
        # not forced: build() re-checks the hash under its lock, so ranks that waited for another
        # rank's rebuild reuse it instead of compiling again
        B.build()
        if B.library_hash() != want:
            raise RuntimeError(f"{LIB_PATH}: rebuild did not produce a library of the current sources")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.clasfv_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI version {lib.clasfv_version()}, expected {ABI_VERSION}: rebuild it "
                           f"(python -m clasfv_amd.build --force)")
    got = lib.clasfv_source_hash().decode()
    if got != B.HASH_MARK.decode() + want:
        raise RuntimeError(f"{LIB_PATH}: loaded library reports {got}, sources hash to {want}")
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != 0:
        msg = load().clasfv_last_error()
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


def stream_ptr(stream=None, device=None):
    """hipStream_t of ``stream``, else the current stream of ``device`` (a tensor's device: the
    stream the caller's work on that device is ordered on), else of the current device."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())

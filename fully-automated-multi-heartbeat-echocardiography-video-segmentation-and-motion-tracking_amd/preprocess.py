"""Video preprocessing on the device.

``preprocess_video`` (motion_segment.py:96-106 + src/echonet_dataset.py:38-50): (T,H,W,3) uint8 RGB
frames -> (3,T,H,W) float32 -> trilinear align_corners=True resize to (T,height,width) -> zero-one
normalisation, all in HBM (``clasfv_preprocess_video`` + ``clasfv_zeroone_normalize``). Only the
uint8 frames cross PCIe (from pinned host memory), a quarter of the float video's bytes.

``zeroone_normalizer`` (src/echonet_dataset.py:38-50): per colour channel subtract the channel
minimum over the whole video, then divide by the maximum of the result; float32, as the reference's
in-place numpy ops (bit-exact: subtraction and division are correctly rounded on both sides).
"""
import numpy as np
import torch

from . import _lib


def zeroone_normalize_(video):
    """In place on a (3, ...) float32 contiguous device tensor; returns it."""
    if video.shape[0] != 3 or video.dtype != torch.float32 or not video.is_contiguous():
        raise ValueError("expected a contiguous float32 (3, ...) tensor")
    lib = _lib.load()
    # scratch for the per-block min/max partials, stream-ordered by the caching allocator
    ws = torch.empty(int(lib.clasfv_zeroone_workspace_bytes()) // 4, device=video.device, dtype=torch.float32)
    _lib.check(lib.clasfv_zeroone_normalize(_lib.ptr(video), video[0].numel(), _lib.ptr(ws),
                                            _lib.stream_ptr(device=video.device)), "clasfv_zeroone_normalize")
    return video


def zeroone_normalizer(image_data):
    """Drop-in for the reference function: numpy in -> numpy out (normalised in place, like the
    reference's ``-=``/``/=``); a device tensor is normalised in place on the device."""
    if torch.is_tensor(image_data):
        return zeroone_normalize_(image_data)
    arr = np.asarray(image_data)
    dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32)).to(dev)
    zeroone_normalize_(t)
    out = t.cpu().numpy()
    if isinstance(image_data, np.ndarray) and image_data.dtype == np.float32 and image_data.flags.writeable:
        image_data[...] = out.reshape(image_data.shape)
        return image_data
    return out.reshape(arr.shape)


def preprocess_video(frames, height=112, width=112, device=None, normalize=True):
    """(T,Hs,Ws,3) uint8 RGB frames (numpy array or uint8 tensor, host or device) -> normalised
    (3,T,height,width) float32 device tensor, as the reference CLI's cv2 frames -> F.interpolate ->
    zeroone_normalizer sequence (motion_segment.py:96-106)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if torch.is_tensor(frames):
        f = frames
    else:
        f = torch.from_numpy(np.ascontiguousarray(frames))
        if f.dtype == torch.uint8:
            f = f.pin_memory()
    if f.dim() != 4 or f.shape[-1] != 3 or f.dtype != torch.uint8:
        raise ValueError(f"expected (T,H,W,3) uint8 frames, got {tuple(f.shape)} {f.dtype}")
    f = f.to(dev, non_blocking=True).contiguous()
    t, hs, ws, _ = f.shape
    out = torch.empty((3, t, height, width), device=dev, dtype=torch.float32)
    lib = _lib.load()
    _lib.check(lib.clasfv_preprocess_video(_lib.ptr(f), t, hs, ws, height, width, _lib.ptr(out),
                                           _lib.stream_ptr(device=dev)), "clasfv_preprocess_video")
    return zeroone_normalize_(out) if normalize else out

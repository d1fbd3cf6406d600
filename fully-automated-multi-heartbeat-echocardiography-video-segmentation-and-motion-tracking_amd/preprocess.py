"""Video preprocessing on the device.

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
    _lib.check(lib.clasfv_zeroone_normalize(_lib.ptr(video), video[0].numel(), _lib.stream_ptr()),
               "clasfv_zeroone_normalize")
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

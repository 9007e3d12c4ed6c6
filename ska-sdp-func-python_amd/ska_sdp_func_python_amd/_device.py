"""Host <-> device plumbing for the reference-shaped API (torch tensors on HIP)."""

import numpy as np
import torch

from . import _lib


def device():
    """The HIP device for this process (LOCAL_RANK-aware); raises without a GPU."""
    if not torch.cuda.is_available():
        raise _lib.HipLibraryError(
            "no HIP device visible: the ska_sdp_func_python_amd compute path runs only on "
            "MI355X (there is no CPU fallback)")
    _lib.load()
    return torch.device("cuda", torch.cuda.current_device())


def is_device(a):
    return isinstance(a, torch.Tensor) and a.is_cuda


def to_dev(a, dtype=None, dev=None):
    """numpy / torch -> device tensor (no copy when already there and typed)."""
    dev = dev or device()
    if isinstance(a, torch.Tensor):
        t = a.to(dev)
    else:
        t = torch.as_tensor(np.ascontiguousarray(np.asarray(a)), device=dev)
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t


def like_input(result, reference):
    """Return ``result`` on the host unless ``reference`` lives on the device."""
    if is_device(reference):
        return result
    return result.detach().cpu().numpy()

"""Array plumbing between Python callers and the C-ABI.

numpy arrays / lists -> JW_HOST (the library stages through HBM and synchronises);
torch tensors on a HIP device -> JW_DEVICE on torch's current stream (no copies).
"""
import ctypes

import numpy as np

from . import _native


class Arr:
    __slots__ = ("obj", "device", "torch_cpu")

    def __init__(self, obj, device, torch_cpu=False):
        self.obj = obj
        self.device = device
        self.torch_cpu = torch_cpu

    @property
    def shape(self):
        return tuple(self.obj.shape)

    @property
    def ptr(self):
        if self.device:
            return ctypes.c_void_p(self.obj.data_ptr())
        return ctypes.c_void_p(self.obj.ctypes.data)

    @property
    def where(self):
        return _native.JW_DEVICE if self.device else _native.JW_HOST

    @property
    def stream(self):
        if not self.device:
            return None
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(self.obj.device).cuda_stream)

    def empty(self, shape):
        if self.device:
            import torch
            return Arr(torch.empty(shape, dtype=torch.float64, device=self.obj.device), True)
        return Arr(np.empty(shape, dtype=np.float64), False, self.torch_cpu)

    def result(self):
        if self.torch_cpu:
            import torch
            return torch.from_numpy(self.obj)
        return self.obj


def _is_torch(a):
    return type(a).__module__.startswith("torch")


def as_input(a):
    if _is_torch(a):
        import torch
        if a.device.type == "cuda":
            return Arr(a.detach().to(torch.float64).contiguous(), True)
        return Arr(np.ascontiguousarray(a.detach().cpu().numpy(), dtype=np.float64), False, True)
    return Arr(np.ascontiguousarray(np.asarray(a, dtype=np.float64)), False)

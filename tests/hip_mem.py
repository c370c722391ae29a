"""Minimal device-memory helper over the HIP runtime librps already loaded (test-only; no
torch in GPU test processes, so there is exactly one HIP runtime)."""
import ctypes

import numpy as np

_hip = None


def hip():
    global _hip
    if _hip is None:
        import rps_amd

        rps_amd.lib()  # loads libamdhip64.so.7 first
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        _hip.hipFree.argtypes = [ctypes.c_void_p]
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipDeviceSynchronize.argtypes = []
    return _hip


def copy_d2d(dst, src, nbytes):
    """hipMemcpy device -> device (raw pointers as ints)."""
    assert hip().hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, 3) == 0


def copy_h2d(dst, host: np.ndarray):
    """hipMemcpy host -> device of a contiguous numpy array (dst: raw device pointer)."""
    host = np.ascontiguousarray(host)
    assert hip().hipMemcpy(ctypes.c_void_p(dst), host.ctypes.data_as(ctypes.c_void_p), host.nbytes, 1) == 0


class DeviceBuffer:
    def __init__(self, nbytes):
        self.ptr = ctypes.c_void_p()
        assert hip().hipMalloc(ctypes.byref(self.ptr), nbytes) == 0
        self.nbytes = nbytes

    def to_host(self, dtype):
        out = np.empty(self.nbytes // np.dtype(dtype).itemsize, dtype=dtype)
        assert hip().hipDeviceSynchronize() == 0
        assert hip().hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), self.ptr, self.nbytes, 2) == 0  # D2H
        return out

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        hip().hipFree(self.ptr)

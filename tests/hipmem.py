"""Device buffers for GPU tests through the HIP runtime libtbg.so links (ctypes; no torch: a
second HIP runtime in the process -- torch's bundled one -- fails to initialise once libtbg's
has)."""
import ctypes

import numpy as np


class Hip:
    def __init__(self, device=0):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        self.hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_int]
        self.hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        self.hip.hipFree.argtypes = [ctypes.c_void_p]
        self.hip.hipSetDevice.argtypes = [ctypes.c_int]
        assert self.hip.hipSetDevice(device) == 0
        self.ptrs = []

    def upload(self, a: np.ndarray) -> int:
        a = np.ascontiguousarray(a)
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), max(a.nbytes, 16)) == 0, "hipMalloc"
        assert self.hip.hipMemcpy(p, a.ctypes.data_as(ctypes.c_void_p), a.nbytes, 1) == 0
        self.ptrs.append(p)
        return p.value

    def zeros(self, nbytes) -> int:
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), max(nbytes, 16)) == 0, "hipMalloc"
        assert self.hip.hipMemset(p, 0, max(nbytes, 16)) == 0
        self.ptrs.append(p)
        return p.value

    def download(self, ptr: int, a: np.ndarray) -> np.ndarray:
        assert self.hip.hipMemcpy(a.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr),
                                  a.nbytes, 2) == 0
        return a

    def free_all(self):
        for p in self.ptrs:
            self.hip.hipFree(p)
        self.ptrs = []

"""In-place batched complex64 transforms through hipFFT (plumbing for fdutils.HannConvolution).

torch.fft copies its input before every rocFFT call on this build (an out-of-place plan may
overwrite it), which cost the windowed likelihood two full passes over its [rows][m] complex64
buffer per transform pair; an in-place plan needs neither the copy nor a second buffer. The
library is the one torch itself loaded (torch/lib/libhipfft.so), so there is one rocFFT in the
process. Plans are made per (m, rows) by the caller, which bounds how many it keeps.
"""

import ctypes
import os

HIPFFT_C2C = 0x29
FORWARD = -1
BACKWARD = 1

_LIB = None


def _load():
    global _LIB
    if _LIB is None:
        import torch
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libhipfft.so")
        lib = ctypes.CDLL(path)
        vp, ip, i = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int
        lib.hipfftPlanMany.restype = i
        lib.hipfftPlanMany.argtypes = [ctypes.POINTER(vp), i, ip, ip, i, i, ip, i, i, i, i]
        lib.hipfftSetStream.restype = i
        lib.hipfftSetStream.argtypes = [vp, vp]
        lib.hipfftExecC2C.restype = i
        lib.hipfftExecC2C.argtypes = [vp, vp, vp, i]
        lib.hipfftDestroy.restype = i
        lib.hipfftDestroy.argtypes = [vp]
        _LIB = lib
    return _LIB


class C2CPlan:
    """rows transforms of m complex64 points each, contiguous rows, in place."""

    def __init__(self, m, rows):
        self.m, self.rows = int(m), int(rows)
        lib = _load()
        h = ctypes.c_void_p()
        n = (ctypes.c_int * 1)(self.m)
        rc = lib.hipfftPlanMany(ctypes.byref(h), 1, n, None, 1, self.m, None, 1, self.m,
                                HIPFFT_C2C, self.rows)
        if rc != 0:
            raise RuntimeError(f"hipfftPlanMany(m={self.m}, rows={self.rows}) failed: {rc}")
        self._h = h
        self._lib = lib

    def __call__(self, ptr, direction, stream):
        """Transform the rows at device address ptr in place on stream (a hipStream_t)."""
        lib = self._lib
        rc = lib.hipfftSetStream(self._h, stream)
        if rc == 0:
            rc = lib.hipfftExecC2C(self._h, ptr, ptr, direction)
        if rc != 0:
            raise RuntimeError(f"hipfftExecC2C(m={self.m}, rows={self.rows}) failed: {rc}")

    def destroy(self):
        """Release the plan (and its work buffer) once the device has finished the transforms
        already queued with it."""
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            import torch
            torch.cuda.synchronize()
            self._lib.hipfftDestroy(h)
            self._h = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.hipfftDestroy(h)
            except Exception:
                pass
            self._h = None

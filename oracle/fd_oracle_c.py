"""ctypes wrapper of the oracle's C restatement (fd_oracle_c.c) -- TEST INFRASTRUCTURE ONLY.

Used by tests/ (checked against fd_oracle.py) and by bench.py's cpu_baseline leg.
"""

import ctypes
import os

import numpy as np

from . import build as _build

_lib = None


def load():
    """Load (building if needed) liboracle; returns None if it cannot be built."""
    global _lib
    if _lib is not None:
        return _lib
    path = _build.OUT
    if not os.path.exists(path):
        try:
            path = _build.build()
        except Exception:
            return None
    if path is None or not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    lib.fdo_modesum.restype = ctypes.c_int
    lib.fdo_modesum.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int,
                                vp, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                ctypes.c_int, ctypes.c_int, vp]
    _lib = lib
    return lib


def modesum(t, amps, phi_phi, phi_r, f_phi, f_r, m, n, ylm_p, ylm_m, freq, prefactor=1.0,
            caustic="uniform", nthreads=0):
    """Same contract as fd_oracle.fd_modesum (amps complex [K, N_t])."""
    lib = load()
    if lib is None:
        raise RuntimeError("oracle C library unavailable (gcc build failed)")
    c = lambda x, dt: np.ascontiguousarray(x, dtype=dt)  # noqa: E731
    t, phi_phi, phi_r, f_phi, f_r, freq = (c(x, np.float64) for x in
                                            (t, phi_phi, phi_r, f_phi, f_r, freq))
    amps = c(amps, np.complex128)
    m, n = c(m, np.int32), c(n, np.int32)
    ylm_p, ylm_m = c(ylm_p, np.complex128), c(ylm_m, np.complex128)
    K, nt = amps.shape
    out = np.zeros(len(freq), dtype=np.complex128)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    sc = complex(prefactor)
    rc = lib.fdo_modesum(p(t), nt, p(amps), p(phi_phi), p(phi_r), p(f_phi), p(f_r), p(m), p(n),
                         p(ylm_p), p(ylm_m), K, p(freq), len(freq), sc.real, sc.imag,
                         1 if caustic == "uniform" else 0, int(nthreads), p(out))
    if rc != 0:
        raise RuntimeError(f"fdo_modesum failed ({rc})")
    return out

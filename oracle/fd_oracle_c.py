"""ctypes wrapper of the oracle's C restatement (fd_oracle_c.c) -- TEST INFRASTRUCTURE ONLY.

Used by tests/ (checked against fd_oracle.py) and by bench.py's cpu_baseline leg.
"""

import ctypes
import os

import numpy as np

from . import build as _build

_libs = {}


def load(variant="exact"):
    """Load (building if needed) liboracle; returns None if it cannot be built.

    variant "exact": the checker (no FMA contraction, as written); "fma": the same source
    compiled with FMA contraction (a second rounding realisation, for conditioning probes)."""
    if variant in _libs:
        return _libs[variant]
    path = _build.OUT if variant == "exact" else _build.OUT_FMA
    if not os.path.exists(path):
        try:
            _build.build()
        except Exception:
            return None
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    lib.fdo_modesum.restype = ctypes.c_int
    lib.fdo_modesum.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int,
                                vp, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                ctypes.c_int, ctypes.c_int, vp]
    lib.fdo_modesum_ex.restype = ctypes.c_int
    lib.fdo_modesum_ex.argtypes = lib.fdo_modesum.argtypes + [vp]
    _libs[variant] = lib
    return lib


def modesum(t, amps, phi_phi, phi_r, f_phi, f_r, m, n, ylm_p, ylm_m, freq, prefactor=1.0,
            caustic="uniform", nthreads=0, variant="exact", extrap=False):
    """Same contract as fd_oracle.fd_modesum (amps complex [K, N_t]). extrap=True also returns
    the per-bin magnitude of the terms whose t(g) is extrapolated outside the trajectory
    (fd_oracle_c.c: fdo_modesum_ex)."""
    lib = load(variant)
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
    E = np.zeros(len(freq)) if extrap else None
    rc = lib.fdo_modesum_ex(p(t), nt, p(amps), p(phi_phi), p(phi_r), p(f_phi), p(f_r), p(m),
                            p(n), p(ylm_p), p(ylm_m), K, p(freq), len(freq), sc.real, sc.imag,
                            1 if caustic == "uniform" else 0, int(nthreads), p(out),
                            p(E) if extrap else None)
    if rc != 0:
        raise RuntimeError(f"fdo_modesum failed ({rc})")
    return (out, E) if extrap else out

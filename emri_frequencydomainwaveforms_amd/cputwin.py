"""Host twin of the FD mode sum (efd_modesum_cpu in libemrifd.so, csrc/emrifd_cpu.cpp).

The same algorithm as the HIP path (grouping, splines, interval records, tile-wise
output-stationary sum with the uniform K_{1/3} fast path) on the CPU with OpenMP: the CPU
baseline of bench.py and a second implementation the HIP kernels are held
to in the parity tests. It is never a fallback of the GPU path: the product classes
(summation.py, waveform.py) only ever call the HIP entry points.
"""

import ctypes

import numpy as np

from . import _lib

CAUSTIC = {"spa": _lib.EFD_CAUSTIC_SPA, "uniform": _lib.EFD_CAUSTIC_UNIFORM}


def _lib_cpu():
    lib = _lib.load()
    if not hasattr(lib, "efd_modesum_cpu"):
        raise _lib.EFDError("libemrifd.so lacks efd_modesum_cpu: rebuild it")
    return lib


def set_threads(n):
    """OpenMP threads of the twins (n <= 0: all); returns the previous setting."""
    return int(_lib_cpu().efd_cpu_threads(int(n)))


def last_error():
    buf = ctypes.create_string_buffer(512)
    _lib_cpu().efd_cpu_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def modesum(t, amp, phi_phi, phi_r, f_phi, f_r, m, n, ylm_p, ylm_m, freq, scale=1.0 + 0.0j,
            caustic="uniform", grid_symmetric=None, out=None, polarizations=False, k0=0,
            accumulate=False):
    """S(freq) (complex128 [nf]) of one waveform on the host; amp complex [nt][K] (FEW layout).

    polarizations=True (symmetric grids) returns (hp, hc) over bins [k0, nf) instead, written
    from the same registers as the kernel's fused h+/hx."""
    lib = _lib_cpu()
    f64 = lambda x: np.ascontiguousarray(x, dtype=np.float64)  # noqa: E731
    c128 = lambda x: np.ascontiguousarray(x, dtype=np.complex128)  # noqa: E731
    i32 = lambda x: np.ascontiguousarray(x, dtype=np.int32)  # noqa: E731
    t, phi_phi, phi_r, f_phi, f_r, freq = (f64(x) for x in (t, phi_phi, phi_r, f_phi, f_r, freq))
    amp, ylm_p, ylm_m = c128(amp), c128(ylm_p), c128(ylm_m)
    m, n = i32(m), i32(n)
    nt, K = amp.shape
    nf = len(freq)
    if grid_symmetric is None:
        grid_symmetric = bool(np.array_equal(freq, -freq[::-1]))
    hp = hc = None
    # (the twin writes every output bin, so a fresh output needs no zeroing unless accumulating)
    new = np.zeros if accumulate else np.empty
    if polarizations:
        hp = new(nf - k0, dtype=np.complex128)
        hc = new(nf - k0, dtype=np.complex128)
        S = None
    else:
        S = out if out is not None else new(nf, dtype=np.complex128)
    p = lambda x: x.ctypes.data if x is not None else None  # noqa: E731
    sc = complex(scale)
    a = _lib.ModesumArgs(
        t=p(t), phi_phi=p(phi_phi), phi_r=p(phi_r), f_phi=p(f_phi), f_r=p(f_r), nt=nt,
        amp=p(amp), m=p(m), n=p(n), ylm_p=p(ylm_p), ylm_m=p(ylm_m), K=K, freq=p(freq), nf=nf,
        grid_symmetric=1 if grid_symmetric else 0, scale_re=sc.real, scale_im=sc.imag,
        caustic=CAUSTIC[caustic], accumulate=1 if accumulate else 0, out=p(S),
        prof_begin=None, prof_end=None, hp=p(hp), hc=p(hc), k0=int(k0))
    rc = lib.efd_modesum_cpu(ctypes.byref(a), None, 0, None)
    if rc != _lib.EFD_OK:
        raise _lib.EFDError(f"efd_modesum_cpu failed ({rc}): {last_error()}")
    return (hp, hc) if polarizations else S


def stats():
    """(contributions C, SPA evaluations, groups) of this thread's last modesum."""
    c, e, g = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
    _lib_cpu().efd_modesum_cpu_stats(ctypes.byref(c), ctypes.byref(e), ctypes.byref(g))
    return int(c.value), int(e.value), int(g.value)


def loglike(h, d, w):
    """efd_loglike_cpu: -1/2 * 4 * sum |d - h w|^2 over [nchan][nbin] host arrays (the host
    twin of efd_loglike, same partition and reduction order)."""
    lib = _lib_cpu()
    h = np.ascontiguousarray(h, dtype=np.complex128)
    d = np.ascontiguousarray(d, dtype=np.complex128)
    w = np.ascontiguousarray(w, dtype=np.float64)
    if h.shape != d.shape or w.shape != d.shape or d.ndim != 2:
        raise ValueError("loglike: h, d, w must share one [nchan][nbin] shape")
    out = np.zeros(1)
    rc = lib.efd_loglike_cpu(h.ctypes.data, d.ctypes.data, w.ctypes.data, d.shape[0],
                             d.shape[1], out.ctypes.data, None, None)
    if rc != _lib.EFD_OK:
        raise _lib.EFDError(f"efd_loglike_cpu failed ({rc}): {last_error()}")
    return float(out[0])

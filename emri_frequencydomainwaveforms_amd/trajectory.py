"""Inspiral trajectory STAND-IN (host side, upstream of the hot path; NOT FEW physics).

The reference builds its inspiral with `EMRIInspiral(func="SchwarzEccFlux")`
(check_mode_by_mode.py:34-35, Tutorial_FD_construction_single_mode.ipynb:45, :122), an adaptive
ODE over Teukolsky-flux interpolants whose data files are absent offline (SURVEY.md section 2,
row 1b: out of scope for HIP). This module keeps that call surface and returns the same
sparse-trajectory tuple ``(t, p, e, x, Phi_phi, Phi_theta, Phi_r)``, but drives it with the
leading-order Peters-Mathews (quadrupole) fluxes in (p, e) and the exact Schwarzschild geodesic
frequencies of `frequencies.py` for the phases. The integration stops 0.1 outside the
separatrix p = 6 + 2e or at T, as FEW's trajectory does.

The hot path only needs *a* smooth sparse trajectory of FEW's shape (N_t ~ 10^2 knots, ~86 per
year in the reference notebook :356); RK45 at rtol = atol = 1e-12 gives ~50-100 knots per year.
`get_p_at_t` mirrors `few.utils.utility.get_p_at_t` as called at check_mode_by_mode.py:200-212.

Two backends with the same equations and integrator: "native" (csrc/emrifd_host.cpp in
libemrifd.so: scipy RK45's Dormand-Prince tableau, step control, dense output and event root
restated in C++, ~1 ms per trajectory, releases the GIL) and "python" (scipy.solve_ivp with the
numpy right-hand side, ~50-100 ms). "auto" takes the native one when the library is built.
"""

import ctypes

import numpy as np
from scipy.integrate import solve_ivp
from scipy.optimize import brentq

from .constants import MTSUN_SI, YRSID_SI
from .frequencies import get_fundamental_frequencies

DIST_TO_SEPARATRIX = 0.1


def _pn_rhs(tau, y, q):
    """d/d tau of (p, e, Phi_phi, Phi_r); tau = t / M in geometric units."""
    p, e = y[0], y[1]
    e2 = e * e
    a = p / (1.0 - e2)
    da = -(64.0 / 5.0) * q / (a ** 3 * (1.0 - e2) ** 3.5) * (1.0 + 73.0 / 24.0 * e2 + 37.0 / 96.0 * e2 * e2)
    de = -(304.0 / 15.0) * q * e / (a ** 4 * (1.0 - e2) ** 2.5) * (1.0 + 121.0 / 304.0 * e2)
    dp = (1.0 - e2) * da - 2.0 * a * e * de
    om_phi, _, om_r = get_fundamental_frequencies(0.0, p, e, 0.0)
    return [dp, de, om_phi, om_r]


def _separatrix_event(tau, y, q):
    return y[0] - (6.0 + 2.0 * y[1]) - DIST_TO_SEPARATRIX


_separatrix_event.terminal = True
_separatrix_event.direction = -1


def _native_lib():
    try:
        from . import _lib
        lib = _lib.load()
    except Exception:
        return None
    return lib if hasattr(lib, "efd_host_trajectory") else None


class EMRIInspiral:
    """Sparse inspiral trajectory with the FEW `EMRIInspiral` call surface (stand-in physics)."""

    def __init__(self, func="SchwarzEccFlux", rtol=1e-12, atol=1e-12, max_init_len=1000,
                 backend="auto", **kwargs):
        if func not in ("SchwarzEccFlux", "pn5", "PN"):
            raise ValueError(f"unsupported trajectory func {func!r}")
        if backend not in ("auto", "native", "python"):
            raise ValueError("backend must be 'auto', 'native' or 'python'")
        self.func = func
        self.rtol = rtol
        self.atol = atol
        self.max_init_len = max_init_len
        self.lib = None if backend == "python" else _native_lib()
        if backend == "native" and self.lib is None:
            raise RuntimeError("the native trajectory needs libemrifd.so (build it first)")

    @property
    def backend(self):
        return "native" if self.lib is not None else "python"

    def with_frequencies(self, M, mu, a, p0, e0, x0=1.0, Phi_phi0=0.0, Phi_theta0=0.0,
                         Phi_r0=0.0, T=1.0, **kwargs):
        """(t, p, e, Phi_phi, Phi_r, f_phi, f_r): the knots and the orbital frequencies
        Omega / (2 pi M MTSUN_SI) at them (native backend: one call)."""
        if self.lib is None:
            t, p, e, _, pp, _, pr = self(M, mu, a, p0, e0, x0, Phi_phi0, Phi_theta0, Phi_r0, T=T)
            op, _, orr = get_fundamental_frequencies(0.0, p, e, 0.0)
            return t, p, e, pp, pr, op / (2 * np.pi * M * MTSUN_SI), orr / (2 * np.pi * M * MTSUN_SI)
        return self._native(M, mu, a, p0, e0, Phi_phi0, Phi_r0, T, freqs=True)

    def _native(self, M, mu, a, p0, e0, Phi_phi0, Phi_r0, T, freqs=False):
        if a != 0.0:
            raise ValueError("SchwarzEccFlux stand-in requires a = 0")
        if p0 - (6.0 + 2.0 * e0) <= DIST_TO_SEPARATRIX:
            raise ValueError("initial p0 lies inside the separatrix buffer")
        L = int(self.max_init_len)
        bufs = np.empty((7, L))
        n = ctypes.c_int32(0)
        p = lambda i: bufs[i].ctypes.data  # noqa: E731
        rc = self.lib.efd_host_trajectory(float(M), float(mu), float(p0), float(e0),
                                          float(Phi_phi0), float(Phi_r0), float(T), self.rtol,
                                          self.atol, L, p(0), p(1), p(2), p(3), p(4),
                                          p(5) if freqs else None, p(6) if freqs else None,
                                          ctypes.byref(n))
        if rc == -3:
            raise ValueError("trajectory longer than max_init_len")
        if rc != 0:
            raise RuntimeError(f"trajectory integration failed ({rc})")
        k = n.value
        out = [bufs[i, :k].copy() for i in range(7 if freqs else 5)]
        return tuple(out)

    def __call__(self, M, mu, a, p0, e0, x0=1.0, Phi_phi0=0.0, Phi_theta0=0.0, Phi_r0=0.0,
                 T=1.0, dt=10.0, **kwargs):
        if self.lib is not None:
            t, p, e, pp, pr = self._native(M, mu, a, p0, e0, Phi_phi0, Phi_r0, T)
            return t, p, e, np.ones_like(t), pp, np.full_like(t, Phi_theta0), pr
        if a != 0.0:
            raise ValueError("SchwarzEccFlux stand-in requires a = 0")
        if p0 - (6.0 + 2.0 * e0) <= DIST_TO_SEPARATRIX:
            raise ValueError("initial p0 lies inside the separatrix buffer")
        q = mu / M
        tscale = M * MTSUN_SI                      # seconds per unit of tau
        tau_max = T * YRSID_SI / tscale
        # a sensible first step (scipy's default guess is ~1e-3 s, which would put several
        # nearly coincident knots at t = 0 and make every spline over them ill-conditioned;
        # FEW's sparse trajectories start with an orbit-scale step)
        first_step = min(1e-3 * tau_max, 1e4)
        sol = solve_ivp(_pn_rhs, (0.0, tau_max), [p0, e0, Phi_phi0, Phi_r0], method="RK45",
                        rtol=self.rtol, atol=self.atol, args=(q,), events=_separatrix_event,
                        first_step=first_step)
        if not sol.success:
            raise RuntimeError(f"trajectory integration failed: {sol.message}")
        t = sol.t * tscale
        if len(t) > self.max_init_len:
            raise ValueError("trajectory longer than max_init_len")
        p, e, phi_phi, phi_r = sol.y
        x = np.ones_like(t)
        phi_theta = np.full_like(t, Phi_theta0)
        return t, p.copy(), e.copy(), x, phi_phi.copy(), phi_theta, phi_r.copy()

    def plunge_time(self, M, mu, a, p0, e0, x0=1.0, T_max=100.0):
        t = self(M, mu, a, p0, e0, x0, T=T_max)[0]
        return t[-1]


def get_p_at_t(traj_module, t_out, traj_args, index_of_p=3, index_of_a=2, index_of_e=4,
               index_of_x=5, traj_kwargs=None, xtol=2e-12, rtol=8.881784197001252e-16,
               bounds=None):
    """p0 such that the inspiral plunges after t_out years (few.utils.utility.get_p_at_t)."""
    traj_kwargs = {} if traj_kwargs is None else dict(traj_kwargs)
    # traj_args holds every argument but p (FEW convention): the index_of_* are positions in
    # the full (M, mu, a, p, e, x) list, so re-insert a placeholder at index_of_p
    full = list(traj_args[:index_of_p]) + [None] + list(traj_args[index_of_p:])
    M, mu = full[0], full[1]
    a, e0, x0 = full[index_of_a], full[index_of_e], full[index_of_x]
    T_max = 2.0 * t_out + 1.0

    def f(p0):
        t = traj_module(M, mu, a, p0, e0, x0, T=T_max, **traj_kwargs)[0]
        return t[-1] / YRSID_SI - t_out

    lo = 6.0 + 2.0 * e0 + DIST_TO_SEPARATRIX + 1e-3 if bounds is None or bounds[0] is None else bounds[0]
    hi = 40.0 if bounds is None or bounds[1] is None else bounds[1]
    lib = getattr(traj_module, "lib", None)
    if lib is not None and not traj_kwargs and a == 0.0:
        out = ctypes.c_double(0.0)
        rc = lib.efd_host_p_at_t(float(M), float(mu), float(e0), float(t_out), traj_module.rtol,
                                 traj_module.atol, float(xtol), float(rtol), float(lo), float(hi),
                                 ctypes.byref(out))
        if rc != 0:
            raise ValueError("could not bracket p0 for the requested t_out")
        return out.value
    if f(lo) > 0:
        raise ValueError("t_out is shorter than the plunge time from the separatrix buffer")
    while f(hi) < 0:
        hi *= 1.5
        if hi > 500:
            raise ValueError("could not bracket p0 for the requested t_out")
    return brentq(f, lo, hi, xtol=xtol, rtol=max(rtol, 4 * np.finfo(float).eps))

"""Schwarzschild fundamental frequencies (host side, upstream of the hot path).

Replaces `few.utils.utility.get_fundamental_frequencies(a, p, e, x)` as called at
Tutorial_FD_construction_single_mode.ipynb:227/280 (``get_fundamental_frequencies(0.0, p, e, 0.0)``).
Only a = 0 (Schwarzschild) is supported, which is all the reference's
"FastSchwarzschildEccentricFlux" model needs.

Method: Cutler-Kennefick-Poisson (1994) relativistic anomaly chi with r = p/(1 + e cos chi):
    dphi/dchi = sqrt(p / (p - 6 - 2 e cos chi))
    dt/dchi   = p^2 / ((p - 2 - 2 e cos chi)(1 + e cos chi)^2) * sqrt(((p-2)^2 - 4e^2) / (p - 6 - 2 e cos chi))
Both integrands are smooth and 2*pi periodic, so the trapezoid rule on a uniform chi grid
converges exponentially; 64 nodes reach double precision for p - 6 - 2e >= 0.1.
Returns dimensionless Omega (units of 1/M) like FEW; f = Omega / (2 pi M MTSUN_SI).
"""

import numpy as np

_NCHI = 64
_CHI = np.linspace(0.0, 2.0 * np.pi, _NCHI, endpoint=False)
_COS = np.cos(_CHI)


def get_fundamental_frequencies(a, p, e, x):
    """(OmegaPhi, OmegaTheta, OmegaR) for Schwarzschild eccentric equatorial orbits."""
    if np.any(np.asarray(a) != 0.0):
        raise ValueError("only Schwarzschild (a = 0) is supported by this model")
    p = np.asarray(p, dtype=np.float64)
    e = np.asarray(e, dtype=np.float64)
    scalar = p.ndim == 0 and e.ndim == 0
    p1, e1 = np.broadcast_arrays(np.atleast_1d(p), np.atleast_1d(e))
    if np.any(p1 - 6.0 - 2.0 * e1 <= 0.0):
        raise ValueError("p must lie outside the separatrix p = 6 + 2e")
    pc = p1[..., None]
    ec = e1[..., None]
    c = _COS
    den = pc - 6.0 - 2.0 * ec * c
    dphi = np.sqrt(pc / den)
    dt = pc * pc / ((pc - 2.0 - 2.0 * ec * c) * (1.0 + ec * c) ** 2) * np.sqrt(
        ((pc - 2.0) ** 2 - 4.0 * ec * ec) / den)
    t_r = dt.mean(axis=-1) * 2.0 * np.pi
    phi_r = dphi.mean(axis=-1) * 2.0 * np.pi
    omega_phi = phi_r / t_r
    omega_r = 2.0 * np.pi / t_r
    omega_theta = omega_phi.copy()  # equatorial Schwarzschild: Omega_theta = Omega_phi
    if scalar:
        return float(omega_phi[0]), float(omega_theta[0]), float(omega_r[0])
    return omega_phi, omega_theta, omega_r


def get_separatrix(a, e, x):
    """Schwarzschild separatrix p_sep = 6 + 2e (few.utils.utility.get_separatrix for a = 0)."""
    return 6.0 + 2.0 * np.asarray(e, dtype=np.float64)

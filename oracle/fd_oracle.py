"""CPU ORACLE for the FD mode-sum hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / CPU baseline. The product path (emri_frequencydomainwaveforms_amd)
never imports it and fails loudly when its HIP library is missing.

What it restates
----------------
The reference's only executable statement of the FD construction is the notebook function
`FD_waveform(freq)` (Tutorial_FD_construction_single_mode.ipynb:552-623, one (l,m,n) harmonic,
monotonic frequency only). FEW's production kernel (FDInterpolatedModeSum) is external and
absent offline. This module restates the notebook, line for line in
numpy/scipy, and generalises it to a sum over many harmonics:

  notebook line                                   here
  :558-559  phase_spline(t, m Phi_phi + n Phi_r)  _Harmonic.phase
  :561-564  theo_f = (m Om_phi + n Om_r)/(2piM)   F = m f_phi + n f_r (knot values)
  :566      t(f) = CubicSpline(theo_f, t)         one inverse spline per monotonic run
  :569-572  supports (freq > minF) & (freq < maxF) open interval per run; -F mirror
  :579-584  Fdot, Fddot spline derivatives        fdot = F'(t); fdd = (spline of fdot(t_i))'
  :587-594  H spline over Re/Im                   amplitude splines
  :599-613  K_{1/3} uniform amplitude             caustic="uniform" (default of the notebook)
  :615-616  Exp0/Exp1 phases                      identical
  :619-623  scatter + mu MRSUN/(dist Gpc)         sum over harmonics, times `prefactor`

Conventions (pinned by tests against golden vectors exec'd from the notebook itself):
* The notebook builds the spectrum in the *mirror* convention (a harmonic with F > 0 at +f;
  compared to the FFT at -f with a sign flip, notebook :503-504, :659). FEW's 'fd' output is
  the FFT convention, S(f) = fftshift(fft(h_+ - i h_x)) dt (Tutorial_FrequencyDomain_Waveforms
  .ipynb:187, :253-262), i.e. S(f) = -h_nb(-f). `fd_modesum` returns S on the caller's grid.
* Harmonics with m > 0 carry the -m partner branch (conjugated amplitude, partner Ylm that
  already contains (-1)^l, notebook :611); m = 0 harmonics have a single branch (their -n
  mirrors are separate modes in the list).
* Generalisations beyond the notebook (documented in DESIGN.md):
  - non-monotonic F(t): the knot sequence is split into maximal strictly monotonic runs and
    each run gets its own inverse spline and open support (notebook :1 says the notebook
    covers monotonic harmonics only); decreasing runs are reversed for CubicSpline;
  - caustic="spa": the plain stationary-phase limit, i.e. K_{1/3}(z) e^z replaced by its
    leading asymptote sqrt(pi/(2z)), which reduces exactly to
    Q = exp(i sgn(Fdot) 3 pi/4) / sqrt|Fdot|.
Spline boundary condition: not-a-knot (scipy CubicSpline default), the SURVEY.md section 8c
working assumption for FEW's CubicSplineInterpolant.
"""

import numpy as np
from scipy import special
from scipy.interpolate import CubicSpline

TWO_OVER_SQRT3 = 2.0 / np.sqrt(3.0)


def monotonic_runs(F):
    """Maximal runs [a, b] (knot indices, b > a) on which F is strictly monotonic."""
    d = np.sign(np.diff(F))
    runs = []
    i = 0
    nint = len(d)
    while i < nint:
        if d[i] == 0:
            i += 1
            continue
        j = i
        while j + 1 < nint and d[j + 1] == d[i]:
            j += 1
        runs.append((i, j + 1, int(d[i])))
        i = j + 1
    return runs


def _kv13_scaled_asymptotic(z, terms=8):
    """K_{1/3}(z) e^z for large |z|: sqrt(pi/(2z)) sum_k a_k z^-k (DLMF 10.40.2)."""
    acc = np.ones_like(z)
    a = np.ones_like(z)
    for k in range(1, terms):
        a = a * (4.0 / 9.0 - (2 * k - 1) ** 2) / (8.0 * k) / z
        acc = acc + a
    return np.sqrt(np.pi / (2.0 * z)) * acc


def _kfactor(fdot, fdd, caustic):
    """Q(t) such that the mirror-convention term is A Y Q exp(i(2 pi f t - Phi))."""
    if caustic == "uniform":
        arg = -2.0 * np.pi * 1j * fdot ** 3 / (3.0 * fdd ** 2)           # notebook :599
        with np.errstate(invalid="ignore", over="ignore"):
            kk = special.kv(1.0 / 3.0, arg) * np.exp(arg)               # notebook :600
        # scipy's AMOS kv returns NaN once |z| passes ~1e9 (total loss of significance in its
        # argument reduction; F'' -> 0 near an inflection of F'(t)). There the asymptotic
        # series is exact to double precision (|z|^-8 terms < 1e-70); the notebook itself
        # would emit NaN, which is a numerical artefact of scipy, not the construction.
        bad = ~np.isfinite(kk)
        if np.any(bad):
            kk = np.where(bad, _kv13_scaled_asymptotic(np.where(bad, arg, 1.0)), kk)
        with np.errstate(invalid="ignore", divide="ignore"):
            q = 1j * fdot / np.abs(fdd) * kk * TWO_OVER_SQRT3           # notebook :607-608
        # F'' = 0 exactly (e.g. a linear F on a 2-knot trajectory): |z| = inf, where the
        # uniform form's limit is the plain SPA factor (the notebook's expression is 0 * inf);
        # the C restatement and the kernel take the same limit
        flat = np.asarray(fdd) == 0.0
        if np.any(flat):
            q = np.where(flat, _kfactor(fdot, np.where(flat, 1.0, fdd), "spa"), q)
        return q
    if caustic == "spa":
        return np.exp(1j * np.sign(fdot) * 0.75 * np.pi) / np.sqrt(np.abs(fdot))
    raise ValueError(f"unknown caustic mode {caustic!r}")


class _Harmonic:
    def __init__(self, t, amp, phi_phi, phi_r, f_phi, f_r, m, n):
        self.m, self.n = int(m), int(n)
        self.t = t
        self.F = m * f_phi + n * f_r
        self.phase = CubicSpline(t, m * phi_phi + n * phi_r)
        self.H = CubicSpline(t, np.stack([amp.real, amp.imag]), axis=1)
        self.fdot = CubicSpline(t, self.F).derivative()
        self.fdd = CubicSpline(t, self.fdot(t)).derivative()

    def eval_at(self, tt):
        h = self.H(tt)
        return h[0] + 1j * h[1], self.phase(tt), self.fdot(tt), self.fdd(tt)


def single_harmonic_mirror(t, amp, phi_phi, phi_r, f_phi, f_r, m, n, ylm_p, ylm_m, fgrid,
                           caustic="uniform", partner=None):
    """Notebook-convention h_nb(fgrid) for one harmonic (no distance scaling)."""
    hm = _Harmonic(t, amp, phi_phi, phi_r, f_phi, f_r, m, n)
    partner = (m != 0) if partner is None else partner
    h = np.zeros(len(fgrid), dtype=np.complex128)
    for a, b, sgn in monotonic_runs(hm.F):
        x = hm.F[a:b + 1]
        y = t[a:b + 1]
        if sgn < 0:
            x, y = x[::-1], y[::-1]
        tinv = CubicSpline(x, y)
        lo, hi = x[0], x[-1]
        # +F branch (notebook Amp0/Exp0, :569, :607-609, :615)
        sel = (fgrid > lo) & (fgrid < hi)
        if np.any(sel):
            g = fgrid[sel]
            tt = tinv(g)
            A, Phi, fd, fdd = hm.eval_at(tt)
            Q = _kfactor(fd, fdd, caustic)
            h[sel] += A * ylm_p * Q * np.exp(1j * (2.0 * np.pi * g * tt - Phi))
        if not partner:
            continue
        # -F partner branch (notebook Amp1/Exp1, :570, :611-613, :616): conj amplitude,
        # partner Ylm, Fdot -> -Fdot, Fddot -> -Fddot, t(f) evaluated at -f
        sel = (fgrid > -hi) & (fgrid < -lo)
        if np.any(sel):
            g = fgrid[sel]
            tt = tinv(-g)
            A, Phi, fd, fdd = hm.eval_at(tt)
            Q1 = _kfactor(-fd, -fdd, caustic)
            h[sel] += np.conj(A) * ylm_m * Q1 * np.exp(1j * (2.0 * np.pi * g * tt + Phi))
    return h


def fd_modesum(t, amps, phi_phi, phi_r, f_phi, f_r, m, n, ylm_p, ylm_m, freq, prefactor=1.0,
               caustic="uniform"):
    """FEW-convention two-sided spectrum S(freq) = sum over harmonics, times prefactor.

    amps: complex [K, N_t]; m, n: [K]; ylm_p/ylm_m: complex [K]; freq: sorted grid.
    """
    freq = np.asarray(freq, dtype=np.float64)
    mirror = -freq
    h = np.zeros(len(freq), dtype=np.complex128)
    for k in range(len(m)):
        h += single_harmonic_mirror(t, amps[k], phi_phi, phi_r, f_phi, f_r, m[k], n[k],
                                    ylm_p[k], ylm_m[k], mirror, caustic=caustic)
    return -h * prefactor


def contributions(t, f_phi, f_r, m, n, freq):
    """C = number of (harmonic branch, bin) SPA contributions.

    Same supports as fd_modesum (open intervals on the mirror grid), counted by binary search
    on the sorted grid: -freq in (lo, hi) <=> freq in (-hi, -lo).
    """
    freq = np.asarray(freq)
    total = 0
    for mk, nk in zip(m, n):
        F = mk * f_phi + nk * f_r
        for a, b, sgn in monotonic_runs(F):
            lo, hi = (F[a], F[b]) if sgn > 0 else (F[b], F[a])
            total += int(np.searchsorted(freq, -lo, "left") - np.searchsorted(freq, -hi, "right"))
            if mk != 0:
                total += int(np.searchsorted(freq, hi, "left") - np.searchsorted(freq, lo, "right"))
    return total


def polarizations(S, freq=None, mask_positive=False):
    """FEW 'fd' list output [h+, hx] from S = h+ - i hx by the array flip (FEW-ext).

    mask_positive keeps the bins with freq >= 0 (emri_pe.py:239-241 compares it with
    `frequency >= 0.0`).
    """
    Sf = S[::-1]
    hp = 0.5 * (S + np.conj(Sf))
    hc = 0.5j * (S - np.conj(Sf))
    if mask_positive:
        keep = np.asarray(freq) >= 0.0
        return hp[keep], hc[keep]
    return hp, hc

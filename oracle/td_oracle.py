"""CPU ORACLE for the time-domain (TD) mode sum -- TEST INFRASTRUCTURE ONLY.

Only tests/ and __graft_entry__.smoke() may import this module, and only as the checker. The
product path never imports it.

What it restates
----------------
The reference compares its FD waveform against the DFT of FEW's time-domain waveform
(`td_gen = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux", sum_kwargs=dict(
pad_output=True, odd_len=True), return_list=True)`, Tutorial_FrequencyDomain_Waveforms.ipynb
:61-66, :184-188; check_mode_by_mode.py:85-99, :254-264). FEW's TD
summation (`InterpolatedModeSum`) is external and absent offline [FEW-ext], so this restates
its published construction directly:

    h(t_i) = h+ - i hx = scale * sum_k [ Y+_k A_k(t_i) e^{-i Phi_k(t_i)}
                                         + (m_k > 0) Y-_k conj(A_k(t_i)) e^{+i Phi_k(t_i)} ]
    Phi_k = m Phi_phi + n Phi_r,  t_i = i dt,  h = 0 for t_i > t[-1] (pad_output)

with not-a-knot cubic splines (scipy CubicSpline, as fd_oracle) of Re/Im A_k, Phi_phi and
Phi_r over the sparse trajectory, and Y-_k the partner harmonic that already holds (-1)^l
(the same arrays fd_oracle takes; notebook :611). The sign and phase conventions are the ones
under which the FD spectrum is the DFT of this waveform, S(f) ~ fftshift(fft(h)) dt
(Tutorial_FrequencyDomain_Waveforms.ipynb:187, :253-262): tests/test_oracle_td.py checks that
against fd_oracle (itself pinned to the notebook's FD_waveform), so the TD restatement is pinned
through the FD one; FEW's own TD output stays unpinned (FEW absent).
"""

import numpy as np
from scipy.interpolate import CubicSpline


def valid_samples(t_end, dt, nsamples):
    """Number of samples t_i = i dt (float64 product, as the kernel forms it) with t_i <= t_end."""
    ts = np.arange(nsamples, dtype=np.float64) * dt
    return int(np.searchsorted(ts, t_end, side="right"))


def td_modesum(t, amps, phi_phi, phi_r, m, n, ylm_p, ylm_m, dt, nsamples, prefactor=1.0,
               chunk=1 << 15):
    """Complex h = h+ - i hx at t_i = i dt, i < nsamples (zero past the trajectory's end).

    amps: complex [K, N_t]; m, n: [K]; ylm_p / ylm_m: complex [K]. Evaluated in chunks of
    samples so long waveforms stay within memory.
    """
    t = np.asarray(t, dtype=np.float64)
    amps = np.asarray(amps, dtype=np.complex128)
    m = np.asarray(m)
    n = np.asarray(n)
    ylm_p = np.asarray(ylm_p, dtype=np.complex128)
    ylm_m = np.asarray(ylm_m, dtype=np.complex128)
    spA = CubicSpline(t, np.concatenate([amps.real, amps.imag]), axis=1)
    spPp = CubicSpline(t, phi_phi)
    spPr = CubicSpline(t, phi_r)
    K = len(m)
    part = m > 0
    h = np.zeros(nsamples, dtype=np.complex128)
    nvalid = valid_samples(t[-1], dt, nsamples)
    for s0 in range(0, nvalid, chunk):
        ts = np.arange(s0, min(nvalid, s0 + chunk), dtype=np.float64) * dt
        a = spA(ts)
        A = a[:K] + 1j * a[K:]                                  # [K, ns]
        Phi = np.outer(m, spPp(ts)) + np.outer(n, spPr(ts))     # [K, ns]
        E = np.exp(-1j * Phi)
        acc = (ylm_p[:, None] * A * E).sum(axis=0)
        if np.any(part):
            acc += (ylm_m[part, None] * np.conj(A[part] * E[part])).sum(axis=0)
        h[s0:s0 + len(ts)] = acc
    return h * prefactor


def td_polarizations(h):
    """FEW's TD list output [h+, hx] from h = h+ - i hx."""
    return h.real.copy(), -h.imag


def dft_spectrum(x, dt):
    """fftshift(fft(x)) dt: the reference's DFT of a TD channel (FDutils.py:62-63)."""
    return np.fft.fftshift(np.fft.fft(x)) * dt

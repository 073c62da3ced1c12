"""CPU ORACLE for the likelihood side of the path -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker. Plain numpy restatements of:
  inner_product   LISAanalysistools/lisatools/diagnostic.py:95-110 (right-sum rule,
                  x = diff(f) with x[0] = x[1]; 4 sum Re(conj(a) b) / PSD * x)
  noise_factor    LISAanalysistools/lisatools/sampling/likelihood.py:177-180, 213-220
                  (w = sqrt(diff(f) / PSD), diff(f)[0] = diff(f)[1])
  loglike         likelihood.py:257-274 (ll = -1/2 * 4 * sum |d - h w|^2, bin 0 skipped
                  when w[0][0] is NaN)
  get_convolution FDutils.py:35-47 (convolve(hstack((a[1:], a)), b, 'valid') / len(b), direct)
  get_convolution_fft   the same for len(a) == len(b): the circular convolution, by FFTs
  windowed_polarizations  get_fd_windowed (FDutils.py:66-101) of the channels of a two-sided
                  spectrum S = h+ - i hx on an odd grid, through S: h+ = (S + M S) / 2,
                  hx = i (S - M S) / 2 with M the mirror-conjugation, which commutes with the
                  convolution by a Hermitian kernel (a real window's conj(fft(w)))
Pinned against tests/golden/likelihood_golden.npz, produced by the reference's own modules
(tests/golden/make_golden_likelihood.py).
"""

import numpy as np


def right_sum_weights(freqs):
    x = np.zeros(len(freqs))
    x[1:] = np.diff(freqs)
    x[0] = x[1]
    return x


def inner_product(a, b, freqs, psd, complex=False):
    if not isinstance(a, list):
        a, b = [a], [b]
    x = right_sum_weights(freqs)
    out = 0.0
    for p, q in zip(a, b):
        y = np.conj(p) * q
        y = y if complex else y.real
        out = out + 4.0 * np.sum(x * y / psd)
    return out


def noise_factor(freqs, psds):
    x = right_sum_weights(freqs)
    return np.asarray([(x / p) ** 0.5 for p in psds])


def loglike(h, d, w):
    """h, d complex [nchan][nbin] (d already weighted), w real [nchan][nbin]."""
    start = 1 if np.isnan(w[0, 0]) else 0
    r = d - h * w
    return -0.5 * 4.0 * np.sum((r[:, start:].conj() * r[:, start:]).real)


def get_convolution(a, b):
    return np.convolve(np.hstack((a[1:], a)), b, mode="valid") / len(b)


def get_convolution_fft(a, b, workers=None):
    """get_convolution for len(a) == len(b) = N: sum_j a[(k - j) mod N] b[j] / N, by FFTs."""
    import scipy.fft as sf
    if len(a) != len(b):
        raise ValueError("get_convolution_fft: equal lengths only")
    return sf.ifft(sf.fft(a, workers=workers) * sf.fft(b, workers=workers),
                   workers=workers) / len(b)


def polarizations(S):
    """[h+, hx] of a two-sided spectrum S = h+ - i hx on an odd grid (index k <-> N-1-k is
    f <-> -f): h+ = (S + conj(S[::-1])) / 2, hx = i (S - conj(S[::-1])) / 2."""
    Sm = np.conj(S[::-1])
    return 0.5 * (S + Sm), 0.5j * (S - Sm)


def windowed_polarizations(S, window, workers=None):
    """get_fd_windowed(polarizations(S), window) (each channel convolved with conj(fft(w)),
    FDutils.py:95-96), evaluated through S: (conj(fft(w)) (*) S) / N = ifft(w fft(S)) for a real
    window, then the polarizations of the result."""
    import scipy.fft as sf
    w = np.asarray(window, dtype=np.float64)
    Sw = sf.ifft(w * sf.fft(np.asarray(S, dtype=np.complex128), workers=workers),
                 workers=workers)
    return polarizations(Sw)

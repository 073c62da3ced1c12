"""The likelihood-side oracle (oracle/likelihood_oracle.py) against the reference's own outputs.

Golden vectors: tests/golden/likelihood_golden.npz from tests/golden/make_golden_likelihood.py,
which imports lisatools' inner_product/snr/Likelihood and FDutils from /root/reference and
runs them on seeded inputs. Tolerance 1e-12 relative: same float64 formulas, summation order
differs (numpy pairwise sums on both sides, different grouping).
"""

import os

import numpy as np
import pytest

from oracle import likelihood_oracle as lo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RTOL = 1e-12


@pytest.fixture(scope="module")
def g():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "likelihood_golden.npz")))


def _close(x, y, rtol=RTOL):
    x, y = np.asarray(x), np.asarray(y)
    return np.abs(x - y).max() <= rtol * max(np.abs(y).max(), 1e-300)


def test_inner_products(g):
    a, b, f, psd = list(g["ip_a"]), list(g["ip_b"]), g["ip_f"], g["ip_psd"]
    assert _close(lo.inner_product(a, b, f, psd), g["ip_plain"])
    assert _close(lo.inner_product(a, b, f, psd, complex=True), g["ip_complex"])
    aa = lo.inner_product(a, a, f, psd)
    bb = lo.inner_product(b, b, f, psd)
    assert _close(lo.inner_product(a, b, f, psd) / np.sqrt(aa * bb), g["ip_norm"])
    assert _close(lo.inner_product(a, b, f, psd) / aa, g["ip_norm_sig1"])
    a0, b0 = a[0], b[0]
    n0 = np.sqrt(lo.inner_product(a0, a0, f, psd) * lo.inner_product(b0, b0, f, psd))
    assert _close(lo.inner_product(a0, b0, f, psd) / n0, g["ip_chan0"])
    assert _close(np.sqrt(aa), g["snr_a"])
    assert _close(np.sqrt(lo.inner_product(a, b, f, psd)), g["snr_ab"])
    df = f[1] - f[0]
    fdf = (np.arange(len(f)) + 1) * df
    assert _close(lo.inner_product(a, b, fdf, psd), g["ip_df"])
    assert _close(lo.inner_product(list(g["ipu_a"]), list(g["ipu_b"]), g["ipu_f"], g["ipu_psd"]),
                  g["ipu_plain"])


def test_likelihood(g):
    f = g["ll_f"]
    from emri_frequencydomainwaveforms_amd.fdutils import get_sensitivity
    psd = [get_sensitivity(f)] * 2
    w = lo.noise_factor(f, psd)
    np.testing.assert_array_equal(w, g["ll_noise_factor"])

    def templ(amp, slope):
        return g["ll_base"] * amp + g["ll_tilt"] * slope

    d = templ(*g["ll_truth"]) * w
    np.testing.assert_array_equal(d, g["ll_injection"])
    ll = np.array([lo.loglike(templ(*p), d, w) for p in g["ll_params"]])
    assert ll[0] == 0.0
    assert _close(ll, g["ll_get_ll"])
    np.testing.assert_array_equal(g["ll_call"], g["ll_get_ll"])


def test_sensitivity_table_matches_reference(g):
    from emri_frequencydomainwaveforms_amd.fdutils import get_sensitivity
    np.testing.assert_array_equal(get_sensitivity(g["psd_f"]), g["psd"])
    np.testing.assert_array_equal(get_sensitivity(g["psd_fq"]), g["psd_q"])


def test_convolution_and_window(g):
    sig, win = g["win_sig"], g["win_window"]
    fw = np.conj(np.fft.fft(win))
    assert _close(lo.get_convolution(fw, sig[0]), g["win_conv"])
    assert _close(lo.get_convolution(fw, sig[1]), g["win_fd"][1])
    # circular-convolution identity the device path uses (len(a) == len(b))
    circ = np.fft.ifft(np.fft.fft(fw) * np.fft.fft(sig[0])) / len(win)
    assert _close(circ, g["win_conv"])
    np.testing.assert_allclose(g["win_fd_infd"], g["win_fd"], rtol=0, atol=1e-12)


def test_windowed_convolution_forms(g):
    """The FFT forms the full-size GPU test checks against (get_convolution_fft per channel,
    windowed_polarizations through S) equal the direct get_convolution of the reference's form
    (pinned to its scipy output by the golden fixture above) on the reference's own windowing
    inputs and on a random odd-grid spectrum with a Hann window (scipy.signal.windows.hann, as
    emri_pe.py:261)."""
    from scipy.signal.windows import hann
    sig, win = g["win_sig"], g["win_window"]
    a = np.conj(np.fft.fft(win))
    for ch in range(2):
        assert _close(lo.get_convolution_fft(a, sig[ch]), lo.get_convolution(a, sig[ch]), 1e-12)
    rng = np.random.default_rng(3)
    for N in (101, 1001):
        S = rng.normal(size=N) + 1j * rng.normal(size=N)
        w = hann(N)
        hp, hc = lo.polarizations(S)
        np.testing.assert_allclose(hp - 1j * hc, S, rtol=0, atol=1e-14)   # S = h+ - i hx
        aw = np.conj(np.fft.fft(w))
        ref_p, ref_c = lo.get_convolution(aw, hp), lo.get_convolution(aw, hc)
        wp, wc = lo.windowed_polarizations(S, w)
        assert _close(wp, ref_p, 1e-12) and _close(wc, ref_c, 1e-12)

"""Analytic LISA sensitivity (emri_frequencydomainwaveforms_amd/sensitivity.py) against the
reference's own lisatools/sensitivity.py outputs (tests/golden/likelihood_golden.npz, written by
tests/golden/make_golden_likelihood.py). Same constants and operation order, so the PSD must
match bitwise, including PSD(0) = inf (the f = 0 bin of the notebooks' positive grid)."""

import os

import numpy as np
import pytest

from emri_frequencydomainwaveforms_amd import sensitivity

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def g():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "likelihood_golden.npz")))


def test_cornish_psd_bitwise(g):
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        psd = sensitivity.cornish_lisa_psd(g["cornish_f"])
    assert np.isinf(psd[0]) and np.isinf(g["cornish_psd"][0])
    np.testing.assert_array_equal(psd, g["cornish_psd"])
    np.testing.assert_array_equal(sensitivity.cornish_lisa_psd(g["psd_fq"], sky_averaged=True),
                                  g["cornish_psd_sky"])


def test_get_sensitivity_return_types(g):
    fq = g["psd_fq"]
    np.testing.assert_array_equal(
        sensitivity.get_sensitivity(fq, sens_fn="cornish_lisa_psd", return_type="ASD"),
        g["cornish_asd_q"])
    np.testing.assert_array_equal(
        sensitivity.get_sensitivity(fq, sens_fn="cornish_lisa_psd", return_type="char_strain"),
        g["cornish_char_q"])


def test_get_sensitivity_errors():
    f = np.geomspace(1e-4, 1e-2, 8)
    with pytest.raises(NotImplementedError):
        sensitivity.get_sensitivity(f)                       # lisatools' default "lisasens"
    with pytest.raises(ValueError):
        sensitivity.get_sensitivity(f, sens_fn="no_such_curve")
    with pytest.raises(ValueError):
        sensitivity.get_sensitivity(f, sens_fn="cornish_lisa_psd", return_type="XSD")

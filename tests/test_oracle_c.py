"""The oracle's C restatement (CPU baseline) agrees with the numpy oracle (scipy splines/kv)."""

import numpy as np
import pytest

from oracle import fd_oracle, fd_oracle_c
from tests.helpers import source_inputs

pytestmark = pytest.mark.skipif(fd_oracle_c.load() is None, reason="gcc oracle build unavailable")


def _cmp(d, freq, caustic):
    args = (d["t"], d["amp"], d["phi_phi"], d["phi_r"], d["f_phi"], d["f_r"], d["m"], d["n"],
            d["ylm_p"], d["ylm_m"], freq, d["prefactor"])
    R = fd_oracle.fd_modesum(*args, caustic=caustic)
    C = fd_oracle_c.modesum(*args, caustic=caustic, nthreads=4)
    assert np.array_equal(np.nonzero(R)[0], np.nonzero(C)[0])
    return np.abs(C - R).max() / np.abs(R).max()


def test_golden_cases_c(golden_cases):
    for name, d in golden_cases.items():
        freq = np.fft.fftshift(np.fft.fftfreq(int(d["nf"]), float(d["dt"])))
        d = dict(d, prefactor=float(d["prefactor"]))
        assert _cmp(d, freq, "uniform") < 1e-9, name


@pytest.mark.parametrize("caustic", ["uniform", "spa"])
def test_multimode_c(caustic):
    d = source_inputs(M=3e5, mu=10.0, e0=0.35, T=0.01, dt=20.0, eps=1e-2)
    assert _cmp(d, d["freq"], caustic) < 1e-9


def test_turning_points_c():
    modes = [(2, 1, -2), (3, 2, -4), (2, 0, -3), (4, 1, -3), (3, 3, -5)]
    d = source_inputs(M=3e5, mu=10.0, e0=0.5, T=0.01, dt=20.0, modes=modes)
    assert _cmp(d, d["freq"], "uniform") < 1e-9

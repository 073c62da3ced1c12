"""GPU edge cases of the FD mode sum against the oracle (tolerance as test_gpu_modesum.py:
max|S_gpu - S_ref| <= 1e-9 max|S_ref|), and the C ABI's error behaviour.

- short trajectories: N_t = 2, 3 (scipy's linear / parabola special cases of CubicSpline, in the
  amplitude, phase and inverse splines alike), 4 and 5 (smallest not-a-knot systems);
- long trajectories up to the ABI's maximum N_t = 1024 knots, and 1025 rejected;
- a single m = 0 harmonic (one branch, no -m partner) and m > 0 with the partner switched off
  (ylm_m = 0, FEW's include_minus_m=False);
- a grid with no bin inside any harmonic's support (all-zero spectrum, C = 0);
- rejected shapes: K = 0, K > 8192, |m| > 255 (device-side check, reported by status).
"""

import numpy as np
import pytest
from scipy.interpolate import CubicSpline

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from emri_frequencydomainwaveforms_amd import _lib  # noqa: E402
from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine  # noqa: E402
from oracle import fd_oracle  # noqa: E402
from tests.helpers import source_inputs  # noqa: E402

RTOL = 1e-9


def _inp(d):
    return DeviceInputs.from_host(d["t"], np.asarray(d["amp"]).T, d["phi_phi"], d["phi_r"],
                                  d["f_phi"], d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"])


def _gpu(d, freq_h=None):
    freq_h = d["freq"] if freq_h is None else freq_h
    eng = ModeSumEngine()
    S = eng.run(_inp(d), torch.as_tensor(freq_h, device="cuda"), scale=float(d["prefactor"]))
    return S.cpu().numpy(), eng


def _oracle(d, freq_h=None):
    freq_h = d["freq"] if freq_h is None else freq_h
    return fd_oracle.fd_modesum(d["t"], np.asarray(d["amp"]), d["phi_phi"], d["phi_r"],
                                d["f_phi"], d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"],
                                freq_h, float(d["prefactor"]))


def _check(d, freq_h=None):
    S, eng = _gpu(d, freq_h)
    R = _oracle(d, freq_h)
    assert np.abs(R).max() > 0
    err = np.abs(S - R).max() / np.abs(R).max()
    assert err < RTOL, err
    assert np.array_equal(S != 0, R != 0)
    return eng


@pytest.fixture(scope="module")
def base():
    return source_inputs(M=3e5, mu=10.0, e0=0.35, T=0.02, dt=20.0, eps=1e-2)


def _resample(d, tn):
    """The same source on knots tn (per-knot data through a cubic spline of the originals)."""
    out = dict(d)
    t = d["t"]
    for key in ("phi_phi", "phi_r", "f_phi", "f_r"):
        out[key] = CubicSpline(t, d[key])(tn)
    amp = np.asarray(d["amp"])
    out["amp"] = CubicSpline(t, amp.real, axis=1)(tn) + 1j * CubicSpline(t, amp.imag, axis=1)(tn)
    out["t"] = tn
    return out


@pytest.mark.parametrize("nt", [2, 3, 4, 5])
def test_short_trajectories(base, nt):
    t = base["t"]
    d = _resample(base, np.linspace(t[0], t[-1], nt))
    _check(d)


# 512 / 513: the last knot count the preparation's parallel-cyclic-reduction splines take and
# the first that goes back to the Thomas kernel (emrifd.hip PCR_NMAX)
@pytest.mark.parametrize("nt", [257, 512, 513, 1024])
def test_long_trajectories(base, nt):
    t = base["t"]
    d = _resample(base, np.linspace(t[0], t[-1], nt))
    d = {**d, "amp": np.asarray(d["amp"])[:8], "m": d["m"][:8], "n": d["n"][:8],
         "ylm_p": d["ylm_p"][:8], "ylm_m": d["ylm_m"][:8]}
    _check(d)


def test_too_many_knots_rejected(base):
    t = base["t"]
    d = _resample(base, np.linspace(t[0], t[-1], 1025))
    with pytest.raises(_lib.EFDError):
        _gpu(d)


def test_single_m0_harmonic_and_no_partner(base):
    k0 = int(np.nonzero(base["m"] == 0)[0][0])
    one = {**base, "amp": np.asarray(base["amp"])[k0:k0 + 1], "m": base["m"][k0:k0 + 1],
           "n": base["n"][k0:k0 + 1], "ylm_p": base["ylm_p"][k0:k0 + 1],
           "ylm_m": base["ylm_m"][k0:k0 + 1]}
    _check(one)
    nopartner = {**base, "ylm_m": np.zeros_like(base["ylm_m"])}
    _check(nopartner)


def test_grid_outside_every_support(base):
    # bins far above every harmonic's frequency range: the spectrum is exactly zero
    fmax = max(np.abs(base["m"] * base["f_phi"][:, None] + base["n"] * base["f_r"][:, None]).max(),
               1e-3)
    p = np.linspace(2.0 * fmax, 3.0 * fmax, 501)
    freq = np.concatenate([-p[::-1], p])
    S, eng = _gpu(base, freq)
    assert not S.any()
    assert eng.contributions() == 0


def test_rejected_shapes(base):
    d = base
    empty = {**d, "amp": np.asarray(d["amp"])[:0], "m": d["m"][:0], "n": d["n"][:0],
             "ylm_p": d["ylm_p"][:0], "ylm_m": d["ylm_m"][:0]}
    with pytest.raises((_lib.EFDError, ValueError)):
        _gpu(empty)
    big = {**d, "m": d["m"].copy()}
    big["m"][0] = 300                              # |m| > 255
    with pytest.raises(_lib.EFDError):
        _gpu(big)
    K = 8193
    many = {**d, "amp": np.tile(np.asarray(d["amp"])[:1], (K, 1)), "m": np.ones(K, np.int32),
            "n": np.zeros(K, np.int32), "ylm_p": np.ones(K, complex), "ylm_m": np.ones(K, complex)}
    with pytest.raises(_lib.EFDError):
        _gpu(many)


@pytest.mark.parametrize("K", [8, 100])
def test_runs_overflow_reported(base, K):
    """A frequency track with more than MAXRUNS (8) monotonic runs is reported by the status
    check (sticky runs_overflow flag), whether the preparation groups the harmonics inside its
    spline kernel (K <= 64, every role on PCR) or in k_group (K > 64); the report clears it, and
    a clean source on the same engine then runs clean."""
    t = base["t"]
    d = _resample(base, np.linspace(t[0], t[-1], 256))
    idx = np.arange(K) % len(base["m"])
    d = {**d, "amp": np.asarray(d["amp"])[idx], "m": d["m"][idx], "n": d["n"][idx],
         "ylm_p": d["ylm_p"][idx], "ylm_m": d["ylm_m"][idx]}
    tt = d["t"]
    wiggle = 1.0 + 0.2 * np.sin(2 * np.pi * 12 * (tt - tt[0]) / (tt[-1] - tt[0]))
    bad = {**d, "f_phi": d["f_phi"] * wiggle}
    eng = ModeSumEngine()
    freq = torch.as_tensor(d["freq"], device="cuda")
    with pytest.raises(_lib.EFDError):
        eng.run(_inp(bad), freq, scale=float(d["prefactor"]))
    S = eng.run(_inp(d), freq, scale=float(d["prefactor"])).cpu().numpy()
    R = _oracle(d)
    assert np.abs(S - R).max() <= RTOL * np.abs(R).max()


@pytest.mark.parametrize("seed", range(6))
def test_random_sources_finite_and_oracle(seed):
    """Seeded random sources over the configs' parameter ranges (M in [1e5, 1e7], e0 in
    [0.05, 0.7], random viewing angles, inspirals ending in the plunge at 0.99 T): every bin
    finite, the oracle's support, and the oracle's spectrum to 1e-9 of max|S|. The fast path's
    masked lanes (out-of-interval, F' of the other sign, |y| past the series' range) must never
    leak a NaN or inf into the sums."""
    rng = np.random.default_rng(1000 + seed)
    M = float(10.0 ** rng.uniform(5.0, 7.0))
    d = source_inputs(M=M, mu=1e-5 * M, e0=float(rng.uniform(0.05, 0.7)),
                      T=float(rng.choice([0.01, 0.03])), dt=20.0, eps=1e-2,
                      theta=float(rng.uniform(0.1, 3.0)), phi=float(rng.uniform(-3.0, 3.0)))
    S, _ = _gpu(d)
    assert np.all(np.isfinite(S))
    _check(d)

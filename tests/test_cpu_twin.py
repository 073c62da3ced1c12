"""The host twin efd_modesum_cpu (csrc/emrifd_cpu.cpp, in libemrifd.so) against the oracle.

The twin is the same algorithm as the HIP path on the CPU (grouping, splines, interval records,
tile-wise output-stationary sum, uniform K_{1/3} fast path); it is bench.py's CPU baseline and
the GPU tests hold the kernels to it (tests/test_gpu_twin.py). Here, on the CPU:
- the notebook's own FD_waveform golden vectors (tests/golden, make_golden.py): 1e-9 max|S|;
- multi-harmonic sums against the numpy oracle, both caustic modes, symmetric and asymmetric
  grids: 1e-9 max|S|;
- config 1 at full size (3,155,815 bins) against the C oracle with the per-bin split tolerance
  of tests/helpers.split_check (1e-9 max|R| off folds and extrapolated terms), identical
  support and contribution count;
- the fused h+/hx output, accumulate, linearity in the harmonic set, thread-count invariance,
  argument errors, and the other twins (spline build vs scipy, loglike and inner product vs
  the likelihood oracle).
"""

import numpy as np
import pytest

from emri_frequencydomainwaveforms_amd import _lib, cputwin
from oracle import fd_oracle, fd_oracle_c
from oracle import likelihood_oracle as lo
from tests.helpers import source_inputs, split_check, ulp_perturbation

KEYS = ("t", "phi_phi", "phi_r", "f_phi", "f_r", "m", "n", "ylm_p", "ylm_m")


def _twin(d, freq, **kw):
    return cputwin.modesum(d["t"], np.ascontiguousarray(d["amp"].T), d["phi_phi"], d["phi_r"],
                           d["f_phi"], d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"], freq,
                           d["prefactor"], **kw)


def _oracle(d, freq, caustic="uniform"):
    return fd_oracle.fd_modesum(d["t"], d["amp"], d["phi_phi"], d["phi_r"], d["f_phi"], d["f_r"],
                                d["m"], d["n"], d["ylm_p"], d["ylm_m"], freq, d["prefactor"],
                                caustic=caustic)


@pytest.mark.parametrize("name", ["nb_params_220", "plunge_220", "plunge_331", "plunge_211",
                                  "plunge_42m1"])
def test_twin_matches_notebook_golden(golden_cases, name):
    d = golden_cases[name]
    freq = np.fft.fftshift(np.fft.fftfreq(int(d["nf"]), float(d["dt"])))
    S = cputwin.modesum(d["t"], d["amp"].T, d["phi_phi"], d["phi_r"], d["f_phi"], d["f_r"],
                        d["m"], d["n"], d["ylm_p"], d["ylm_m"], freq, float(d["prefactor"]))
    G = np.zeros(len(freq), dtype=np.complex128)
    G[d["idx"]] = d["val"]
    assert np.array_equal(np.nonzero(S)[0], d["idx"])
    assert np.abs(S - G).max() <= 1e-9 * np.abs(G).max()


@pytest.fixture(scope="module")
def src():
    return source_inputs(M=3e5, e0=0.35, T=0.02, dt=20.0, eps=1e-2)


@pytest.mark.parametrize("caustic", ["uniform", "spa"])
def test_twin_multimode_vs_oracle(src, caustic):
    d = src
    S = _twin(d, d["freq"], caustic=caustic)
    R = _oracle(d, d["freq"], caustic)
    assert len(d["m"]) > 20
    assert np.abs(S - R).max() <= 1e-9 * np.abs(R).max()
    np.testing.assert_array_equal(S != 0, R != 0)
    C, ev, G = cputwin.stats()
    assert C == fd_oracle.contributions(d["t"], d["f_phi"], d["f_r"], d["m"], d["n"], d["freq"])
    assert G == len(set(zip(d["m"].tolist(), d["n"].tolist()))) and ev <= C


def test_twin_asymmetric_and_downsampled_grids(src):
    d = src
    R0 = _oracle(d, d["freq"])
    nz = np.abs(R0[d["freq"] >= 0]) > 0
    fmax = d["freq"][d["freq"] >= 0][nz].max() * 1.01
    asym = np.hstack((-np.linspace(fmax, 0.0, 40)[:-1], np.linspace(0.0, fmax, 61)))
    p = np.linspace(0.0, fmax, 77)
    down = np.hstack((-p[::-1][:-1], p))
    for grid, sym in ((asym, False), (down, True)):
        assert bool(np.array_equal(grid, -grid[::-1])) == sym
        S = _twin(d, grid)
        R = _oracle(d, grid)
        assert np.abs(S - R).max() <= 1e-9 * np.abs(R).max()


def test_twin_polarizations_accumulate_linearity_threads(src):
    d = src
    freq = d["freq"]
    S = _twin(d, freq)
    k0 = int(np.searchsorted(freq, 0.0))
    hp, hc = _twin(d, freq, polarizations=True, k0=k0)
    rp, rc = fd_oracle.polarizations(S, freq, mask_positive=True)
    np.testing.assert_array_equal(hp, rp)
    np.testing.assert_array_equal(hc, rc)
    # linearity in the harmonic set, through accumulate (splits (m, n) groups apart)
    idx = np.arange(len(d["m"]))
    a, b = idx[idx % 3 == 0], idx[idx % 3 != 0]
    sub = lambda sel: {**{k: d[k][sel] for k in ("m", "n", "ylm_p", "ylm_m")},  # noqa: E731
                       **{k: d[k] for k in ("t", "phi_phi", "phi_r", "f_phi", "f_r", "prefactor")},
                       "amp": d["amp"][sel]}
    P = _twin(sub(a), freq)
    _twin(sub(b), freq, out=P, accumulate=True)
    assert np.abs(P - S).max() <= 1e-12 * np.abs(S).max()
    # thread count changes the schedule only: bitwise the same spectrum
    prev = cputwin.set_threads(1)
    try:
        S1 = _twin(d, freq)
    finally:
        cputwin.set_threads(prev)
    np.testing.assert_array_equal(S1, S)


def test_twin_argument_errors(src):
    d = dict(src)
    d["m"] = d["m"].copy()
    d["m"][0] = 300
    with pytest.raises(_lib.EFDError, match=r"\|m\| > 255"):
        _twin(d, src["freq"])
    d = dict(src)
    nt = len(d["t"])
    d["f_r"] = d["f_r"] * (1.0 + 0.3 * (-1.0) ** np.arange(nt))   # > 8 monotonic runs
    with pytest.raises(_lib.EFDError, match="monotonic runs"):
        _twin(d, src["freq"])
    with pytest.raises(_lib.EFDError, match="symmetric"):
        _twin(src, src["freq"][1:], polarizations=True)


def test_twin_config1_full_grid_vs_c_oracle():
    import bench
    w = bench.build_workload(T=1.0, dt=10.0, eps=1e-2)
    S = cputwin.modesum(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"], w["f_r"], w["m"],
                        w["n"], w["ylm_p"], w["ylm_m"], w["freq"], w["prefactor"])
    C, _, _ = cputwin.stats()
    args = (w["amp"].T,)

    def orc(p=None, extrap=False):
        p = p or (lambda x: x)
        return fd_oracle_c.modesum(p(w["t"]), *args, p(w["phi_phi"]), p(w["phi_r"]),
                                   p(w["f_phi"]), p(w["f_r"]), w["m"], w["n"], w["ylm_p"],
                                   w["ylm_m"], w["freq"], w["prefactor"], extrap=extrap)
    R, E = orc(extrap=True)
    ok, stats, _ = split_check(S, R, [orc(ulp_perturbation(s)) for s in (21, 22)], E=E)
    assert ok, stats
    assert stats["max_err_off_fold_rel"] <= 1e-9
    np.testing.assert_array_equal(S != 0, R != 0)
    assert C == fd_oracle.contributions(w["t"], w["f_phi"], w["f_r"], w["m"], w["n"], w["freq"])


def test_spline_build_cpu_matches_scipy():
    import ctypes
    from scipy.interpolate import CubicSpline
    rng = np.random.default_rng(3)
    lib = _lib.load()
    for n in (2, 3, 4, 7, 40):
        x = np.cumsum(rng.uniform(0.5, 2.0, n))
        y = rng.normal(size=(n, 5))
        coef = np.empty((n - 1, 4, 5))
        assert lib.efd_spline_build_cpu(x.ctypes.data, n, y.ctypes.data, 5, coef.ctypes.data,
                                        None) == 0
        ref = CubicSpline(x, y).c.transpose(1, 0, 2)            # [n-1][4][5]
        np.testing.assert_allclose(coef, ref, rtol=1e-11, atol=1e-11 * np.abs(ref).max())
    _ = ctypes


def test_loglike_and_inner_product_cpu_vs_oracle():
    lib = _lib.load()
    rng = np.random.default_rng(4)
    nb = 1001
    h = rng.normal(size=(2, nb)) + 1j * rng.normal(size=(2, nb))
    d = rng.normal(size=(2, nb)) + 1j * rng.normal(size=(2, nb))
    w = rng.uniform(0.1, 2.0, size=(2, nb))
    out = np.zeros(2)
    assert lib.efd_loglike_cpu(h.ctypes.data, d.ctypes.data, w.ctypes.data, 2, nb,
                               out.ctypes.data, None, None) == 0
    ref = lo.loglike(h, d, w)
    assert abs(out[0] - ref) <= 1e-12 * abs(ref)
    assert lib.efd_inner_product_cpu(h.ctypes.data, d.ctypes.data, w.ctypes.data, 2, nb,
                                     out.ctypes.data, None, None) == 0
    ref = 4.0 * np.sum(np.conj(h) * d * w)
    assert abs(out[0] - ref.real) <= 1e-12 * abs(ref) and abs(out[1] - ref.imag) <= 1e-12 * abs(ref)


_ENV_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import bench
from emri_frequencydomainwaveforms_amd import cputwin
w = bench.build_workload(T=0.25, eps=1e-3)
S = cputwin.modesum(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"], w["f_r"], w["m"],
                    w["n"], w["ylm_p"], w["ylm_m"], w["freq"], w["prefactor"])
np.save(sys.argv[2], S)
"""


def test_twin_envelope_records_on_and_off(tmp_path):
    """The twin's envelope records (env_fit.inc, as k_items: A(w) of degree 6 and theta(w)
    folded into the phase cubic on records whose polynomials pass the 1e-11 / 1e-10 check)
    against the per-bin arithmetic (EFD_ENV=0, a child process each): within 1e-10 of max|S|
    on a 0.25-yr eps = 1e-3 source, identical support."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    S = {}
    for env in ("1", "0"):
        path = str(tmp_path / f"S{env}.npy")
        r = subprocess.run([sys.executable, "-c", _ENV_CHILD, root, path], capture_output=True,
                           text=True, timeout=300, env=dict(os.environ, EFD_ENV=env), cwd=root)
        assert r.returncode == 0, r.stderr[-3000:]
        S[env] = np.load(path)
    mx = np.abs(S["0"]).max()
    np.testing.assert_array_equal(S["1"] != 0, S["0"] != 0)
    assert 0.0 < np.abs(S["1"] - S["0"]).max() <= 1e-10 * mx

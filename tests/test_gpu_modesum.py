"""GPU parity of the HIP FD mode sum against the oracle and the notebook golden vectors.

Tolerance (stated per BASELINE.json:north_star "stated relative tolerance on the complex
spectrum"): max_k |S_gpu - S_ref| <= 1e-9 * max_k |S_ref|. Both sides are FP64; the remaining
difference is rounding in phases of up to ~1e6 rad (1 ulp ~ 1e-10 rad) and the K_{1/3}
evaluation (series here vs AMOS in scipy), measured at ~1e-11.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine  # noqa: E402
from oracle import fd_oracle  # noqa: E402
from tests.helpers import source_inputs  # noqa: E402

RTOL = 1e-9


def _gpu(d, freq_h, caustic="uniform", sym=None, scale=None):
    inp = DeviceInputs.from_host(d["t"], np.asarray(d["amp"]).T, d["phi_phi"], d["phi_r"],
                                 d["f_phi"], d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"])
    freq = torch.as_tensor(np.asarray(freq_h, dtype=np.float64), device="cuda")
    eng = ModeSumEngine(caustic=caustic)
    sc = float(d["prefactor"]) if scale is None else scale
    S = eng.run(inp, freq, grid_symmetric=sym, scale=sc)
    return S.cpu().numpy(), eng


def _oracle(d, freq_h, caustic="uniform", scale=None):
    sc = float(d["prefactor"]) if scale is None else scale
    return fd_oracle.fd_modesum(d["t"], np.asarray(d["amp"]), d["phi_phi"], d["phi_r"],
                                d["f_phi"], d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"],
                                freq_h, sc, caustic=caustic)


def _relerr(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.fixture(scope="module")
def multimode():
    return source_inputs(M=3e5, mu=10.0, e0=0.35, T=0.02, dt=20.0, eps=1e-2)


def test_golden_notebook_vectors(golden_cases):
    for name, d in golden_cases.items():
        nf = int(d["nf"])
        freq = np.fft.fftshift(np.fft.fftfreq(nf, float(d["dt"])))
        S, _ = _gpu(d, freq)
        G = np.zeros(nf, dtype=np.complex128)
        G[d["idx"]] = d["val"]
        assert np.array_equal(np.nonzero(S)[0], d["idx"]), f"{name}: support differs"
        assert _relerr(S, G) < RTOL, f"{name}: {_relerr(S, G):.3e}"


@pytest.mark.parametrize("caustic", ["uniform", "spa"])
def test_multimode_vs_oracle(multimode, caustic):
    d = multimode
    S, eng = _gpu(d, d["freq"], caustic=caustic)
    R = _oracle(d, d["freq"], caustic=caustic)
    assert len(d["m"]) > 20
    assert _relerr(S, R) < RTOL
    assert np.array_equal(np.nonzero(S)[0], np.nonzero(R)[0])
    # the kernel's own contribution count equals the oracle's
    C = fd_oracle.contributions(d["t"], d["f_phi"], d["f_r"], d["m"], d["n"], d["freq"])
    assert eng.contributions() == C


def test_non_monotonic_and_negative_harmonics():
    # m = 1, 2 with large negative n: F = m f_phi + n f_r crosses zero / turns over
    modes = [(2, 1, -2), (3, 2, -4), (2, 0, -3), (2, 0, 2), (4, 1, -3), (3, 3, -5), (2, 2, 0)]
    d = source_inputs(M=3e5, mu=10.0, e0=0.5, T=0.02, dt=20.0, modes=modes)
    for caustic in ("uniform", "spa"):
        S, _ = _gpu(d, d["freq"], caustic=caustic)
        R = _oracle(d, d["freq"], caustic=caustic)
        assert _relerr(S, R) < RTOL, caustic


def test_asymmetric_grid_unpaired(multimode):
    d = multimode
    N = len(d["freq"]) - 1                      # even length: fftfreq grid is not symmetric
    freq = np.fft.fftshift(np.fft.fftfreq(N, d["dt"]))
    S, _ = _gpu(d, freq, sym=False)
    R = _oracle(d, freq)
    assert _relerr(S, R) < RTOL


def test_paired_equals_unpaired_on_symmetric_grid(multimode):
    d = multimode
    Sp, _ = _gpu(d, d["freq"], sym=True)
    Su, _ = _gpu(d, d["freq"], sym=False)
    assert _relerr(Sp, Su) < 1e-13


def test_downsampled_linspace_grid(multimode):
    # emri_pe.py:333-349: p_freq = linspace(0, 1.01 fmax, num); f_arr = hstack(-p[::-1][:-1], p)
    d = multimode
    R0 = _oracle(d, d["freq"])
    fpos = d["freq"][d["freq"] >= 0]
    nz = np.abs(R0[d["freq"] >= 0]) > 0
    p_freq = np.linspace(0.0, fpos[nz].max() * 1.01, num=int(nz.sum() / 10))
    f_arr = np.hstack((-p_freq[::-1][:-1], p_freq))
    S, _ = _gpu(d, f_arr)
    R = _oracle(d, f_arr)
    assert _relerr(S, R) < RTOL


def test_deterministic(multimode):
    d = multimode
    S1, _ = _gpu(d, d["freq"])
    S2, _ = _gpu(d, d["freq"])
    assert np.array_equal(S1, S2)


def test_complex_scale_and_accumulate(multimode):
    d = multimode
    sc = 0.3 - 0.7j
    S, _ = _gpu(d, d["freq"], scale=sc)
    R = _oracle(d, d["freq"], scale=1.0) * sc
    assert _relerr(S, R) < RTOL
    inp = DeviceInputs.from_host(d["t"], d["amp"].T, d["phi_phi"], d["phi_r"], d["f_phi"],
                                 d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"])
    freq = torch.as_tensor(d["freq"], device="cuda")
    eng = ModeSumEngine()
    out = eng.run(inp, freq, scale=1.0)
    out = eng.run(inp, freq, out=out, scale=1.0, accumulate=True)
    assert _relerr(out.cpu().numpy(), 2.0 * _oracle(d, d["freq"], scale=1.0)) < RTOL


def test_coarse_grid_many_records_per_tile():
    # a coarse symmetric grid puts thousands of interval records in one tile: exercises the
    # multi-pass (KEYCAP = 2048 keys) path of the in-LDS tile lists
    d = source_inputs(M=3e5, mu=10.0, e0=0.35, T=0.01, dt=20.0, eps=1e-4)
    fmax = d["freq"].max()
    p_freq = np.linspace(0.0, fmax, 400)
    f_arr = np.hstack((-p_freq[::-1][:-1], p_freq))      # 799 bins -> 400 lanes, one tile
    nrec = len(d["m"]) * (len(d["t"]) - 1)
    assert nrec > 2 * 2048
    S, _ = _gpu(d, f_arr)
    R = _oracle(d, f_arr)
    assert _relerr(S, R) < RTOL


def test_spline_build_matches_scipy():
    import ctypes
    from scipy.interpolate import CubicSpline
    from emri_frequencydomainwaveforms_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(1)
    for n in (2, 3, 4, 5, 17, 120):
        x = np.cumsum(rng.uniform(0.5, 2.0, n))
        y = rng.normal(size=(n, 7))
        coef = torch.empty((n - 1) * 4 * 7, dtype=torch.float64, device="cuda")
        xd = torch.as_tensor(x, device="cuda")
        yd = torch.as_tensor(y, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.efd_spline_build(xd.data_ptr(), n, yd.data_ptr(), 7, coef.data_ptr(),
                                        ctypes.c_void_p(st)), "spline")
        torch.cuda.synchronize()
        c = coef.cpu().numpy().reshape(n - 1, 4, 7)
        ref = CubicSpline(x, y, axis=0).c            # [4][n-1][7]
        np.testing.assert_allclose(np.transpose(c, (1, 0, 2)), ref, rtol=1e-11,
                                   atol=1e-11 * np.abs(ref).max())


def test_polarizations_and_mask(multimode):
    from emri_frequencydomainwaveforms_amd.summation import FDInterpolatedModeSum
    d = multimode
    mod = FDInterpolatedModeSum(use_gpu=True)
    S = mod.spectrum(d["t"], d["amp"].T, d["ylm_p"], d["ylm_m"], d["phi_phi"], d["phi_r"],
                     d["m"], d["n"], d["M"], d["p"], d["e"], dt=d["dt"], T=d["T"])
    Sh = S.cpu().numpy()
    for mask in (False, True):
        hp, hc = mod.polarizations(S, mask_positive=mask)
        rp, rc = fd_oracle.polarizations(Sh, d["freq"], mask_positive=mask)
        np.testing.assert_array_equal(hp.cpu().numpy(), rp)
        np.testing.assert_array_equal(hc.cpu().numpy(), rc)
    # check_mode_by_mode.py:247 identity: <h+ - i hx, S> / <S, S> == 1
    hp, hc = mod.polarizations(S)
    comb = (hp - 1j * hc).cpu().numpy()
    ratio = np.vdot(comb, Sh) / np.vdot(Sh, Sh)
    assert abs(ratio - 1.0) < 1e-14


def test_loglike_matches_numpy():
    import ctypes
    from emri_frequencydomainwaveforms_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(3)
    nbin = 100_003
    h = rng.normal(size=(2, nbin)) + 1j * rng.normal(size=(2, nbin))
    dd = rng.normal(size=(2, nbin)) + 1j * rng.normal(size=(2, nbin))
    w = rng.uniform(0.1, 2.0, size=(2, nbin))
    ref = -0.5 * 4.0 * np.sum(np.abs(dd - h * w) ** 2)
    H = torch.as_tensor(h, device="cuda")
    D = torch.as_tensor(dd, device="cuda")
    W = torch.as_tensor(w, device="cuda")
    out = torch.zeros(1, dtype=torch.float64, device="cuda")
    scr = torch.zeros(_lib.EFD_LOGLIKE_SCRATCH, dtype=torch.float64, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.efd_loglike(torch.view_as_real(H).data_ptr(), torch.view_as_real(D).data_ptr(),
                               W.data_ptr(), 2, nbin, out.data_ptr(), scr.data_ptr(), st), "ll")
    assert abs(out.item() - ref) <= 1e-12 * abs(ref)


def test_fused_polarizations_and_two_phase_api(multimode):
    """efd_modesum_prepare + efd_modesum_sum with hp/hc == efd_modesum then efd_polarizations,
    bitwise, for k0 at f = 0 (mask_positive) and k0 = 0 (full grid), plus accumulate."""
    import ctypes
    from emri_frequencydomainwaveforms_amd import _lib
    d = multimode
    inp = DeviceInputs.from_host(d["t"], np.asarray(d["amp"]).T, d["phi_phi"], d["phi_r"],
                                 d["f_phi"], d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"])
    freq = torch.as_tensor(d["freq"], device="cuda")
    nf = len(d["freq"])
    eng = ModeSumEngine()
    S = eng.run(inp, freq, grid_symmetric=True, scale=d["prefactor"])
    st = torch.cuda.current_stream().cuda_stream
    for k0 in (int(np.searchsorted(d["freq"], 0.0)), 0):
        rp = torch.empty(nf - k0, dtype=torch.complex128, device="cuda")
        rc = torch.empty_like(rp)
        _lib.check(eng.lib.efd_polarizations(torch.view_as_real(S).data_ptr(), nf, k0,
                                             torch.view_as_real(rp).data_ptr(),
                                             torch.view_as_real(rc).data_ptr(),
                                             ctypes.c_void_p(st)), "pol")
        hp = torch.full_like(rp, np.nan)
        hc = torch.full_like(rp, np.nan)
        eng.launch(inp, freq, None, True, d["prefactor"], phase="prepare")
        eng.launch(inp, freq, None, True, d["prefactor"], phase="sum",
                   hp=torch.view_as_real(hp), hc=torch.view_as_real(hc), k0=k0)
        assert eng.status()
        assert torch.equal(hp, rp) and torch.equal(hc, rc)
        eng.launch(inp, freq, None, True, d["prefactor"], accumulate=True,
                   hp=torch.view_as_real(hp), hc=torch.view_as_real(hc), k0=k0)
        assert eng.status()
        assert torch.allclose(hp, 2 * rp, rtol=1e-15, atol=0) and torch.allclose(hc, 2 * rc,
                                                                                rtol=1e-15, atol=0)
    with pytest.raises(_lib.EFDError):   # fused outputs need a symmetric grid
        eng.launch(inp, freq, None, False, d["prefactor"], hp=torch.view_as_real(hp),
                   hc=torch.view_as_real(hc), k0=0)


def test_wide_mn_range_grouping(multimode):
    """k_group's two paths: the counting sort over the (m, n) box the harmonics span (at most
    2048 cells, every other test) and, past that, the bitonic sort of (m, n, h) keys. Shifting n
    of every third harmonic by 250 widens the box to > 2048 cells (those harmonics then lie
    beyond the grid's Nyquist frequency); the spectrum of the others, grouped by the second
    path, must still match the oracle (which takes the harmonics one by one)."""
    d = dict(multimode)
    n = np.array(d["n"]).copy()
    n[::3] += 250
    d["n"] = n
    m = np.asarray(d["m"])
    assert (m.max() - m.min() + 1) * (n.max() - n.min() + 1) > 2048
    S, eng = _gpu(d, d["freq"])
    R = _oracle(d, d["freq"])
    assert _relerr(S, R) < RTOL


def _dev_inputs(d):
    return DeviceInputs.from_host(d["t"], np.asarray(d["amp"]).T, d["phi_phi"], d["phi_r"],
                                  d["f_phi"], d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"])


def test_sum_batch_matches_single_sums(multimode):
    """efd_modesum_sum_batch: three different waveforms (different trajectories, harmonic
    counts and amplitudes) on one grid, summed in one launch, give bitwise the spectra (and fused
    h+/hx) of their own efd_modesum_sum, on the paired and the unpaired kernel; mismatched grids
    and bad counts are rejected."""
    from emri_frequencydomainwaveforms_amd import _lib
    from emri_frequencydomainwaveforms_amd.summation import sum_batch
    d1 = multimode
    d2 = source_inputs(M=3e5, mu=10.0, e0=0.2, T=0.02, dt=20.0, eps=1e-2)
    assert np.array_equal(d2["freq"], d1["freq"])
    d3 = dict(d1)
    keep = np.arange(len(d1["m"])) % 2 == 0
    for k in ("m", "n", "ylm_p", "ylm_m"):
        d3[k] = np.asarray(d1[k])[keep]
    d3["amp"] = 0.5 * np.asarray(d1["amp"])[keep]
    freq = torch.as_tensor(d1["freq"], device="cuda")
    nf = len(d1["freq"])
    k0 = int(np.searchsorted(d1["freq"], 0.0))
    cases = [(d, _dev_inputs(d), ModeSumEngine()) for d in (d1, d2, d3)]
    for sym in (True, False):
        single, outs, jobs = [], [], []
        for d, inp, eng in cases:
            eng.launch(inp, freq, None, sym, d["prefactor"], phase="prepare")
            S = torch.full((nf,), np.nan, dtype=torch.complex128, device="cuda")
            eng.launch(inp, freq, torch.view_as_real(S), sym, d["prefactor"], phase="sum")
            single.append(S)
            B = torch.full_like(S, np.nan)
            outs.append(B)
            jobs.append((eng, dict(inp=inp, freq=freq, out=torch.view_as_real(B),
                                   grid_symmetric=sym, scale=d["prefactor"])))
        sum_batch(jobs)
        for (d, inp, eng), S, B in zip(cases, single, outs):
            assert eng.status()
            assert torch.equal(S, B)
    # fused h+/hx (symmetric grid, f >= 0) in a batch == each waveform's own fused sum
    ref, jobs, outs = [], [], []
    for d, inp, eng in cases:
        eng.launch(inp, freq, None, True, d["prefactor"], phase="prepare")
        hp = torch.empty(nf - k0, dtype=torch.complex128, device="cuda")
        hc = torch.empty_like(hp)
        eng.launch(inp, freq, None, True, d["prefactor"], phase="sum",
                   hp=torch.view_as_real(hp), hc=torch.view_as_real(hc), k0=k0)
        ref.append((hp, hc))
        bp, bc = torch.full_like(hp, np.nan), torch.full_like(hc, np.nan)
        outs.append((bp, bc))
        jobs.append((eng, dict(inp=inp, freq=freq, out=None, grid_symmetric=True,
                               scale=d["prefactor"], hp=torch.view_as_real(bp),
                               hc=torch.view_as_real(bc), k0=k0)))
    sum_batch(jobs)
    for (hp, hc), (bp, bc) in zip(ref, outs):
        assert torch.equal(hp, bp) and torch.equal(hc, bc)
    # every member must share the grid size, kind, caustic mode and accumulate flag
    short = freq[1:]
    bad = [jobs[0], (cases[1][2], dict(inp=cases[1][1], freq=short, out=torch.view_as_real(
        torch.empty(nf - 1, dtype=torch.complex128, device="cuda")), grid_symmetric=False,
        scale=1.0))]
    with pytest.raises(_lib.EFDError):
        sum_batch(bad)
    with pytest.raises(ValueError):
        sum_batch([jobs[0]] * (_lib.EFD_BATCH_MAX + 1))
    with pytest.raises(ValueError):
        sum_batch([])

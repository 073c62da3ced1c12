"""GPU parity of the windowed FD likelihood at the reference's own smoke shape (test.sh:3).

    emri_pe.py -Tobs 4.0 -M 3670041.7362535275 -mu 292.0583167470244 -e0 0.5794130830706371
               -eps 1e-2 -dt 10.0 -template fd -nwalkers 16 -ntemps 1 -window_flag 1

The templates and the injection are the FD mode sum convolved with a Hann window of the grid's
length (emri_pe.py:259-263; FDutils.py:66-101 get_fd_windowed, :105-139 get_fd_waveform_fromFD),
on the full 12,623,261-bin grid. The injection is the FD template of the truth (injectFD 1), so
the truth's logL is exactly 0. One red-blue half-step of 8 walkers from the reference's start
distribution goes through Likelihood.__call__ (GPU: mode sum -> windowed_spectrum, one rocFFT
transform pair per walker -> h+/hx -> efd_loglike).

Checker, per walker (all 8):
  - the GPU spectrum S against the oracle's C-restatement spectrum R of the same walker, bin by
    bin (tests/helpers.split_check: 1e-9 max|R| off the folds, 2 D_k at the folds);
  - the oracle's logL: R windowed on the CPU by likelihood_oracle.windowed_polarizations (the
    reference's per-channel get_convolution, through S; pinned to the direct convolution in
    tests/test_oracle_likelihood.py), positive mask, likelihood_oracle.loglike with the oracle's
    own windowed injection as data;
  - tolerance, written out: with r = d - h w and e = ||(d_gpu - d_R)|| + ||(h_gpu - h_R) w|| the
    measured distance between the GPU's and the oracle's windowed channels (h_gpu: the GPU's S
    windowed on the CPU the same way), |ll_gpu - ll_oracle| <= 4 ||r|| e + 2 e^2
    (Cauchy-Schwarz on -2 sum |r|^2); and the GPU's logL equals the CPU loglike of its own
    windowed spectrum to 1e-10 relative (rocFFT vs pocketfft rounding and reduction order).
"""

import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from emri_frequencydomainwaveforms_amd import pe  # noqa: E402
from emri_frequencydomainwaveforms_amd.fdutils import get_sensitivity  # noqa: E402
from oracle import likelihood_oracle as lo  # noqa: E402
from tests.helpers import oracle_spectra, record_parity, split_check  # noqa: E402

TEST_SH = dict(Tobs=4.0, dt=10.0, eps=1e-2, M=3670041.7362535275, mu=292.0583167470244,
               e0=0.5794130830706371)


def _workers():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _windowed_channels(S, window, grid):
    hp, hc = lo.windowed_polarizations(S, window, workers=_workers())
    keep = np.asarray(grid) >= 0.0
    return np.stack([hp[keep], hc[keep]])


def test_windowed_likelihood_test_sh_full_grid():
    s = pe.setup(nwalkers=16, ntemps=1, window_flag=True, **TEST_SH)
    assert s.info["N_f"] == 12623261 and s.half_step == 8 and s.info.get("window") == "hann"
    gen = s.gen
    assert gen.can_fill and not gen.can_pipeline      # the windowed spectrum path
    like = s.like
    batch = s.half_steps()[0]
    ll = like(batch, **s.kwargs)
    assert np.array_equal(like(batch, **s.kwargs), ll)                 # repeatable
    assert like(s.truth6[None, :], **s.kwargs)[0] == 0.0              # injectFD: exact zero
    assert np.all(ll < 0.0)
    # the batched window (groups of WINDOW_GROUP spectra, one transform pair) against one
    # walker at a time: the batched transform's rounding only
    gen.WINDOW_GROUP = 1
    try:
        ll1 = like(batch, **s.kwargs)
    finally:
        del gen.WINDOW_GROUP
    np.testing.assert_allclose(ll1, ll, rtol=1e-12, atol=0.0)
    # the in-place reduction (efd_hann_loglike) against the written templates + efd_loglike
    nch, nb = like._d.shape
    bufs = torch.empty((len(batch), nch, nb), dtype=torch.complex128, device=like.device)
    params14 = s.transform.both_transforms(batch)
    gen.fill_batch([bufs[i] for i in range(len(batch))], params14, **s.kwargs)
    ll_w = np.array([float(like._red.loglike(bufs[i], like._d, like._w_templ)[0])
                     for i in range(len(batch))])
    # the per-bin form reduced inside the transforms (efd_hann_loglike_local, the default)
    # against the mirror-pair form after them (efd_hann_loglike): the differenced correction's
    # float rounding and the channel recombination only; the pair form against the written
    # templates: the reduction order only
    like.HANN_LOCAL, like._hloc = False, None
    try:
        ll_pair = like(batch, **s.kwargs)
    finally:
        del like.HANN_LOCAL
        like._hloc = None
    assert like._hann_local(gen, s.kwargs) is not None
    np.testing.assert_allclose(ll_w, ll_pair, rtol=1e-12, atol=0.0)
    np.testing.assert_allclose(ll, ll_pair, rtol=1e-10, atol=0.0)
    del bufs

    f = s.f_like
    w = lo.noise_factor(f, [get_sensitivity(f)] * 2)
    window = gen.window
    # the oracle's injection, windowed on the CPU
    R0, _, grid, _ = oracle_spectra(s.few, s.truth14, s.kwargs)
    d_R = _windowed_channels(R0, window, grid) * w
    S0 = s.few._spectrum(*s.truth14, **s.kwargs).cpu().numpy()
    d_gpu = _windowed_channels(S0, window, grid) * w
    e_d = np.sqrt(np.sum(np.abs(d_gpu - d_R) ** 2))
    rows, ok_all = [], True
    for i, p in enumerate(params14):
        R, Rps, _, E = oracle_spectra(s.few, p, s.kwargs, perturb_seeds=(20 + i, 2000 + i))
        S = s.few._spectrum(*p, **s.kwargs).cpu().numpy()
        ok, st, _ = split_check(S, R, Rps, E=E)
        np.testing.assert_array_equal(S != 0, R != 0)
        h_R = _windowed_channels(R, window, grid)
        h_gpu = _windowed_channels(S, window, grid)
        ll_R = lo.loglike(h_R, d_R, w)
        ll_self = lo.loglike(h_gpu, d_gpu, w)      # the GPU's own spectrum, windowed on the CPU
        e = e_d + np.sqrt(np.sum(np.abs((h_gpu - h_R) * w) ** 2))
        rn = np.sqrt(np.sum(np.abs(d_R - h_R * w) ** 2))
        bound = 4.0 * rn * e + 2.0 * e * e
        err = abs(ll[i] - ll_R)
        self_rel = abs(ll[i] - ll_self) / abs(ll_self)
        rows.append(dict(walker=i, ll_gpu=float(ll[i]), ll_oracle=float(ll_R),
                         abs_err=float(err), bound=float(bound),
                         err_over_bound=float(err / bound) if bound > 0 else 0.0,
                         ll_self_rel=float(self_rel), spectrum=st))
        ok_all &= ok and err <= bound and self_rel <= 1e-10
    rec = {"config": "test_sh_windowed", "walkers": len(rows), "N_f": s.info["N_f"],
           "p0": s.info["p0"], "rows": rows,
           "max_err_over_bound": max(r["err_over_bound"] for r in rows),
           "max_bound": max(r["bound"] for r in rows),
           "max_ll_self_rel": max(r["ll_self_rel"] for r in rows)}
    record_parity("test_sh_windowed", rec)
    assert ok_all, rec


@pytest.mark.parametrize("n,support", [(100001, (1 / 3, 1.0)), (1577909, (1 / 3, 1.0)),
                                       (100001, (0.45, 0.55)), (100001, (0.0, 1.0))])
def test_hann_convolution_matches_dft_form(n, support):
    """fdutils.HannConvolution (stencil + complex64 power-of-two correction, the path the
    reference's hann(N) window takes) against the exact size-N DFT form windowed_spectrum (FP64
    rocFFT), on a random odd-grid spectrum nonzero on a sub-range (the support the transforms
    are sized for: 2/3, 1/10 and all of the grid; a walker batch of two rows): within 5/N^2 + 1e-13 of max|S| (the first-order form's truncation, ~3.5/N^2 for a
    random-phase spectrum: 3.6e-10 at N = 1e5, 2e-14 at test.sh's 12.6 M); and the one-pass
    kernel (efd_hann_polarizations, one row's correction transform) against efd_polarizations
    of the two-row call's windowed spectrum: the complex64 correction C rounds differently in a
    batch of two rows and in one row (|dC| ~ 2^-23 |C|, |C| <= max|S| ln N, times e/4 =
    1/(4(N-1))), so within 2^-23 ln(N) / (N - 1) + 1e-14 of max|S| (measured 1.0e-12 at
    N = 1e5, 6.7e-14 at 1.58 M)."""
    from scipy.signal.windows import hann
    from emri_frequencydomainwaveforms_amd.fdutils import (HannConvolution, window_multiplier,
                                                           windowed_spectrum)
    rng = np.random.default_rng(n)
    S = rng.normal(size=(2, n)) + 1j * rng.normal(size=(2, n))
    lo, hi = int(support[0] * n), int(support[1] * n)
    S[:, :lo] = 0.0
    S[:, hi:] = 0.0
    S[1] *= 1e-21                                  # spectra are ~1e-18..1e-24
    St = torch.as_tensor(S, device="cuda")
    w = hann(n)
    assert HannConvolution.matches(w) and not HannConvolution.matches(hann(n, sym=False))
    hc = HannConvolution(n, St.device)
    got = hc(St)
    ref = windowed_spectrum(St, window_multiplier(w))
    tol = 5.0 / n**2 + 1e-13
    for r in range(2):
        mx = float(St[r].abs().max())
        assert float((got[r] - ref[r]).abs().max()) <= tol * mx
    from emri_frequencydomainwaveforms_amd import _lib
    lib = _lib.load()
    k0 = n // 2
    tol_pol = 2.0 ** -23 * np.log(n) / (n - 1) + 1e-14
    for r in range(2):
        hp = torch.empty(n - k0, dtype=torch.complex128, device="cuda")
        hc = torch.empty_like(hp)
        hc_ref = torch.empty_like(hp)
        hp_ref = torch.empty_like(hp)
        hcv = HannConvolution(n, St.device)
        hcv.polarizations(St[r].contiguous(), hp, hc, k0, lib)
        Sw = got[r].contiguous()
        _lib.check(lib.efd_polarizations(torch.view_as_real(Sw).data_ptr(), n, k0,
                                         torch.view_as_real(hp_ref).data_ptr(),
                                         torch.view_as_real(hc_ref).data_ptr(), None), "pol", lib)
        torch.cuda.synchronize()
        mx = float(St[r].abs().max())
        assert float((hp - hp_ref).abs().max()) <= tol_pol * mx
        assert float((hc - hc_ref).abs().max()) <= tol_pol * mx


def test_hann_loglike_matches_templates():
    """efd_hann_loglike (the windowed logL reduced without writing templates) against
    efd_hann_polarizations + efd_loglike on the same rows, including an all-zero row (its logL
    is the data-only term) and rows of different supports: 1e-12 relative (reduction order)."""
    from emri_frequencydomainwaveforms_amd import _lib
    from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution
    from emri_frequencydomainwaveforms_amd.reductions import Reducer
    lib = _lib.load()
    n = 200001
    k0 = n // 2
    nb = n - k0
    rng = np.random.default_rng(7)
    S = (rng.normal(size=(3, n)) + 1j * rng.normal(size=(3, n))) * 1e-20
    S[0, : n // 4] = S[0, 3 * n // 4:] = 0.0
    S[1, : 2 * n // 5] = S[1, 3 * n // 5:] = 0.0
    S[2] = 0.0
    St = torch.as_tensor(S, device="cuda")
    d = torch.as_tensor((rng.normal(size=(2, nb)) + 1j * rng.normal(size=(2, nb))) * 1e-20,
                        device="cuda")
    w = torch.as_tensor(rng.uniform(0.5, 2.0, size=(2, nb)), device="cuda")
    hcv = HannConvolution(n, St.device)
    out = torch.empty(3, dtype=torch.float64, device="cuda")
    scr = torch.empty(3 * _lib.EFD_LOGLIKE_SCRATCH, dtype=torch.float64, device="cuda")
    hcv.loglike_batch(St, d, w, k0, out, scr, lib)
    red = Reducer(St.device)
    ref = []
    for r in range(3):
        h = torch.empty((2, nb), dtype=torch.complex128, device="cuda")
        hcv.polarizations(St[r].contiguous(), h[0], h[1], k0, lib)
        ref.append(float(red.loglike(h, d, w)[0]))
    got = out.cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=0.0)
    np.testing.assert_allclose(got[2], float(red.loglike(None, d, w)[0]), rtol=1e-12, atol=0.0)


@pytest.mark.parametrize("n,m", [(1000001, 1 << 21), (12623261, 1 << 24)])
def test_hann_loglike_local(n, m):
    """efd_hann_loglike_local (the windowed logL in its per-bin form, reduced inside the inverse
    column pass from the differenced correction) against efd_hann_loglike (the mirror-pair form
    after the transforms) on the same rows and d, w (the same weight on both channels), rows of
    different supports and an all-zero row: 1e-11 relative (the correction's float rounding,
    ~1e-7 of a term ~1e-6 of max|S|, and the channel recombination). Its emit mode against
    HannConvolution's own windowed spectrum (the plain pipeline, complex128 stencil) times the
    weight, every bin (the wrapped bin nf-1 - first and the mirror layout included): within
    2^-23 ln(n) / (n - 1) + 1e-14 of max|S| max w (tol_pol above); and the emitted data's logL
    against the same spectrum is exactly 0."""
    from emri_frequencydomainwaveforms_amd import _lib
    from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution
    lib = _lib.load()
    k0 = (n - 1) // 2
    nb = n - k0
    rng = np.random.default_rng(n % 997)
    rows = 3
    S = torch.zeros((rows, n), dtype=torch.complex128, device="cuda")
    for r, (a, b) in enumerate([(0.45, 0.55), (0.43, 0.56)]):
        lo_, hi_ = int(a * n), int(b * n)
        S[r, lo_:hi_] = torch.complex(torch.randn(hi_ - lo_, dtype=torch.float64, device="cuda"),
                                      torch.randn(hi_ - lo_, dtype=torch.float64,
                                                  device="cuda")) * 1e-21
    d = torch.as_tensor((rng.normal(size=(2, nb)) + 1j * rng.normal(size=(2, nb))) * 1e-20,
                        device="cuda")
    w1 = rng.uniform(0.5, 2.0, size=nb)
    w1[0] = 0.0                                  # a masked bin (the likelihood's start_ind)
    w = torch.as_tensor(np.stack([w1, w1]), device="cuda")
    hcv = HannConvolution(n, S.device)
    assert hcv.local_ok(d, w, k0)
    assert not hcv.local_ok(d, torch.as_tensor(np.stack([w1, w1 * 1.5]), device="cuda"), k0)
    local = hcv.local_data(d, w, k0)
    assert local[2] == k0                        # odd grid: k0 is its own mirror
    out = torch.empty(rows, dtype=torch.float64, device="cuda")
    scr = torch.empty(rows * _lib.EFD_HANN_LOCAL_PARTIALS, dtype=torch.float64, device="cuda")
    assert hcv.loglike_local(S, local, out, scr, lib)
    assert lib.efd_hann_loglike_local_partials(m) <= _lib.EFD_HANN_LOCAL_PARTIALS
    ref = torch.empty(rows, dtype=torch.float64, device="cuda")
    scr2 = torch.empty(rows * _lib.EFD_LOGLIKE_SCRATCH, dtype=torch.float64, device="cuda")
    hcv.loglike_batch(S, d, w, k0, ref, scr2, lib)
    _, _, mm = hcv.transform(S, lib)
    assert mm == m
    np.testing.assert_allclose(out.cpu().numpy(), ref.cpu().numpy(), rtol=1e-11, atol=0.0)
    # emit: wl S_w per bin, against the plain pipeline's windowed spectrum
    tol = 2.0 ** -23 * np.log(n) / (n - 1) + 1e-14
    wl, kself = local[1], local[2]
    for r in range(2):
        row = S[r:r + 1].contiguous()
        e = hcv.local_emit(row, wl, kself, lib)
        Sw = hcv(row)[0]
        mx = float(row.abs().max()) * float(wl.max())
        assert float((e[:n] - wl * Sw).abs().max()) <= tol * mx
        assert complex(e[n]) == complex(e[kself])
        zero = torch.empty(1, dtype=torch.float64, device="cuda")
        assert hcv.loglike_local(row, (e, wl, kself), zero, scr, lib)
        assert float(zero[0]) == 0.0


@pytest.mark.parametrize("n,support,rows,m", [
    (1000001, (0.4, 0.9), 3, 1 << 21), (2000001, (0.3, 0.9), 2, 1 << 22),
    (4000001, (0.3, 0.9), 2, 1 << 23), (12623261, (0.43, 0.57), 2, 1 << 24),
    (12623261, (0.2, 0.8), 2, 1 << 25),
    # the most rows a call takes (EFD_HANN_ROWS_MAX) and a lone all-zero row
    (12623261, (0.45, 0.55), 16, 1 << 24), (12623261, (0.45, 0.55), 1, 1 << 24)])
def test_four_step_convolution(n, support, rows, m):
    """efd_hann_convolve (the four-step complex64 FFT pipeline, every split it has: m = 2^21,
    2^22, 2^23 and 2^25 as R x 8192, R = 256, 512, 1024 and 4096, and 2^24 as 1024 x 16384;
    round 6 deleted the rejected variants and their switches) against
    the same correction on hipFFT transforms and against an exact complex128 convolution
    (torch.fft on the zero-padded support): C within 1e-5 of max|C| in both comparisons (float
    transforms: ~1e-6; the correction needs ~3 digits), rows of different supports, one of
    them all zero."""
    _four_step_check(n, support, rows, m, 16384 if m == 1 << 24 else 8192)


def _four_step_check(n, support, rows, m, cols):
    from emri_frequencydomainwaveforms_amd import _lib
    from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution
    lib = _lib.load()
    assert lib.efd_hann_four_step_cols(m) == cols
    rng = np.random.default_rng(n % 1000)
    S = torch.zeros((rows, n), dtype=torch.complex128, device="cuda")
    lo, hi = int(support[0] * n), int(support[1] * n)
    for r in range(rows - 1):
        a, b = lo + 1000 * r, hi - 7 * r
        S[r, a:b] = torch.complex(torch.randn(b - a, dtype=torch.float64, device="cuda"),
                                  torch.randn(b - a, dtype=torch.float64, device="cuda")) * 1e-21
    hcv = HannConvolution(n, S.device)
    C4 = hcv.correction(S, lib)
    assert hcv.size_for(n, hi - lo) == m and hcv._four(m), m
    hcv.four_step = False
    C_fft = hcv.correction(S, lib)
    hcv.four_step = True
    # exact: the circular convolution with K as one complex128 linear convolution
    k = torch.arange(-(n - 1), n, device="cuda", dtype=torch.int64)
    mm = torch.remainder(k, n).to(torch.float64)
    zero = mm == 0
    K = torch.complex(torch.where(zero, torch.zeros_like(mm), (np.pi / n) / torch.tan(np.pi * mm / n)),
                      torch.where(zero, torch.full_like(mm, np.pi * (n - 1) / n),
                                  torch.full_like(mm, -np.pi / n)))
    L = 1 << (3 * n - 2).bit_length()
    Kf = torch.fft.fft(K, L)
    for r in range(rows - 1):
        # K at lag u = k - j in (-n, n) sits at u + n - 1, so C[k] = (S * K)[k + n - 1]
        C = torch.fft.ifft(torch.fft.fft(S[r], L) * Kf)[n - 1:2 * n - 1]
        scale = float(C.abs().max())
        assert float((C4[r] - C_fft[r]).abs().max()) <= 1e-5 * scale
        assert float((C4[r] - C).abs().max()) <= 1e-5 * scale
        del C
    assert float(C4[-1].abs().max()) == 0.0 and float(C_fft[-1].abs().max()) == 0.0


def test_extent_from_lane_ranges():
    """The extent scan restricted to each row's lane range (efd_modesum_lane_ranges after
    GenerateEMRIWaveform.spectrum_batch) gives bitwise the full scan's scale, support and
    transformed rows; the lane range covers every nonzero bin (and its mirror)."""
    from emri_frequencydomainwaveforms_amd import _lib
    from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution
    s = pe.setup(nwalkers=16, ntemps=1, window_flag=True, **TEST_SH)
    lib = _lib.load()
    params = s.transform.both_transforms(s.half_steps()[0][:3])
    n = s.info["N_f"]
    S = torch.empty((3, n), dtype=torch.complex128, device="cuda")
    lanes = torch.empty((3, 2), dtype=torch.int32, device="cuda")
    s.few.spectrum_batch(params, S, lanes=lanes, **s.kwargs)
    torch.cuda.synchronize()
    hcv = HannConvolution(n, S.device)
    Y1, info1, m1 = hcv.transform(S, lib, lanes)
    Y1, info1 = Y1.clone(), info1.clone()
    Y0, info0, m0 = hcv.transform(S, lib)
    assert m1 == m0 and torch.equal(info1, info0) and torch.equal(Y1, Y0)
    ln = lanes.cpu().numpy()
    nz = (S != 0).cpu().numpy()
    for r in range(3):
        lo, hi = int(ln[r, 0]), int(ln[r, 1])
        k = np.nonzero(nz[r])[0]
        assert len(k) and k.min() >= min(lo, n - hi) and k.max() < max(hi, n - lo)
    # the host's bound from the lane ranges (what the likelihood chooses m from without a
    # synchronisation) covers every row's support and gives the same transform length here
    ext = info0[:, 1:3].cpu().numpy()
    sup = int((ext[:, 1] - ext[:, 0]).max())
    bound = HannConvolution.lane_support(ln, n)
    assert bound >= sup and hcv.size_for(n, bound) == m0
    Y2, info2, m2 = hcv.transform(S, lib, lanes, support=bound)
    assert m2 == m0 and torch.equal(info2, info0) and torch.equal(Y2, Y0)
    # lanes_host: the same ranges copied to pinned memory before the sums
    lh = torch.empty((3, 2), dtype=torch.int32, pin_memory=True)
    s.few.spectrum_batch(params, S, lanes=lanes, lanes_host=lh, check=False, **s.kwargs)
    s.few.lanes_ready()
    assert np.array_equal(lh.numpy(), ln)
    s.few.check_batch()


def test_windowed_likelihood_short_grid_exact_path():
    """A short grid (Tobs = 0.02 yr, N = 63,115 bins): the first-order Hann form would be off by
    ~3.5-5 / N^2 ~ 1e-9 of max|S| here, so the likelihood must take the exact size-N transform
    pair (windowed_spectrum) instead (HannConvolution.applies). Checked: the path taken, and
    each walker's logL against the CPU loglike of the GPU's own spectrum windowed by the
    reference's convolution (likelihood_oracle.windowed_polarizations) at 1e-10 relative; the
    injection's logL is 0 exactly."""
    from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution
    s = pe.setup(Tobs=0.02, dt=10.0, eps=1e-2, M=1e5, mu=10.0, nwalkers=8, ntemps=1,
                 window_flag=True)
    n = s.info["N_f"]
    assert n == 63117 and not HannConvolution.applies(n) and HannConvolution.applies(12623261)
    gen = s.gen
    assert gen._hann is None and not gen.can_fill_batch     # the exact transform pair
    like = s.like
    batch = s.half_steps()[0]
    ll = like(batch, **s.kwargs)
    assert like(s.truth6[None, :], **s.kwargs)[0] == 0.0
    f = s.f_like
    w = lo.noise_factor(f, [get_sensitivity(f)] * 2)
    window = gen.window
    grid = s.few.waveform_generator.create_waveform.frequency
    grid = grid.cpu().numpy() if hasattr(grid, "detach") else np.asarray(grid)
    S0 = s.few._spectrum(*s.truth14, **s.kwargs).cpu().numpy()
    d_gpu = _windowed_channels(S0, window, grid) * w
    for i, p in enumerate(s.transform.both_transforms(batch)):
        S = s.few._spectrum(*p, **s.kwargs).cpu().numpy()
        ll_self = lo.loglike(_windowed_channels(S, window, grid), d_gpu, w)
        assert abs(ll[i] - ll_self) <= 1e-10 * abs(ll_self), (i, ll[i], ll_self)

"""The reference drivers' call surface end to end on the GPU (emri_pe.py:86-105, 212-271,
381-414; check_mode_by_mode.py:69-83, 226-250): GenerateEMRIWaveform -> get_fd_waveform_fromFD
-> Likelihood, with the HIP path underneath and the numpy oracle as the checker.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from emri_frequencydomainwaveforms_amd.fdutils import get_fd_waveform_fromFD, get_sensitivity  # noqa: E402,E501
from emri_frequencydomainwaveforms_amd.likelihood import Likelihood  # noqa: E402
from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t  # noqa: E402
from emri_frequencydomainwaveforms_amd.waveform import GenerateEMRIWaveform  # noqa: E402
from oracle import fd_oracle, likelihood_oracle as lo  # noqa: E402

SUM_KW = dict(pad_output=True, output_type="fd", odd_len=True)
M, MU, E0, T, DT = 3e5, 10.0, 0.3, 0.02, 20.0


@pytest.fixture(scope="module")
def setup():
    p0 = get_p_at_t(EMRIInspiral(), 0.99 * T, [M, MU, 0.0, E0, 1.0])
    params = np.array([M, MU, 0.0, p0, E0, 1.0, 1.0, 0.5, 0.3, 0.8, 1.1, 0.2, 0.0, 0.4])
    kw = dict(T=T, dt=DT, eps=1e-2)
    gen = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux", sum_kwargs=SUM_KW,
                               use_gpu=True, return_list=False)
    gen_list = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux", sum_kwargs=SUM_KW,
                                    use_gpu=True, return_list=True)
    return params, kw, gen, gen_list


def test_generator_contract(setup):
    params, kw, gen, gen_list = setup
    S = gen(*params, **kw)
    hp, hc = gen_list(*params, **kw)
    freq = gen.waveform_generator.create_waveform.frequency
    assert S.shape == freq.shape and freq.numel() % 2 == 1             # odd two-sided grid
    # check_mode_by_mode.py:247: S = h+ - i hx
    assert torch.equal(hp - 1j * hc, S) or \
        (hp - 1j * hc - S).abs().max().item() <= 1e-15 * S.abs().max().item()
    # mask_positive (emri_pe.py:241) keeps f >= 0
    Sp = gen(*params, mask_positive=True, **kw)
    pos = freq >= 0
    assert torch.equal(Sp, S[pos])
    hpp, hcp = gen_list(*params, mask_positive=True, **kw)
    assert torch.equal(hpp, hp[pos]) and torch.equal(hcp, hc[pos])
    # the spectrum equals the oracle's for the same host inputs: source-frame viewing angle
    # theta = arccos(-R.S) of the sky position (qS, phiS) = (0.5, 0.3) and spin direction
    # (qK, phiK) = (0.8, 1.1), detector-frame rotation exp(-2 i psi) and 1 / dist in the scale
    from emri_frequencydomainwaveforms_amd.constants import Gpc, MRSUN_SI
    wg = gen.waveform_generator
    theta_ref = np.arccos(-(np.sin(0.5) * np.cos(0.3) * np.sin(0.8) * np.cos(1.1)
                            + np.sin(0.5) * np.sin(0.3) * np.sin(0.8) * np.sin(1.1)
                            + np.cos(0.5) * np.cos(0.8)))
    theta, phi, rot = gen._angles(0.5, 0.3, 0.8, 1.1)
    assert abs(theta - theta_ref) <= 1e-14 and phi == -np.pi / 2 and abs(abs(rot) - 1) < 1e-15
    d = wg.prepare(M, MU, params[3], E0, theta, phi, 1.0, params[11], params[13], T, 1e-2)
    K = len(d["m"])
    assert K > 20
    R = fd_oracle.fd_modesum(d["t"], d["teuk"].T, d["Phi_phi"], d["Phi_r"], d["f_phi"],
                             d["f_r"], d["m"], d["n"], d["ylms"][:K], d["ylms"][K:],
                             freq.cpu().numpy(), rot * MU * MRSUN_SI / (1.0 * Gpc))
    Sh = S.cpu().numpy()
    assert np.abs(Sh - R).max() <= 1e-9 * np.abs(R).max()
    np.testing.assert_array_equal(Sh != 0, R != 0)


def test_f_arr_downsampled(setup):
    params, kw, gen, _ = setup
    S = gen(*params, **kw).cpu().numpy()
    freq = gen.waveform_generator.create_waveform.frequency.cpu().numpy()
    nz = np.abs(S[freq >= 0]) > 1e-50 * np.abs(S).max()
    p_freq = np.linspace(0.0, freq[freq >= 0][nz].max() * 1.01, num=int(nz.sum() / 20))
    f_arr = np.hstack((-p_freq[::-1][:-1], p_freq))                  # emri_pe.py:333-349
    Sd = gen(*params, f_arr=torch.as_tensor(f_arr, device="cuda"), **kw)
    assert Sd.numel() == len(f_arr)
    assert np.array_equal(gen.waveform_generator.create_waveform.frequency.cpu().numpy(), f_arr)
    # each downsampled bin equals a full evaluation of the same sum there (grid independence)
    Sd2 = gen(*params, f_arr=f_arr, **kw)
    assert torch.equal(Sd, Sd2)


def test_emri_pe_likelihood_path(setup):
    params, kw, gen, gen_list = setup
    hp, hc = gen_list(*params, **kw)
    freq = gen_list.waveform_generator.create_waveform.frequency
    pos = freq >= 0
    fd_gen = get_fd_waveform_fromFD(gen_list, pos, DT)
    assert fd_gen.can_fill
    sig = fd_gen(*params, **kw)
    assert torch.equal(sig[0], hp[pos]) and torch.equal(sig[1], hc[pos])
    f_arr = freq[pos].cpu().numpy()

    like = Likelihood(fd_gen, 2, f_arr=f_arr, use_gpu=True, subset=2)
    like.inject_signal(data_stream=sig, noise_fn=[get_sensitivity, get_sensitivity],
                       noise_kwargs=[{}, {}])
    walkers = np.stack([params, params, params])
    walkers[1, 0] *= 1.0 + 1e-5
    walkers[2, 4] += 1e-3
    assert fd_gen.can_pipeline
    # default: the likelihood fused into the walkers' batched mode sum (no template written);
    # the injection walker's residual is exactly 0 (same h, same rounding as efd_loglike)
    llf = like(walkers, **kw)
    assert llf[0] == 0.0
    assert np.all(llf[1:] < 0.0)
    like.fused_likelihood = False      # templates through a buffer + efd_loglike, 4 streams
    ll = like(walkers, **kw)
    assert ll[0] == 0.0
    np.testing.assert_allclose(llf, ll, rtol=1e-12, atol=0.0)   # reduction order differs
    like.num_streams, like._pipe = 1, None   # one template in flight at a time: same values
    np.testing.assert_array_equal(like(walkers, **kw), ll)

    # generic path (template returns channels) gives bitwise the unfused values
    like_g = Likelihood(lambda *a, **k: fd_gen(*a, **k), 2, f_arr=f_arr, use_gpu=True)
    like_g.inject_signal(data_stream=sig, noise_fn=[get_sensitivity, get_sensitivity],
                         noise_kwargs=[{}, {}])
    np.testing.assert_array_equal(like_g.get_ll(walkers, **kw), like.get_ll(walkers, **kw))

    # against the oracle on host copies
    w = lo.noise_factor(f_arr, [get_sensitivity(f_arr)] * 2)
    dh = np.array([s.cpu().numpy() for s in sig]) * w
    h1 = np.array([c.cpu().numpy() for c in fd_gen(*walkers[1], **kw)])
    ref = lo.loglike(h1, dh, w)
    assert abs(ll[1] - ref) <= 1e-12 * abs(ref)

    # non_zero_mask (emri_pe.py:245): folded into the template weight on the fused path
    nzm = sig[0].abs() > 1e-50
    fd_nz = get_fd_waveform_fromFD(gen_list, pos, DT, non_zero_mask=nzm)
    like_nz = Likelihood(fd_nz, 2, f_arr=f_arr, use_gpu=True)
    like_nz.inject_signal(data_stream=sig, noise_fn=[get_sensitivity] * 2, noise_kwargs=[{}, {}])
    like_nzg = Likelihood(lambda *a, **k: fd_nz(*a, **k), 2, f_arr=f_arr, use_gpu=True)
    like_nzg.inject_signal(data_stream=sig, noise_fn=[get_sensitivity] * 2,
                           noise_kwargs=[{}, {}])
    np.testing.assert_allclose(like_nz.get_ll(walkers, **kw), like_nzg.get_ll(walkers, **kw),
                               rtol=1e-12, atol=0.0)
    like_nz.fused_likelihood = False
    np.testing.assert_array_equal(like_nz.get_ll(walkers, **kw), like_nzg.get_ll(walkers, **kw))


def test_fused_likelihood_many_walkers(setup):
    """More walkers than two fused groups (slot reuse across groups, a partial last group):
    efd_modesum_sum_loglike's values equal the template-buffer path to 1e-12, repeat bitwise,
    and the fused call rejects bad shapes host-side."""
    from emri_frequencydomainwaveforms_amd import _lib
    from emri_frequencydomainwaveforms_amd.summation import sum_batch_loglike
    params, kw, gen, gen_list = setup
    freq = gen_list.waveform_generator.create_waveform.frequency
    pos = freq >= 0
    fd_gen = get_fd_waveform_fromFD(gen_list, pos, DT)
    sig = fd_gen(*params, **kw)
    f_arr = freq[pos].cpu().numpy()
    like = Likelihood(fd_gen, 2, f_arr=f_arr, use_gpu=True)
    like.inject_signal(data_stream=sig, noise_fn=[get_sensitivity] * 2, noise_kwargs=[{}, {}])
    rng = np.random.default_rng(5)
    walkers = np.stack([params] * 19)
    walkers[1:, 0] *= 1.0 + 1e-5 * rng.standard_normal(18)
    walkers[1:, 4] += 1e-3 * rng.standard_normal(18)
    walkers[1:, 11] += 0.1 * rng.standard_normal(18)
    llf = like.get_ll(walkers, **kw)
    assert llf[0] == 0.0 and np.all(llf[1:] < 0.0)
    np.testing.assert_array_equal(like.get_ll(walkers, **kw), llf)
    like.fused_likelihood = False
    np.testing.assert_allclose(llf, like.get_ll(walkers, **kw), rtol=1e-12, atol=0.0)
    # argument errors: wrong data shape (host-side ValueError), unprepared mix of grids (C ABI)
    jobs = like._fused["prep"].last_jobs[:2]
    out = torch.empty(2, dtype=torch.float64, device="cuda")
    with pytest.raises(ValueError):
        sum_batch_loglike(jobs, like._d[:, 1:].contiguous(), like._w_templ, out)
    bad_args = _lib.ModesumArgs.from_buffer_copy(jobs[0][1]["_args"])
    bad_args.accumulate = 1
    bad = [(jobs[0][0], dict(jobs[0][1], _args=bad_args)), jobs[1]]
    with pytest.raises(_lib.EFDError):
        sum_batch_loglike(bad, like._d, like._w_templ, out)
    # a failure inside the second group's flush, after its upload and preparation are queued:
    # get_ll raises only once every group stream is idle, and the next call is unaffected
    # (both host paths: one native call per group, flush_loglike, and the Python steps, flush)
    like.fused_likelihood = True
    Bp = like._fused["prep"]
    for native, name in ((True, "flush_loglike"), (False, "flush")):
        like.FUSED_NATIVE_GROUP = native
        orig, seen = getattr(Bp, name), []

        def flaky(*a, **k):
            r = orig(*a, **k)
            seen.append(r if native else r[0])
            if len(seen) == 2:
                raise RuntimeError("injected flush failure")
            return r

        setattr(Bp, name, flaky)
        try:
            with pytest.raises(RuntimeError, match="injected"):
                like.get_ll(walkers, **kw)
            assert len(seen) == 2 and seen[0] != seen[1]
            assert all(g["stream"].query() for g in Bp.groups)
        finally:
            delattr(Bp, name)
            del like.FUSED_NATIVE_GROUP
        np.testing.assert_array_equal(like.get_ll(walkers, **kw), llf)


def test_fused_likelihood_large_group(setup):
    """One fused group of 32 walkers (BatchPreparer.GROUP_MAX > EFD_BATCH_MAX: one staging copy
    and upload, the preparation and sum launches 16 walkers at a time) gives bitwise the
    log-likelihoods of groups of at most 16."""
    params, kw, gen, gen_list = setup
    freq = gen_list.waveform_generator.create_waveform.frequency
    pos = freq >= 0
    fd_gen = get_fd_waveform_fromFD(gen_list, pos, DT)
    sig = fd_gen(*params, **kw)
    like = Likelihood(fd_gen, 2, f_arr=freq[pos].cpu().numpy(), use_gpu=True)
    like.inject_signal(data_stream=sig, noise_fn=[get_sensitivity] * 2, noise_kwargs=[{}, {}])
    rng = np.random.default_rng(9)
    walkers = np.stack([params] * 27)
    walkers[1:, 0] *= 1.0 + 1e-5 * rng.standard_normal(26)
    walkers[1:, 11] += 0.1 * rng.standard_normal(26)
    ref = like.get_ll(walkers, **kw)
    like.FUSED_GROUP = 32
    like._fused = None
    got = like.get_ll(walkers, **kw)
    assert like._fused["prep"].group == 32
    np.testing.assert_array_equal(got, ref)
    assert got[0] == 0.0


def test_spectrum_matches_oracle_through_api(setup):
    params, kw, gen, _ = setup
    wg = gen.waveform_generator
    S = wg.spectrum(M, MU, params[3], E0, np.pi / 3, -np.pi / 2, 1.0, 0.2, 0.4, dt=DT, T=T,
                    eps=1e-2).cpu().numpy()
    d = wg.prepare(M, MU, params[3], E0, np.pi / 3, -np.pi / 2, 1.0, 0.2, 0.4, T, 1e-2)
    K = len(d["m"])
    from emri_frequencydomainwaveforms_amd.constants import Gpc, MRSUN_SI
    freq = wg.create_waveform.frequency.cpu().numpy()
    # the upstream's own orbital frequencies at the knots (native trajectory or FEW's formula)
    R = fd_oracle.fd_modesum(d["t"], d["teuk"].T, d["Phi_phi"], d["Phi_r"], d["f_phi"],
                             d["f_r"], d["m"], d["n"], d["ylms"][:K], d["ylms"][K:], freq,
                             MU * MRSUN_SI / Gpc)
    assert np.abs(S - R).max() <= 1e-9 * np.abs(R).max()


def test_pipelined_likelihood_asymmetric_grid(setup):
    """An f_arr that is not mirror-symmetric takes the pipeline's spectrum + efd_polarizations
    branch on the slot streams: same values as the one-at-a-time generic path."""
    params, kw, gen, gen_list = setup
    S = gen(*params, **kw).cpu().numpy()
    freq = gen.waveform_generator.create_waveform.frequency.cpu().numpy()
    nz = np.abs(S[freq >= 0]) > 1e-50 * np.abs(S).max()
    fmax = freq[freq >= 0][nz].max() * 1.01
    # more bins on the positive side than the negative one: sorted, odd length, not symmetric
    f_arr = np.hstack((-np.linspace(fmax, 0.0, 40)[:-1], np.linspace(0.0, fmax, 61)))
    kw2 = dict(kw, f_arr=f_arr)
    gen_list(*params, **kw2)
    assert not gen_list.waveform_generator.create_waveform._sym
    pos = f_arr >= 0
    fd_gen = get_fd_waveform_fromFD(gen_list, pos, DT)
    assert fd_gen.can_pipeline
    sig = fd_gen(*params, **kw2)
    walkers = np.stack([params] * 5)
    walkers[1, 0] *= 1.0 + 1e-5
    walkers[2, 4] += 1e-3
    walkers[3, 11] += 0.1
    walkers[4, 3] += 1e-4
    like = Likelihood(fd_gen, 2, f_arr=f_arr[pos], use_gpu=True)
    like.inject_signal(data_stream=sig, noise_fn=[get_sensitivity] * 2, noise_kwargs=[{}, {}])
    ll = like.get_ll(walkers, **kw2)
    like_g = Likelihood(lambda *a, **k: fd_gen(*a, **k), 2, f_arr=f_arr[pos], use_gpu=True)
    like_g.inject_signal(data_stream=sig, noise_fn=[get_sensitivity] * 2, noise_kwargs=[{}, {}])
    np.testing.assert_array_equal(like_g.get_ll(walkers, **kw2), ll)
    assert ll[0] == 0.0 and np.all(ll[1:] < 0.0)


def test_generate_batch_matches_calls(setup):
    """GenerateEMRIWaveform.generate_batch (the vectorised scan: pooled host upstream, groups of
    BATCH_GROUP on the device) writes, bitwise, each row's [h+, hx] over f >= 0 as the
    one-at-a-time list call with mask_positive=True; a ragged last group and a second call on
    the reused groups included."""
    params, kw, gen, gen_list = setup
    rng = np.random.default_rng(11)
    rows = np.repeat(params[None, :], 5, axis=0)
    rows[:, 0] *= 1.0 + 1e-3 * rng.normal(size=5)          # distinct M
    rows[:, 4] = E0 + 0.01 * rng.normal(size=5)            # distinct e0
    rows[:, 11] = rng.uniform(0, 2 * np.pi, size=5)         # distinct Phi_phi0
    gen_list.BATCH_GROUP = 2                                # groups of 2, 2, 1
    try:
        ref = [torch.stack(gen_list(*r, mask_positive=True, **kw)) for r in rows]
        out = torch.empty((5,) + tuple(ref[0].shape), dtype=torch.complex128, device="cuda")
        for _ in range(2):
            out.zero_()
            gen_list.generate_batch(rows, out, **kw)
            torch.cuda.synchronize()
            for b in range(5):
                assert torch.equal(out[b], ref[b]), b
    finally:
        del gen_list.BATCH_GROUP
    with pytest.raises(ValueError):
        gen_list.generate_batch(rows, out[:4], **kw)
    # spectrum_batch: the two-sided S of each row (the windowed templates' input), bitwise the
    # spectrum path's; stale buffer contents are overwritten everywhere
    refS = [gen_list._spectrum(*r, **kw).clone() for r in rows]
    S = torch.full((5, refS[0].numel()), complex(np.nan, np.nan), dtype=torch.complex128,
                   device="cuda")
    gen_list.BATCH_GROUP = 3
    try:
        gen_list.spectrum_batch(rows, S, **kw)
    finally:
        del gen_list.BATCH_GROUP
    torch.cuda.synchronize()
    for b in range(5):
        assert torch.equal(S[b], refS[b]), b
    with pytest.raises(ValueError):
        gen_list.spectrum_batch(rows, S[:4], **kw)
    # lane ranges over several groups, gathered beside the sums and copied to the host early
    # (lanes_host, lanes_ready), with the status read afterwards (check=False, check_batch)
    lanes = torch.empty((5, 2), dtype=torch.int32, device="cuda")
    lh = torch.full((5, 2), -7, dtype=torch.int32, pin_memory=True)
    S.fill_(complex(np.nan, np.nan))
    gen_list.BATCH_GROUP = 2
    try:
        gen_list.spectrum_batch(rows, S, lanes=lanes, lanes_host=lh, check=False, **kw)
        gen_list.lanes_ready()
        got = lh.numpy().copy()
        gen_list.check_batch()
    finally:
        del gen_list.BATCH_GROUP
    torch.cuda.synchronize()
    assert np.array_equal(got, lanes.cpu().numpy()) and (got[:, 1] > got[:, 0]).all()
    for b in range(5):
        assert torch.equal(S[b], refS[b]), b
    with pytest.raises(ValueError):   # lanes_host must be pinned
        gen_list.spectrum_batch(rows, S, lanes=lanes, lanes_host=torch.empty((5, 2),
                                dtype=torch.int32), **kw)

"""The C++ host upstream (csrc/emrifd_host.cpp, emrifd_modes.cpp) against the numpy/scipy
stand-ins it restates (trajectory.py, amplitude.py). STAND-IN PHYSICS, NOT FEW.

- trajectory: the same ODE and integrator (scipy RK45's tableau, step control, dense output,
  terminal separatrix event). At rtol = 1e-12 the phase components' error estimates sit at the
  rounding floor, so the accepted steps differ with the summation order of the error estimate
  (numpy's BLAS dot vs the C++ loop); the knot count and end agree, and the two trajectories
  agree as functions: a cubic spline through the native knots reproduces the scipy knots' p, e
  to 1e-10 and the phases to 1e-9 relative;
- get_p_at_t: the same Brent root, p0 to 1e-13;
- amplitudes and ModeSelector(eps): the identical kept mode set and amplitudes to 1e-14, over
  sources, viewing angles and eps = 1e-2 / 1e-5;
- the generator's prepare() on the native path against the numpy path, and prefetch() of a
  walker batch (thread pool) giving the same dicts as serial prepare() calls.
"""

import threading

import numpy as np
import pytest
from scipy.interpolate import CubicSpline

from emri_frequencydomainwaveforms_amd import _lib
from emri_frequencydomainwaveforms_amd.amplitude import ModeSelector, RomanAmplitude
from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
from emri_frequencydomainwaveforms_amd.ylm import GetYlms

SOURCES = [(1e6, 10.0, 0.35, 2.0), (1e5, 1.0, 0.1, 1.0), (1e7, 100.0, 0.6, 1.0),
           (3e5, 10.0, 0.3, 0.02)]


@pytest.fixture(scope="module")
def trajs():
    return EMRIInspiral(), EMRIInspiral(backend="python")


def test_native_backend_is_default(trajs):
    assert trajs[0].backend == "native" and trajs[1].backend == "python"


@pytest.mark.parametrize("src", SOURCES)
def test_trajectory_and_p_at_t_match_scipy(trajs, src):
    M, mu, e0, T = src
    tn, tp = trajs
    pn = get_p_at_t(tn, 0.99 * T, [M, mu, 0.0, e0, 1.0])
    pp = get_p_at_t(tp, 0.99 * T, [M, mu, 0.0, e0, 1.0])
    assert abs(pn - pp) <= 1e-13 * pp
    a = tn(M, mu, 0.0, pp, e0, 1.0, Phi_phi0=0.3, Phi_r0=1.1, T=T)
    b = tp(M, mu, 0.0, pp, e0, 1.0, Phi_phi0=0.3, Phi_r0=1.1, T=T)
    assert abs(len(a[0]) - len(b[0])) <= 2
    assert abs(a[0][-1] - b[0][-1]) <= 1e-10 * b[0][-1]
    tt = b[0][1:-1]
    for j, tol in ((1, 1e-10), (2, 1e-10), (4, 1e-9), (6, 1e-9)):
        s = CubicSpline(a[0], a[j])
        assert np.max(np.abs(s(tt) - b[j][1:-1])) <= tol * np.max(np.abs(b[j])), j
    # the knot frequencies of with_frequencies are the fundamental frequencies at the knots
    from emri_frequencydomainwaveforms_amd.constants import MTSUN_SI
    from emri_frequencydomainwaveforms_amd.frequencies import get_fundamental_frequencies
    t, p, e, _, _, fphi, fr = tn.with_frequencies(M, mu, 0.0, pp, e0, 1.0, T=T)
    op, _, orr = get_fundamental_frequencies(0.0, p, e, 0.0)
    np.testing.assert_allclose(fphi, op / (2 * np.pi * M * MTSUN_SI), rtol=1e-13)
    np.testing.assert_allclose(fr, orr / (2 * np.pi * M * MTSUN_SI), rtol=1e-13)


@pytest.mark.parametrize("theta", [1.0, 0.3, 2.5])
@pytest.mark.parametrize("eps", [1e-2, 1e-5])
def test_modes_match_numpy(trajs, theta, eps):
    lib = _lib.load()
    amp = RomanAmplitude()
    ylms = GetYlms(assume_positive_m=True)(amp.l_arr, amp.m_arr, theta, -np.pi / 2)
    for M, mu, e0, T in SOURCES[:3]:
        p0 = get_p_at_t(trajs[0], 0.99 * T, [M, mu, 0.0, e0, 1.0])
        t, p, e, *_ = trajs[0](M, mu, 0.0, p0, e0, 1.0, T=T)
        kp, Ap = amp.select(p, e, ylms, eps)                 # numpy: __call__ + ModeSelector
        kn, An = amp.select(p, e, ylms, eps, lib=lib)
        np.testing.assert_array_equal(kn, kp)
        assert np.abs(An - Ap).max() <= 1e-14 * np.abs(Ap).max()
        np.testing.assert_array_equal(kp, ModeSelector(amp.m0mask)(amp(p, e), ylms, None, eps=eps))


def waveform_nbytes(d):
    from emri_frequencydomainwaveforms_amd.waveform import _nbytes
    return _nbytes(d)


def _bare_generator(backend):
    """The FD generator's host half only (no GPU needed)."""
    from emri_frequencydomainwaveforms_amd.waveform import FastSchwarzschildEccentricFlux
    wg = FastSchwarzschildEccentricFlux.__new__(FastSchwarzschildEccentricFlux)
    wg.inspiral_generator = EMRIInspiral(backend=backend)
    wg.amplitude_generator = RomanAmplitude()
    wg.ylm_gen = GetYlms(assume_positive_m=True)
    wg.mode_selector = ModeSelector(wg.amplitude_generator.m0mask)
    wg.output_type, wg.last_modes = "fd", None
    wg._ylm_cache, wg._prefetched, wg._lock = {}, {}, threading.Lock()
    wg._prefetched_bytes, wg._inflight = 0, {}
    return wg


def test_prepare_native_vs_numpy_and_prefetch():
    wn, wp = _bare_generator("auto"), _bare_generator("python")
    rng = np.random.default_rng(5)
    calls = [(1e6 * (1 + 1e-6 * rng.normal()), 10.0, 9.425031792736052 + 1e-5 * rng.normal(),
              0.35, 1.0, -np.pi / 2, 2.45, 1.0, 2.0, 0.1, 1e-2) for _ in range(6)]
    for c in calls[:2]:
        dn, dp = wn.prepare(*c), wp.prepare(*c)
        np.testing.assert_array_equal(dn["m"], dp["m"])
        np.testing.assert_array_equal(dn["n"], dp["n"])
        assert abs(dn["t"][-1] - dp["t"][-1]) <= 1e-10 * dp["t"][-1]
        assert dn["teuk"].shape[1] == dp["teuk"].shape[1]
    serial = [wn.prepare(*c) for c in calls]
    assert wn.prefetch(calls) == len(calls)
    assert wn.prefetch(calls[:3]) == 0             # held already: not run again
    for c, ref in zip(calls, serial):
        got = wn.prepare(*c)                       # taken from the prefetched results
        for k in ("t", "teuk", "ylms", "m", "f_phi", "Phi_r"):
            np.testing.assert_array_equal(got[k], ref[k])
    assert not wn._prefetched and wn._prefetched_bytes == 0
    # results nobody takes are dropped once they pass the byte bound
    wn.PREFETCH_MAX_BYTES = 3 * waveform_nbytes(serial[0])
    wn.prefetch(calls[:2])
    wn.prefetch(calls[2:4])                        # 4 results would pass 3: the first 2 go
    assert len(wn._prefetched) == 2 and wn._prefetched_bytes <= wn.PREFETCH_MAX_BYTES
    # wait=False: each prepare() takes its own walker's Future (the likelihood's groups), the
    # same arrays; a worker's exception is raised by the prepare() that takes it
    wn._prefetched.clear()
    wn._prefetched_bytes = 0
    assert wn.prefetch(calls, wait=False) == len(calls) and len(wn._inflight) == len(calls)
    # a second prefetch of the same batch (spectrum_batch's after the likelihood's) runs
    # nothing again: the in-flight results serve it
    assert wn.prefetch(calls) == 0 and wn.prefetch(calls, wait=False) == 0
    assert len(wn._inflight) == len(calls) and not wn._prefetched
    for c, ref in zip(calls, serial):
        got = wn.prepare(*c)
        for k in ("t", "teuk", "ylms", "m", "f_phi", "Phi_r"):
            np.testing.assert_array_equal(got[k], ref[k])
    assert not wn._inflight and not wn._prefetched
    # concurrency: two at a time, in order; the same arrays
    assert wn.prefetch(calls, wait=False, concurrency=2) == len(calls)
    for c, ref in zip(calls, serial):
        got = wn.prepare(*c)
        for k in ("t", "teuk", "ylms", "m", "f_phi", "Phi_r"):
            np.testing.assert_array_equal(got[k], ref[k])
    assert not wn._inflight
    bad = calls[0][:2] + (3.0,) + calls[0][3:]     # p0 inside the separatrix buffer
    wn.prefetch([bad], wait=False)
    with pytest.raises(ValueError):
        wn.prepare(*bad)
    assert not wn._inflight
    # a failing call releases its slot: the calls after it still run
    wn.prefetch([bad] + calls[:2], wait=False, concurrency=1)
    with pytest.raises(ValueError):
        wn.prepare(*bad)
    for c, ref in zip(calls[:2], serial[:2]):
        np.testing.assert_array_equal(wn.prepare(*c)["teuk"], ref["teuk"])


def test_host_modes_threads_bitwise():
    """efd_host_set_threads: a one-at-a-time efd_host_modes call split over threads (the API's
    path) keeps bitwise the kept set and complex amplitudes of the one-thread call (the prefetch
    pool's path)."""
    from emri_frequencydomainwaveforms_amd import _lib
    from emri_frequencydomainwaveforms_amd.waveform import FastSchwarzschildEccentricFlux
    lib = _lib.load()
    g = FastSchwarzschildEccentricFlux(sum_kwargs=dict(output_type="fd"))
    tr = g.inspiral_generator
    if tr.lib is None:
        pytest.skip("native upstream not built")
    t, p, e = tr.with_frequencies(1e6, 10.0, 0.0, 10.0, 0.35, 1.0, T=1.0)[:3]
    y = g._ylms(np.pi / 3, -np.pi / 2)
    amp = g.amplitude_generator
    res = []
    try:
        for n in (1, 3, 8):
            lib.efd_host_set_threads(n)
            keep, teuk = amp.select(p, e, y, 1e-4, lib=lib)
            res.append((keep.copy(), teuk.copy()))
    finally:
        lib.efd_host_set_threads(_lib.host_threads())   # the value load() chose
    for keep, teuk in res[1:]:
        np.testing.assert_array_equal(keep, res[0][0])
        np.testing.assert_array_equal(teuk, res[0][1])

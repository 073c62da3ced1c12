"""GPU parity on BASELINE.json's other configurations, against the oracle's C restatement.

- config 1 (M=1e6, mu=10, e0=0.35, Tobs=1 yr, dt=10 s, eps=1e-2, full 3,155,815-bin grid);
- config 3, the four corners of the 10x10 (M, e0) scan (M in {1e5, 1e7}, e0 in {0.1, 0.6},
  mu = 1e-5 M, Tobs = 1 yr, eps = 1e-2): the extreme harmonic counts, knot counts and
  frequency ranges of the grid;
- config 3's whole 10x10 grid against the host twin (same algorithm, itself pinned to the
  oracle), per bin at 1e-10;
- config 5's grid: emri_pe.py:333-349's downsampled uniform f_arr (downsample = 100) at
  Tobs = 4 yr, symmetric but with spacing != 1/T (the mirror-paired kernel on a non-FFT grid).

Tolerance as tests/test_gpu_fullsize.py, per bin (tests/helpers.split_check): 1e-9 max|S_ref| off
the folds, 2 D_k on fold bins (D_k the oracle's own response to 4-ulp input perturbations, two
of them here, the turning-point conditioning floor), with identical support and identical
contribution count C.
"""

import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import bench  # noqa: E402
from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine  # noqa: E402
from oracle import fd_oracle, fd_oracle_c  # noqa: E402
from tests.helpers import record_parity, split_check, ulp_perturbation  # noqa: E402

THREADS = min(16, len(os.sched_getaffinity(0)))


def _oracle(w, freq, perturb=None, extrap=False):
    t, fphi, pphi, fr, pr = w["t"], w["f_phi"], w["phi_phi"], w["f_r"], w["phi_r"]
    if perturb is not None:
        t, fphi, pphi, fr, pr = (perturb(x) for x in (t, fphi, pphi, fr, pr))
    return fd_oracle_c.modesum(t, w["amp"].T, pphi, pr, fphi, fr, w["m"], w["n"],
                               w["ylm_p"], w["ylm_m"], freq, w["prefactor"], caustic="uniform",
                               nthreads=THREADS, extrap=extrap)


def _check(w, freq_host, name):
    inp = DeviceInputs.from_host(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"],
                                 w["f_r"], w["m"], w["n"], w["ylm_p"], w["ylm_m"])
    freq = torch.as_tensor(freq_host, device="cuda")
    eng = ModeSumEngine(caustic="uniform")
    S = eng.run(inp, freq, grid_symmetric=True, scale=w["prefactor"]).cpu().numpy()
    C, _, _ = eng.stats()
    R, E = _oracle(w, freq_host, extrap=True)
    Rps = [_oracle(w, freq_host, ulp_perturbation(seed)) for seed in (11, 12)]
    ok, stats, _ = split_check(S, R, Rps, E=E)
    record_parity(name, dict(stats, contributions=C, harmonics=int(len(w["m"]))))
    assert ok, stats
    np.testing.assert_array_equal(S != 0, R != 0)
    assert C == fd_oracle.contributions(w["t"], w["f_phi"], w["f_r"], w["m"], w["n"], freq_host)
    return stats


def test_config1_full_grid():
    w = bench.build_workload(T=1.0, dt=10.0, eps=1e-2)
    assert len(w["freq"]) == 3155815
    _check(w, w["freq"], "config1")


@pytest.mark.parametrize("M,e0", [(1e5, 0.1), (1e5, 0.6), (1e7, 0.1), (1e7, 0.6)])
def test_config3_grid_corners(M, e0):
    w = bench.build_workload(T=1.0, dt=10.0, eps=1e-2, M=M, mu=1e-5 * M, e0=e0)
    _check(w, w["freq"], f"config3_M{M:.0e}_e{e0}")


def test_config3_full_grid_vs_twin():
    """All 100 points of config 3's scan (check_mode_by_mode.py's parameter-space loop,
    BASELINE configs[2]: M = logspace(5, 7, 10), e0 = linspace(0.1, 0.6, 10), mu = 1e-5 M,
    p0 from get_p_at_t for a 0.99 Tobs plunge, Tobs = 1 yr, dt = 10 s, eps = 1e-2; the native
    upstream builds the inputs). Each point's HIP spectrum is held to the host twin
    efd_modesum_cpu, which runs the same algorithm and is itself pinned to the oracle
    (tests/test_cpu_twin.py; the oracle checks the grid's corners above). The bound is the
    config-2 twin test's per-bin rule: 1e-10 max|S| wherever the twin's response to four 4-ulp
    input perturbations stays below that, 2x that response elsewhere. Supports, contribution
    and evaluation counts must be identical."""
    from emri_frequencydomainwaveforms_amd import cputwin
    from emri_frequencydomainwaveforms_amd.constants import Gpc, MRSUN_SI
    from emri_frequencydomainwaveforms_amd.summation import fd_grid
    from emri_frequencydomainwaveforms_amd.trajectory import get_p_at_t
    from emri_frequencydomainwaveforms_amd.waveform import FastSchwarzschildEccentricFlux
    gen = FastSchwarzschildEccentricFlux(sum_kwargs=dict(output_type="fd"))
    traj = gen.inspiral_generator
    assert traj.backend == "native"
    freq_h = fd_grid(1.0, 10.0)
    freq = torch.as_tensor(freq_h, device="cuda")
    eng = ModeSumEngine(caustic="uniform")
    worst = {"max_err_off_fold_rel": 0.0, "max_err_over_D_at_folds": 0.0, "fold_bins": 0}
    Ks = []
    for M in np.logspace(5, 7, 10):
        for e0 in np.linspace(0.1, 0.6, 10):
            mu = 1e-5 * M
            p0 = get_p_at_t(traj, 0.99, [M, mu, 0.0, e0, 1.0])
            d = gen.prepare(M, mu, p0, e0, np.pi / 3, -np.pi / 2, 1.0, T=1.0, eps=1e-2)
            K = len(d["m"])
            Ks.append(K)
            m, n = d["m"].astype(np.int32), d["n"].astype(np.int32)
            yp, ym = d["ylms"][:K], d["ylms"][K:]
            scale = mu * MRSUN_SI / Gpc
            inp = DeviceInputs.from_host(d["t"], d["teuk"], d["Phi_phi"], d["Phi_r"], d["f_phi"],
                                         d["f_r"], m, n, yp, ym)
            S = eng.run(inp, freq, grid_symmetric=True, scale=scale).cpu().numpy()

            def twin(p=lambda x: x):
                return cputwin.modesum(p(d["t"]), d["teuk"], p(d["Phi_phi"]), p(d["Phi_r"]),
                                       p(d["f_phi"]), p(d["f_r"]), m, n, yp, ym, freq_h, scale)
            T = twin()
            assert eng.stats() == cputwin.stats(), (M, e0)
            # four 4-ulp draws for D (as the config-2 twin test; two recorded beside)
            Tps = [twin(ulp_perturbation(s)) for s in (41, 42, 43, 44)]
            ok, stats, _ = split_check(S, T, Tps, rel=1e-10)
            assert ok, (M, e0, stats)
            _, stats2, _ = split_check(S, T, Tps[:2], rel=1e-10)
            stats["max_err_over_D_at_folds_2draws"] = stats2["max_err_over_D_at_folds"]
            np.testing.assert_array_equal(S != 0, T != 0)
            for k in ("max_err_off_fold_rel", "max_err_over_D_at_folds", "fold_bins",
                      "max_err_over_D_at_folds_2draws"):
                worst[k] = max(worst.get(k, 0.0), stats[k])
    record_parity("config3_grid_vs_twin", dict(worst, points=len(Ks), harmonics_min=min(Ks),
                                               harmonics_max=max(Ks), perturbation_draws=4,
                                               ok=True))


def test_config5_downsampled_grid():
    w = bench.build_workload(T=4.0, dt=10.0, eps=1e-2)
    freq = w["freq"]
    pos = freq >= 0.0
    # non-zero support of the full-grid injection over f >= 0 (emri_pe.py:333-337), from the
    # oracle's contribution map: a bin is non-zero iff some branch's support covers it
    R = _oracle(w, freq)
    fixed = freq[pos]
    nz = np.abs(R[pos]) > 0
    num = int(nz.sum() / 100)
    p_freq = np.linspace(0.0, fixed[nz].max() * 1.01, num=num)
    newfreq = np.hstack((-p_freq[::-1][:-1], p_freq))
    assert np.array_equal(newfreq, -newfreq[::-1])
    _check(w, newfreq, "config5_grid")

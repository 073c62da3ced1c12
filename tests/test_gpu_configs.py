"""GPU parity on BASELINE.json's other configurations, against the oracle's C restatement.

- config 1 (M=1e6, mu=10, e0=0.35, Tobs=1 yr, dt=10 s, eps=1e-2, full 3,155,815-bin grid);
- config 3, the four corners of the 10x10 (M, e0) scan (M in {1e5, 1e7}, e0 in {0.1, 0.6},
  mu = 1e-5 M, Tobs = 1 yr, eps = 1e-2): the extreme harmonic counts, knot counts and
  frequency ranges of the grid;
- config 5's grid: emri_pe.py:333-349's downsampled uniform f_arr (downsample = 100) at
  Tobs = 4 yr, symmetric but with spacing != 1/T (the mirror-paired kernel on a non-FFT grid).

Tolerance as tests/test_gpu_fullsize.py: max|S_gpu - S_ref| <= max(1e-9 max|S_ref|, 2 D), D the
oracle's own response to 1-ulp input perturbations (the turning-point conditioning floor), with
identical support and identical contribution count C.
"""

import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import bench  # noqa: E402
from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine  # noqa: E402
from oracle import fd_oracle, fd_oracle_c  # noqa: E402

THREADS = min(16, len(os.sched_getaffinity(0)))


def _oracle(w, freq, perturb=None):
    t, fphi, pphi = w["t"], w["f_phi"], w["phi_phi"]
    if perturb is not None:
        t, fphi, pphi = perturb(t), perturb(fphi), perturb(pphi)
    return fd_oracle_c.modesum(t, w["amp"].T, pphi, w["phi_r"], fphi, w["f_r"], w["m"], w["n"],
                               w["ylm_p"], w["ylm_m"], freq, w["prefactor"], caustic="uniform",
                               nthreads=THREADS)


def _check(w, freq_host):
    inp = DeviceInputs.from_host(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"],
                                 w["f_r"], w["m"], w["n"], w["ylm_p"], w["ylm_m"])
    freq = torch.as_tensor(freq_host, device="cuda")
    eng = ModeSumEngine(caustic="uniform")
    S = eng.run(inp, freq, grid_symmetric=True, scale=w["prefactor"]).cpu().numpy()
    C, _, _ = eng.stats()
    R = _oracle(w, freq_host)
    rng = np.random.default_rng(11)
    Rp = _oracle(w, freq_host,
                 lambda x: x * (1.0 + rng.choice([-1.0, 1.0], len(x)) * 2.0 ** -52))
    mx = np.abs(R).max()
    assert mx > 0
    floor = np.abs(Rp - R).max()
    err = np.abs(S - R).max()
    assert err <= max(1e-9 * mx, 2.0 * floor), (err / mx, floor / mx)
    np.testing.assert_array_equal(S != 0, R != 0)
    assert C == fd_oracle.contributions(w["t"], w["f_phi"], w["f_r"], w["m"], w["n"], freq_host)
    return err / mx


def test_config1_full_grid():
    w = bench.build_workload(T=1.0, dt=10.0, eps=1e-2)
    assert len(w["freq"]) == 3155815
    _check(w, w["freq"])


@pytest.mark.parametrize("M,e0", [(1e5, 0.1), (1e5, 0.6), (1e7, 0.1), (1e7, 0.6)])
def test_config3_grid_corners(M, e0):
    w = bench.build_workload(T=1.0, dt=10.0, eps=1e-2, M=M, mu=1e-5 * M, e0=e0)
    _check(w, w["freq"])


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
    _check(w, newfreq)

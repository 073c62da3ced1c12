"""GPU parity of the HIP time-domain mode sum (efd_td_modesum, k_td_modesum) against the TD
oracle, and the reference's FD-vs-TD comparison run on the device (td_gen ->
get_fd_waveform_fromTD vs few_gen; Tutorial_FrequencyDomain_Waveforms.ipynb:184-262,
check_mode_by_mode.py:85-99, 254-309).

Tolerance: max_i |h_gpu - h_ref| <= 1e-9 max_i |h_ref| (both FP64; the kernel forms
e^{-i (m Phi_phi + n Phi_r)} by Horner's rule in e^{-i Phi_r} from one sin/cos per m, the
oracle per harmonic: rounding of phases up to ~1e5 rad). Samples past the inspiral's end are
exactly zero on both sides.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from emri_frequencydomainwaveforms_amd.summation import (  # noqa: E402
    DeviceInputs, ModeSumEngine, TDEngine)
from oracle import td_oracle  # noqa: E402
from tests.helpers import source_inputs  # noqa: E402

RTOL = 1e-9


def _inp(d):
    return DeviceInputs.from_host(d["t"], np.asarray(d["amp"]).T, d["phi_phi"], d["phi_r"],
                                  d["f_phi"], d["f_r"], d["m"], d["n"], d["ylm_p"], d["ylm_m"])


def _ref(d, ns, scale=None):
    sc = d["prefactor"] if scale is None else scale
    return td_oracle.td_modesum(d["t"], d["amp"], d["phi_phi"], d["phi_r"], d["m"], d["n"],
                                d["ylm_p"], d["ylm_m"], d["dt"], ns, sc)


def _relerr(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.fixture(scope="module")
def multimode():
    # includes (l, 0, 0) harmonics, negative n, gaps in n per m
    return source_inputs(M=3e5, mu=10.0, e0=0.35, T=0.02, dt=20.0, eps=1e-2)


def test_td_vs_oracle(multimode):
    d = multimode
    ns = len(d["freq"])
    h = TDEngine().run(_inp(d), d["dt"], ns, scale=d["prefactor"]).cpu().numpy()
    R = _ref(d, ns)
    assert len(d["m"]) > 20 and np.any((d["m"] == 0) & (d["n"] == 0))
    assert _relerr(h, R) < RTOL
    nv = td_oracle.valid_samples(d["t"][-1], d["dt"], ns)
    assert np.all(h[nv:] == 0) and np.all(h[:nv] != 0)


def test_td_single_and_sparse_harmonics():
    # one harmonic; then harmonics with large gaps in n for one m and a lone m = 0 mode
    for modes in ([(2, 2, 0)], [(2, 2, -5), (3, 2, 4), (2, 1, 3), (2, 0, 2)]):
        d = source_inputs(M=3e5, mu=10.0, e0=0.35, T=0.02, dt=20.0, modes=modes)
        ns = len(d["freq"])
        h = TDEngine().run(_inp(d), d["dt"], ns, scale=d["prefactor"]).cpu().numpy()
        assert _relerr(h, _ref(d, ns)) < RTOL, modes


def test_td_outputs_scale_accumulate(multimode):
    d = multimode
    ns = len(d["freq"]) + 777   # not a multiple of the block
    inp = _inp(d)
    eng = TDEngine()
    sc = 0.7 - 0.4j
    h = torch.empty(ns, dtype=torch.complex128, device="cuda")
    hp = torch.empty(ns, dtype=torch.float64, device="cuda")
    hc = torch.empty(ns, dtype=torch.float64, device="cuda")
    eng.launch(inp, d["dt"], ns, out=torch.view_as_real(h), hp=hp, hc=hc, scale=sc)
    assert eng.status()
    R = _ref(d, ns, scale=sc)
    assert _relerr(h.cpu().numpy(), R) < RTOL
    # h = h+ - i hx exactly
    assert torch.equal(hp, h.real) and torch.equal(hc, -h.imag)
    # accumulate adds a second copy
    eng.launch(inp, d["dt"], ns, out=torch.view_as_real(h), hp=hp, hc=hc, scale=sc,
               accumulate=True)
    assert eng.status()
    assert _relerr(h.cpu().numpy(), 2 * R) < RTOL
    assert torch.equal(hp, h.real) and torch.equal(hc, -h.imag)


def test_td_deterministic(multimode):
    d = multimode
    ns = len(d["freq"])
    eng = TDEngine()
    inp = _inp(d)
    a = eng.run(inp, d["dt"], ns, scale=d["prefactor"])
    b = eng.run(inp, d["dt"], ns, scale=d["prefactor"])
    assert torch.equal(a, b)


def test_dft_of_gpu_td_matches_gpu_fd():
    # the reference's FD-vs-TD comparison, both sides on the device (rocFFT for the DFT)
    from scipy.signal.windows import hann
    d = source_inputs(M=1e6, mu=10.0, e0=0.35, T=0.05, dt=10.0, eps=1e-2)
    keep = ~((d["m"] == 0) & (d["n"] == 0))   # F = 0 harmonics exist in TD only
    for k in ("amp", "m", "n", "ylm_p", "ylm_m"):
        d[k] = d[k][keep]
    ns = len(d["freq"])
    inp = _inp(d)
    h = TDEngine().run(inp, d["dt"], ns, scale=d["prefactor"])
    freq = torch.as_tensor(d["freq"], device="cuda")
    S = ModeSumEngine().run(inp, freq, grid_symmetric=True, scale=d["prefactor"])
    w = torch.as_tensor(hann(ns), device="cuda")
    a = torch.fft.fftshift(torch.fft.fft(h * w)) * d["dt"]
    b = torch.fft.fftshift(torch.fft.fft(torch.fft.ifft(torch.fft.ifftshift(S)) * w))
    ov = (torch.vdot(a, b) / torch.sqrt(torch.vdot(a, a).real * torch.vdot(b, b).real)).real
    assert 1.0 - ov.item() < 5e-3


def test_td_generator_api():
    from emri_frequencydomainwaveforms_amd.fdutils import get_fd_waveform_fromTD
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    from emri_frequencydomainwaveforms_amd.waveform import GenerateEMRIWaveform
    M, MU, E0, T, DT = 3e5, 10.0, 0.3, 0.02, 20.0
    p0 = get_p_at_t(EMRIInspiral(), 0.99 * T, [M, MU, 0.0, E0, 1.0])
    params = [M, MU, 0.0, p0, E0, 1.0, 1.0, 0.5, 0.3, 0.8, 1.1, 0.2, 0.0, 0.4]
    kw = dict(T=T, dt=DT, eps=1e-2)
    td_gen = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux",
                                  sum_kwargs=dict(pad_output=True, odd_len=True),
                                  use_gpu=True, return_list=True)
    fd_gen = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux",
                                  sum_kwargs=dict(pad_output=True, output_type="fd",
                                                  odd_len=True), use_gpu=True)
    hp, hc = td_gen(*params, **kw)
    S = fd_gen(*params, **kw)
    freq = fd_gen.waveform_generator.create_waveform.frequency
    assert hp.dtype == torch.float64 and hp.shape == freq.shape   # lines up with the FD grid
    h = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux",
                             sum_kwargs=dict(pad_output=True, odd_len=True), use_gpu=True)(
        *params, **kw)
    assert torch.equal(h.real, hp) and torch.equal(-h.imag, hc)
    mask = freq >= 0
    conv = get_fd_waveform_fromTD(td_gen, mask, DT)
    ch1, ch2 = conv(*params, **kw)
    ref = torch.fft.fftshift(torch.fft.fft(hp.to(torch.complex128))) * DT
    assert torch.equal(ch1, ref[mask]) and ch2.shape == ch1.shape
    assert S.shape == freq.shape

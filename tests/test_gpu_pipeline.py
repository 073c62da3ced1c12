"""WaveformPipeline: several waveforms in flight on separate streams give bitwise the results of
the one-at-a-time path, and device-side errors of any slot surface at wait().

Parity: the oracle (notebook restatement) pins the one-at-a-time path elsewhere
(test_gpu_modesum.py); here every pipelined spectrum is compared bitwise with it, plus one
oracle check of a pipelined spectrum at the 1e-9 relative tolerance of the small cases.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from emri_frequencydomainwaveforms_amd import _lib  # noqa: E402
from emri_frequencydomainwaveforms_amd.summation import (DeviceInputs, ModeSumEngine,  # noqa: E402
                                                         WaveformPipeline)
from oracle.fd_oracle import fd_modesum  # noqa: E402
from tests.helpers import source_inputs  # noqa: E402

KEYS = ("t", "phi_phi", "phi_r", "f_phi", "f_r", "m", "n", "ylm_p", "ylm_m")


def _host(d):
    h = {k: d[k] for k in KEYS}
    h["amp"] = np.ascontiguousarray(d["amp"].T)     # [nt][K]
    return h


@pytest.fixture(scope="module")
def sources():
    out = []
    for M, e0 in ((3e5, 0.35), (5e5, 0.2), (2e5, 0.5), (4e5, 0.1), (3e5, 0.6)):
        out.append(source_inputs(M=M, e0=e0, T=0.02, dt=20.0, eps=1e-2))
    return out


def _serial(d, freq):
    h = _host(d)
    inp = DeviceInputs.from_host(h["t"], h["amp"], h["phi_phi"], h["phi_r"], h["f_phi"],
                                 h["f_r"], h["m"], h["n"], h["ylm_p"], h["ylm_m"])
    return ModeSumEngine().run(inp, freq, grid_symmetric=True, scale=d["prefactor"])


@pytest.mark.parametrize("slots", [1, 3])
def test_pipeline_bitwise_equals_serial(sources, slots):
    freq = torch.as_tensor(sources[0]["freq"], device="cuda")
    nf = int(freq.numel())
    k0 = int(np.searchsorted(sources[0]["freq"], 0.0))
    pipe = WaveformPipeline(slots)
    S = [torch.empty(nf, dtype=torch.complex128, device="cuda") for _ in sources]
    hp = [torch.empty(nf - k0, dtype=torch.complex128, device="cuda") for _ in sources]
    hc = [torch.empty_like(x) for x in hp]
    for i, d in enumerate(sources):     # spectra, then fused polarisations, interleaved
        pipe.submit(_host(d), freq, True, d["prefactor"], out=torch.view_as_real(S[i]))
        pipe.submit(_host(d), freq, True, d["prefactor"], hp=torch.view_as_real(hp[i]),
                    hc=torch.view_as_real(hc[i]), k0=k0)
    pipe.wait()
    for i, d in enumerate(sources):
        ref = _serial(d, freq)
        assert torch.equal(S[i], ref)
        b = torch.flip(ref, [0])[k0:]
        a = ref[k0:]
        assert torch.equal(hp[i], 0.5 * (a + b.conj()))
        assert torch.equal(hc[i], 0.5j * (a - b.conj()))


def test_pipeline_matches_oracle(sources):
    d = sources[2]
    freq_h = d["freq"]
    freq = torch.as_tensor(freq_h, device="cuda")
    pipe = WaveformPipeline(2)
    S = torch.empty(len(freq_h), dtype=torch.complex128, device="cuda")
    pipe.submit(_host(d), freq, True, d["prefactor"], out=torch.view_as_real(S))
    pipe.wait()
    ref = fd_modesum(d["t"], d["amp"], d["phi_phi"], d["phi_r"], d["f_phi"], d["f_r"], d["m"],
                     d["n"], d["ylm_p"], d["ylm_m"], freq_h, d["prefactor"])
    assert np.abs(S.cpu().numpy() - ref).max() <= 1e-9 * np.abs(ref).max()


def test_pipeline_surfaces_slot_errors(sources):
    d = dict(sources[0])
    d["m"] = d["m"].copy()
    d["m"][0] = 300                       # |m| > 255: flagged by k_group on the device
    freq = torch.as_tensor(d["freq"], device="cuda")
    pipe = WaveformPipeline(2)
    S = torch.empty(len(d["freq"]), dtype=torch.complex128, device="cuda")
    pipe.submit(_host(sources[1]), freq, True, 1.0, out=torch.view_as_real(S))
    pipe.submit(_host(d), freq, True, 1.0, out=torch.view_as_real(S))
    with pytest.raises(_lib.EFDError):
        pipe.wait()


def test_slot_errors_survive_slot_reuse(sources):
    """a device-side error of an early waveform on a slot is not erased when later
    waveforms reuse that slot before wait() (sticky header flags); wait() reports it once and
    the slot is clean afterwards. Covers both error kinds a preparation raises: |m| > 255 and a
    harmonic with more than 8 monotonic frequency runs (an f_r oscillating along the
    trajectory makes F = m f_phi + n f_r turn at every knot)."""
    freq = torch.as_tensor(sources[0]["freq"], device="cuda")
    S = torch.empty(int(freq.numel()), dtype=torch.complex128, device="cuda")
    bad_m = _host(sources[0])
    bad_m["m"] = bad_m["m"].copy()
    bad_m["m"][0] = 300
    bad_runs = _host(sources[0])
    nt = len(bad_runs["t"])
    assert nt > 20
    bad_runs["f_r"] = bad_runs["f_r"] * (1.0 + 0.3 * (-1.0) ** np.arange(nt))
    for bad in (bad_m, bad_runs):
        pipe = WaveformPipeline(2)
        pipe.submit(bad, freq, True, 1.0, out=torch.view_as_real(S))      # slot 0
        for d in sources[1:4]:                                             # slots 1, 0, 1
            pipe.submit(_host(d), freq, True, 1.0, out=torch.view_as_real(S))
        with pytest.raises(_lib.EFDError):
            pipe.wait()
        pipe.submit(_host(sources[1]), freq, True, 1.0, out=torch.view_as_real(S))
        pipe.submit(_host(sources[2]), freq, True, 1.0, out=torch.view_as_real(S))
        pipe.wait()                                                        # reported once

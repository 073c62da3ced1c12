"""efd_modesum_prepare_batch: a walker batch prepared in one chain of launches.

Each waveform of a batch (different N_t, K and (m, n) sets, on one shared grid) must give
bitwise the spectrum, polarisations, contribution / evaluation counts and fused log-likelihood of
its own efd_modesum_prepare (the one-waveform path, itself pinned to the oracle in
test_gpu_modesum.py / test_gpu_configs.py). efd_modesum_status_batch must name the failing
waveform of a batch and clear its flag. The batched Likelihood path (BatchPreparer) is held to
the per-walker unfused path in test_gpu_api.py and test_gpu_pe_configs.py.
"""

import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from emri_frequencydomainwaveforms_amd import _lib  # noqa: E402
from emri_frequencydomainwaveforms_amd.summation import (BatchPreparer, DeviceInputs,  # noqa: E402
                                                         ModeSumEngine, sum_batch,
                                                         sum_batch_loglike)
from tests.helpers import source_inputs  # noqa: E402

KEYS = ("t", "phi_phi", "phi_r", "f_phi", "f_r", "m", "n", "ylm_p", "ylm_m")


def _host(d):
    h = {k: d[k] for k in KEYS}
    h["amp"] = np.ascontiguousarray(d["amp"].T)     # [nt][K]
    return h


@pytest.fixture(scope="module")
def sources():
    out = []
    for M, e0, eps in ((3e5, 0.35, 1e-2), (5e5, 0.2, 1e-3), (2e5, 0.5, 1e-2), (4e5, 0.1, 1e-5),
                       (3e5, 0.6, 1e-2), (6e5, 0.3, 1e-4)):
        out.append(source_inputs(M=M, e0=e0, T=0.02, dt=20.0, eps=eps))
    return out


def _single(d, freq, caustic):
    h = _host(d)
    inp = DeviceInputs.from_host(h["t"], h["amp"], h["phi_phi"], h["phi_r"], h["f_phi"],
                                 h["f_r"], h["m"], h["n"], h["ylm_p"], h["ylm_m"])
    eng = ModeSumEngine(caustic=caustic)
    S = eng.run(inp, freq, grid_symmetric=True, scale=d["prefactor"])
    return S, eng.stats()


@pytest.mark.parametrize("caustic", ["uniform", "spa"])
def test_prepare_batch_bitwise_equals_single(sources, caustic):
    assert len({(len(d["t"]), len(d["m"])) for d in sources}) == len(sources)  # ragged batch
    freq = torch.as_tensor(sources[0]["freq"], device="cuda")
    nf = int(freq.numel())
    B = BatchPreparer(group=len(sources), depth=2, caustic=caustic)
    for rep in range(2):   # the second flush reuses the other group's workspaces, then this one
        for d in sources:
            B.submit(_host(d), freq, True, d["prefactor"], prepare_only=True)
        gi, jobs = B.flush()
        outs = [torch.empty(nf, dtype=torch.complex128, device="cuda") for _ in sources]
        with torch.cuda.stream(B.stream(gi)):
            sum_batch([(eng, dict(kw, out=torch.view_as_real(o)))
                       for (eng, kw), o in zip(jobs, outs)], stream=B.stream(gi).cuda_stream)
        B.wait()
        for (eng, _), o, d in zip(jobs, outs, sources):
            S, st = _single(d, freq, caustic)
            assert torch.equal(o, S)
            assert eng.stats(B.stream(gi).cuda_stream) == st
            assert st[0] > 0


def test_prepare_batch_polarisations_bitwise(sources):
    """BatchPreparer jobs summed with fused h+/hx (tools/configs.py's config-3 path) give bitwise
    the polarisations of each waveform's own prepare + sum."""
    freq_h = sources[0]["freq"]
    freq = torch.as_tensor(freq_h, device="cuda")
    nf = int(freq.numel())
    k0 = int(np.searchsorted(freq_h, 0.0))
    B = BatchPreparer(group=len(sources))
    B.order_after_current()
    for d in sources:
        B.submit(_host(d), freq, True, d["prefactor"], k0=k0, prepare_only=True)
    gi, jobs = B.flush()
    outs = [(torch.empty(nf - k0, dtype=torch.complex128, device="cuda"),
             torch.empty(nf - k0, dtype=torch.complex128, device="cuda")) for _ in sources]
    sum_batch([(eng, dict(kw, hp=torch.view_as_real(o[0]), hc=torch.view_as_real(o[1])))
               for (eng, kw), o in zip(jobs, outs)], stream=B.stream(gi).cuda_stream)
    B.wait()
    for d, (hp, hc) in zip(sources, outs):
        h = _host(d)
        inp = DeviceInputs.from_host(h["t"], h["amp"], h["phi_phi"], h["phi_r"], h["f_phi"],
                                     h["f_r"], h["m"], h["n"], h["ylm_p"], h["ylm_m"])
        eng = ModeSumEngine()
        rp = torch.empty(nf - k0, dtype=torch.complex128, device="cuda")
        rc = torch.empty_like(rp)
        eng.launch(inp, freq, None, True, d["prefactor"], hp=torch.view_as_real(rp),
                   hc=torch.view_as_real(rc), k0=k0)
        assert eng.status()
        assert torch.equal(hp, rp) and torch.equal(hc, rc)


def test_prepare_batch_loglike_bitwise(sources):
    freq_h = sources[0]["freq"]
    freq = torch.as_tensor(freq_h, device="cuda")
    nf = int(freq.numel())
    k0 = int(np.searchsorted(freq_h, 0.0))
    nb = nf - k0
    rng = np.random.default_rng(3)
    d = torch.as_tensor(rng.standard_normal((2, nb)) + 1j * rng.standard_normal((2, nb)),
                        device="cuda") * 1e-22
    w = torch.as_tensor(rng.uniform(0.5, 2.0, (2, nb)) * 1e40, device="cuda")
    # reference: each walker prepared alone (efd_modesum_prepare), then one fused batch
    engs = [ModeSumEngine() for _ in sources]
    jobs1 = []
    for eng, src in zip(engs, sources):
        h = _host(src)
        inp = DeviceInputs.from_host(h["t"], h["amp"], h["phi_phi"], h["phi_r"], h["f_phi"],
                                     h["f_r"], h["m"], h["n"], h["ylm_p"], h["ylm_m"])
        eng.launch(inp, freq, None, True, src["prefactor"], phase="prepare", k0=k0,
                   hp=None, hc=None)
        jobs1.append((eng, dict(inp=inp, freq=freq, out=None, grid_symmetric=True,
                                scale=src["prefactor"], k0=k0)))
    ref = torch.empty(len(sources), dtype=torch.float64, device="cuda")
    sum_batch_loglike(jobs1, d, w, ref)
    B = BatchPreparer(group=len(sources))
    for src in sources:
        B.submit(_host(src), freq, True, src["prefactor"], k0=k0, prepare_only=True)
    gi, jobs = B.flush()
    got = torch.empty(len(sources), dtype=torch.float64, device="cuda")
    torch.cuda.current_stream().wait_stream(B.stream(gi))
    sum_batch_loglike(jobs, d, w, got)
    torch.cuda.synchronize()
    B.wait()
    assert torch.equal(got, ref)
    assert torch.all(torch.isfinite(got)) and torch.all(got < 0)


def test_prepare_batch_argument_checks(sources):
    freq = torch.as_tensor(sources[0]["freq"], device="cuda")
    B = BatchPreparer(group=2)
    with pytest.raises(ValueError):
        B.submit(_host(sources[0]), freq, True, 1.0)          # not prepare_only
    B.submit(_host(sources[0]), freq, True, 1.0, prepare_only=True)
    B.submit(_host(sources[1]), freq, True, 1.0, prepare_only=True)
    with pytest.raises(ValueError):
        B.submit(_host(sources[2]), freq, True, 1.0, prepare_only=True)   # group full
    B.flush()
    B.wait()
    lib = _lib.load()
    # the C ABI: a shared workspace and a grid mismatch are refused before any launch
    eng = B.groups[0]["engines"][0]
    a = B.last_jobs[0][1]["_args"]
    pa = (ctypes.POINTER(_lib.ModesumArgs) * 2)(ctypes.pointer(a), ctypes.pointer(a))
    pw = (ctypes.c_void_p * 2)(eng._ws.data_ptr(), eng._ws.data_ptr())
    pb = (ctypes.c_size_t * 2)(eng._ws.numel(), eng._ws.numel())
    st = torch.cuda.current_stream().cuda_stream
    assert lib.efd_modesum_prepare_batch(pa, pw, pb, 2, st) == _lib.EFD_ERR_ARG
    a2 = _lib.ModesumArgs.from_buffer_copy(a)
    a2.grid_symmetric = 0
    eng2 = B.groups[0]["engines"][1]
    pa = (ctypes.POINTER(_lib.ModesumArgs) * 2)(ctypes.pointer(a), ctypes.pointer(a2))
    pw = (ctypes.c_void_p * 2)(eng._ws.data_ptr(), eng2._ws.data_ptr())
    pb = (ctypes.c_size_t * 2)(eng._ws.numel(), eng2._ws.numel())
    assert lib.efd_modesum_prepare_batch(pa, pw, pb, 2, st) == _lib.EFD_ERR_ARG
    assert lib.efd_modesum_prepare_batch(pa, pw, pb, 0, st) == _lib.EFD_ERR_ARG
    assert lib.efd_modesum_prepare_batch(pa, pw, pb, _lib.EFD_BATCH_MAX + 1, st) == _lib.EFD_ERR_ARG


def test_status_batch_names_failing_waveform(sources):
    freq = torch.as_tensor(sources[0]["freq"], device="cuda")
    B = BatchPreparer(group=3, depth=1)
    for i in range(3):
        h = _host(sources[i])
        if i == 2:
            h["m"] = h["m"].copy()
            h["m"][0] = 300                                  # |m| > 255: bad_mn on waveform 2
        B.submit(h, freq, True, 1.0, prepare_only=True)
    B.flush()
    with pytest.raises(_lib.EFDError, match="waveform 2 of the batch"):
        B.wait()
    B.wait()   # reported once: the flag is cleared
    lib = _lib.load()
    wss = [eng._ws.data_ptr() for eng in B.groups[0]["engines"]]
    flags = (ctypes.c_int32 * 3)()
    rc = lib.efd_modesum_status_batch((ctypes.c_void_p * 3)(*wss), 3, flags,
                                      B.stream(0).cuda_stream)
    assert rc == _lib.EFD_OK and list(flags) == [0, 0, 0]


def test_fused_loglike_marks_failing_walker_nan(sources):
    """efd_modesum_sum_loglike writes NaN for a walker whose workspace holds a device-side error
    flag (here |m| > 255 on walker 2) and leaves the flag set, so the batched likelihood needs a
    status read only when a NaN comes back (likelihood.py: one synchronisation per batch)."""
    freq = torch.as_tensor(sources[0]["freq"], device="cuda")
    nf = int(freq.numel())
    B = BatchPreparer(group=3, depth=1)
    for i in range(3):
        h = _host(sources[i])
        if i == 2:
            h["m"] = h["m"].copy()
            h["m"][0] = 300
        B.submit(h, freq, True, sources[i]["prefactor"], prepare_only=True)
    gi, jobs = B.flush()
    cur = torch.cuda.current_stream()
    cur.wait_stream(B.stream(gi))
    d = torch.zeros((2, nf), dtype=torch.complex128, device="cuda")
    w = torch.ones((2, nf), dtype=torch.float64, device="cuda")
    out = torch.full((3,), 1.0, dtype=torch.float64, device="cuda")
    B.sum_loglike(gi, d, w, out, cur.cuda_stream)
    ll = out.cpu().numpy()
    assert np.isnan(ll[2]) and np.all(np.isfinite(ll[:2])) and np.all(ll[:2] < 0.0)
    with pytest.raises(_lib.EFDError, match="waveform 2 of the batch"):
        B.wait()


@pytest.mark.parametrize("dt", [20.0, 2.0])
def test_fused_loglike_tile_constants_bitwise(sources, dt):
    """efd_modesum_sum_loglike_ex with efd_loglike_tile_constants gives bitwise the logL of
    efd_modesum_sum_loglike: the tiles no harmonic reaches take the precomputed partial, made
    with the epilogue's own arithmetic on zero sums. dt = 2 s puts Nyquist ten times above the
    sources' highest harmonic, so most tiles take it."""
    from emri_frequencydomainwaveforms_amd.summation import fd_grid, loglike_tile_constants
    freq_h = fd_grid(0.02, dt)
    freq = torch.as_tensor(freq_h, device="cuda")
    nf = int(freq.numel())
    k0 = int(np.searchsorted(freq_h, 0.0))
    nb = nf - k0
    rng = np.random.default_rng(11)
    d = torch.as_tensor(rng.standard_normal((2, nb)) + 1j * rng.standard_normal((2, nb)),
                        device="cuda") * 1e-22
    w = torch.as_tensor(rng.uniform(0.5, 2.0, (2, nb)) * 1e40, device="cuda")
    w[:, 0] = 0.0   # a zeroed bin, as Likelihood's start_ind
    tc = loglike_tile_constants(d, w, nf, k0)
    lib = _lib.load()
    assert tc.numel() == lib.efd_loglike_tile_count(nf)
    B = BatchPreparer(group=len(sources), depth=1)
    for src in sources:
        B.submit(_host(src), freq, True, src["prefactor"], k0=k0, prepare_only=True)
    gi, jobs = B.flush()
    cur = torch.cuda.current_stream()
    cur.wait_stream(B.stream(gi))
    ref = torch.empty(len(sources), dtype=torch.float64, device="cuda")
    got = torch.empty_like(ref)
    got2 = torch.empty_like(ref)
    B.sum_loglike(gi, d, w, ref, cur.cuda_stream)
    B.sum_loglike(gi, d, w, got, cur.cuda_stream, tile_const=tc)
    sum_batch_loglike(jobs, d, w, got2, tile_const=tc)
    torch.cuda.synchronize()
    B.wait()
    assert torch.all(torch.isfinite(ref)) and torch.all(ref < 0)
    # bitwise, split tiles included (k_segments_one's plan evaluates a heavy tile's bins on
    # several workgroups, each bin's sum in the whole tile's order)
    assert torch.equal(got, ref) and torch.equal(got2, ref)
    # the constants alone sum to a zero template's sum |d - 0 w|^2 over every bin (to rounding:
    # another summation order)
    h0 = float((torch.abs(d) ** 2).sum())
    assert abs(float(tc.sum()) - h0) <= 1e-12 * h0
    with pytest.raises(ValueError):
        sum_batch_loglike(jobs, d, w, got2, tile_const=tc[:-1])


def test_fused_loglike_tile_constants_no_segment(sources):
    """A grid whose bins all lie above every harmonic: no walker has a segment (empty lane union),
    so the sparse sum launches no tile work and k_ll_final adds only the constants; bitwise the
    dense launch's logL, which is then the zero template's -2 sum |d|^2."""
    from emri_frequencydomainwaveforms_amd.summation import loglike_tile_constants
    fmax = max(float(np.abs(s["m"] * s["f_phi"][:, None] + s["n"] * s["f_r"][:, None]).max())
               for s in sources[:3])
    p = np.linspace(2.0 * fmax, 3.0 * fmax, 2001)
    freq_h = np.concatenate([-p[::-1], [0.0], p])
    freq = torch.as_tensor(freq_h, device="cuda")
    nf = int(freq.numel())
    k0 = nf // 2
    nb = nf - k0
    rng = np.random.default_rng(5)
    d = torch.as_tensor(rng.standard_normal((2, nb)) + 1j * rng.standard_normal((2, nb)),
                        device="cuda")
    w = torch.ones((2, nb), dtype=torch.float64, device="cuda")
    tc = loglike_tile_constants(d, w, nf, k0)
    B = BatchPreparer(group=3, depth=1)
    for s in sources[:3]:
        B.submit(_host(s), freq, True, s["prefactor"], k0=k0, prepare_only=True)
    gi, jobs = B.flush()
    cur = torch.cuda.current_stream()
    cur.wait_stream(B.stream(gi))
    ref = torch.empty(3, dtype=torch.float64, device="cuda")
    got = torch.empty_like(ref)
    B.sum_loglike(gi, d, w, ref, cur.cuda_stream)
    B.sum_loglike(gi, d, w, got, cur.cuda_stream, tile_const=tc)
    torch.cuda.synchronize()
    B.wait()
    assert torch.equal(got, ref)
    h0 = -2.0 * float((torch.abs(d) ** 2).sum())
    assert np.allclose(ref.cpu().numpy(), h0, rtol=1e-12, atol=0.0)


@pytest.mark.parametrize("split_min", ["", "-1"])
def test_fused_loglike_split_tiles(split_min, monkeypatch):
    """The sparse fused likelihood's split plan (k_segments_one: a tile above the waveform's fair
    share of the chip is evaluated by BPL workgroups, one bin of every lane each; the last
    arriver runs the tile's epilogue from the bins they stored) on config 5's shape: a coarse
    downsampled grid where a few low-frequency tiles hold most records. The plan must be made
    (split tiles > 0), the logL must equal the unsplit dense launch's bitwise, and repeated sums
    on the same preparation (the arrival counters re-armed by the last arrivers) must give
    bitwise the same values. split_min = -1 (EFD_SPLIT_MIN_COST) splits every tile of the union,
    empty ones included."""
    from emri_frequencydomainwaveforms_amd.summation import loglike_tile_constants
    if split_min:
        monkeypatch.setenv("EFD_SPLIT_MIN_COST", split_min)
    # eps = 3e-2: 24-30 modes, inside k_segments_one's K <= SEG1_MAX_K (the plan's condition)
    srcs = [source_inputs(M=M, e0=e0, T=0.5, dt=10.0, eps=3e-2)
            for M, e0 in ((1e6, 0.35), (8e5, 0.3), (1.2e6, 0.4), (9e5, 0.25))]
    fmax = max(float(np.abs(s["m"] * s["f_phi"][:, None] + s["n"] * s["f_r"][:, None]).max())
               for s in srcs)
    p = np.linspace(0.0, 1.01 * fmax, 4001)          # emri_pe.py's downsampled grid shape
    freq_h = np.concatenate([-p[::-1][:-1], p])
    freq = torch.as_tensor(freq_h, device="cuda")
    nf = int(freq.numel())
    k0 = nf // 2
    nb = nf - k0
    rng = np.random.default_rng(3)
    d = torch.as_tensor(rng.standard_normal((2, nb)) + 1j * rng.standard_normal((2, nb)),
                        device="cuda") * 1e-21
    w = torch.as_tensor(rng.uniform(0.5, 2.0, (2, nb)) * 1e20, device="cuda")
    tc = loglike_tile_constants(d, w, nf, k0)
    B = BatchPreparer(group=len(srcs), depth=1)
    for src in srcs:
        B.submit(_host(src), freq, True, src["prefactor"], k0=k0, prepare_only=True)
    gi, jobs = B.flush()
    cur = torch.cuda.current_stream()
    cur.wait_stream(B.stream(gi))
    ref = torch.empty(len(srcs), dtype=torch.float64, device="cuda")
    got = [torch.empty_like(ref) for _ in range(3)]
    B.sum_loglike(gi, d, w, ref, cur.cuda_stream)                       # dense: no plan used
    for g in got:
        B.sum_loglike(gi, d, w, g, cur.cuda_stream, tile_const=tc)     # sparse, split tiles
    torch.cuda.synchronize()
    B.wait()
    plans = [eng.split_plan() for eng, _ in jobs]
    assert any(ns > 0 for _, ns in plans), plans
    assert torch.all(torch.isfinite(ref))
    assert torch.equal(got[0], ref), (got[0] - ref) / ref
    assert torch.equal(got[1], got[0]) and torch.equal(got[2], got[0])

"""FEW-compatible waveform classes: the FD path and its TD comparison path.

Call surfaces kept from the reference (so its drivers only change the import line):
  GenerateEMRIWaveform("FastSchwarzschildEccentricFlux",
                       sum_kwargs=dict(pad_output=True, output_type="fd", odd_len=True),
                       use_gpu=..., return_list=...)          check_mode_by_mode.py:69-83
  few_gen(M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0, Phi_theta0, Phi_r0,
          T=, dt=, eps=, [f_arr=, mask_positive=, mode_selection=, include_minus_m=])
                                                              emri_pe.py:140-155, 212, 242
  few_gen.waveform_generator.create_waveform.frequency        check_mode_by_mode.py:250

Upstream of the hot path (trajectory, amplitudes, Ylm, mode selection) runs on the host with
the stand-ins of trajectory.py / amplitude.py (NOT FEW physics).
The FD summation itself runs in libemrifd.so on the GPU.
`use_gpu` selects the return type (torch tensors on the GPU, or numpy copies); the compute
always runs on the GPU -- there is no CPU fallback.

Frame handling [FEW-ext, FEW 1.x GenerateEMRIWaveform as recalled]: the source-frame viewing
angles are theta = arccos(-R.S), phi = -pi/2 from the sky (qS, phiS) and spin (qK, phiK)
directions; frame="detector" (default) rotates (h+, hx) by the polarisation angle psi, which on
the complex spectrum S = h+ - i hx is the constant factor exp(-2 i psi) -- folded into the
kernel's complex scale, so it costs nothing.
"""

import os
import threading

import numpy as np

from . import _lib
from .amplitude import ModeSelector, RomanAmplitude
from .constants import Gpc, MRSUN_SI, MTSUN_SI
from .frequencies import get_fundamental_frequencies
from .summation import FDInterpolatedModeSum, TDInterpolatedModeSum, require_gpu
from .trajectory import EMRIInspiral
from .ylm import GetYlms


def get_viewing_angles(qS, phiS, qK, phiK):
    R = np.array([np.sin(qS) * np.cos(phiS), np.sin(qS) * np.sin(phiS), np.cos(qS)])
    S = np.array([np.sin(qK) * np.cos(phiK), np.sin(qK) * np.sin(phiK), np.cos(qK)])
    theta = float(np.arccos(np.clip(-np.dot(R, S), -1.0, 1.0)))
    return theta, -np.pi / 2.0


def polarization_angle(qS, phiS, qK, phiK):
    up = np.cos(qS) * np.sin(qK) * np.cos(phiS - phiK) - np.cos(qK) * np.sin(qS)
    dw = np.sin(qK) * np.sin(phiS - phiK)
    return float(-np.arctan2(up, dw)) if dw != 0.0 else 0.5 * np.pi


class FastSchwarzschildEccentricFlux:
    """FD Schwarzschild-eccentric waveform (stand-in upstream, MI355X mode sum)."""

    descriptor = "eccentric"

    def __init__(self, inspiral_kwargs=None, amplitude_kwargs=None, sum_kwargs=None,
                 Ylm_kwargs=None, use_gpu=False, caustic="uniform", **kwargs):
        sum_kwargs = dict(sum_kwargs or {})
        # FEW's default output_type is "td" (InterpolatedModeSum); "fd" selects the FD sum
        self.output_type = sum_kwargs.pop("output_type", "td")
        if self.output_type not in ("fd", "td"):
            raise ValueError("sum_kwargs output_type must be 'fd' or 'td'")
        self.use_gpu = use_gpu
        self.inspiral_generator = EMRIInspiral(func="SchwarzEccFlux", **(inspiral_kwargs or {}))
        self.amplitude_generator = RomanAmplitude(**(amplitude_kwargs or {}))
        self.ylm_gen = GetYlms(assume_positive_m=True, **(Ylm_kwargs or {}))
        self.mode_selector = ModeSelector(self.amplitude_generator.m0mask)
        if self.output_type == "fd":
            sum_kwargs.setdefault("caustic", caustic)
            self.create_waveform = FDInterpolatedModeSum(use_gpu=use_gpu, **sum_kwargs)
        else:
            sum_kwargs.pop("caustic", None)
            self.create_waveform = TDInterpolatedModeSum(use_gpu=use_gpu, **sum_kwargs)
        self.last_modes = None
        self._ylm_cache = {}
        self._prefetched = {}
        self._prefetched_bytes = 0
        self._inflight = {}   # prefetch(wait=False): parameters -> the pool's Future
        self._lock = threading.Lock()

    # -- host-side upstream ------------------------------------------------------------------
    def _ylms(self, theta, phi):
        """GetYlms over the whole mode list, cached per viewing angle (the drivers' walkers
        share their sky and spin angles, emri_pe.py:161-167)."""
        key = (float(theta), float(phi))
        with self._lock:
            y = self._ylm_cache.get(key)
        if y is None:
            amp = self.amplitude_generator
            y = self.ylm_gen(amp.l_arr, amp.m_arr, theta, phi)
            with self._lock:
                if len(self._ylm_cache) > 64:
                    self._ylm_cache.clear()
                self._ylm_cache[key] = y
        return y

    def prepare(self, M, mu, p0, e0, theta, phi, dist, Phi_phi0=0.0, Phi_r0=0.0, T=1.0,
                eps=1e-5, mode_selection=None, include_minus_m=True):
        """Trajectory, amplitudes, Ylm and mode selection (host; stand-in physics).

        With libemrifd.so built, the trajectory, the amplitude model and the selection run in
        C++ (csrc/emrifd_host.cpp, emrifd_modes.cpp; the same equations and integrator as the
        numpy/scipy path below, which serves explicit mode_selection lists)."""
        key = None
        if mode_selection is None:
            key = (float(M), float(mu), float(p0), float(e0), float(theta), float(phi),
                   float(dist), float(Phi_phi0), float(Phi_r0), float(T), float(eps),
                   bool(include_minus_m))
            if self._inflight:
                with self._lock:
                    fut = self._inflight.pop(key, None)
                if fut is not None:
                    return fut.result()   # (a worker's exception is raised here)
            if self._prefetched:
                with self._lock:
                    hit = self._prefetched.pop(key, None)
                    if hit is not None:
                        self._prefetched_bytes -= _nbytes(hit)
                if hit is not None:
                    return hit
        return self._upstream(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, T, eps,
                              mode_selection, include_minus_m)

    def _upstream(self, M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, T, eps,
                  mode_selection, include_minus_m):
        """prepare()'s computation, no cache (the prefetch workers call it directly)."""
        amp = self.amplitude_generator
        lib = getattr(self.inspiral_generator, "lib", None)
        if lib is not None and mode_selection is None and hasattr(lib, "efd_host_modes"):
            t, p, e, Phi_phi, Phi_r, f_phi, f_r = self.inspiral_generator.with_frequencies(
                M, mu, 0.0, p0, e0, 1.0, Phi_phi0=Phi_phi0, Phi_r0=Phi_r0, T=T)
            ylms_all = self._ylms(theta, phi)
            keep, teuk = amp.select(p, e, ylms_all, eps, lib=lib)
            K = amp.num_teuk_modes
            ylms = np.concatenate([ylms_all[:K][keep], ylms_all[K:][keep]])
            if not include_minus_m:
                ylms[len(keep):] = 0.0
            mk, nk = amp.m_arr[keep], amp.n_arr[keep]
            self.last_modes = (amp.l_arr[keep], mk, nk)
            d = dict(t=t, p=p, e=e, Phi_phi=Phi_phi, Phi_r=Phi_r, teuk=teuk, ylms=ylms,
                     m=mk, n=nk, f_phi=f_phi, f_r=f_r)
            # host addresses of the mode sum's ten inputs, for the batched likelihood's native
            # staging (summation.BatchPreparer.flush; computed here, in the prefetch threads)
            arrs = (t, Phi_phi, Phi_r, f_phi, f_r, teuk, mk, nk, ylms)
            dts = (np.float64,) * 5 + (np.complex128, np.int32, np.int32, np.complex128)
            if all(a.flags.c_contiguous and a.dtype == dt for a, dt in zip(arrs, dts)):
                k = len(keep)
                ptr = [a.ctypes.data for a in arrs]
                # as packed bytes: the group's flush joins its walkers' in one call
                d["_src"] = np.array(ptr + [ptr[-1] + 16 * k], dtype=np.uint64).tobytes()
                d["_shape"] = np.array((len(t), k), dtype=np.int32).tobytes()
            return d
        t, p, e, x, Phi_phi, Phi_theta, Phi_r = self.inspiral_generator(
            M, mu, 0.0, p0, e0, 1.0, Phi_phi0=Phi_phi0, Phi_r0=Phi_r0, T=T)
        if mode_selection is not None:
            idx = []
            for lmn in mode_selection:
                l, m, n = (int(v) for v in lmn)
                if m < 0:
                    l, m, n = l, -m, -n  # FEW folds -m requests onto +m with the partner branch
                idx.append(amp.lmn_indices[(l, m, n)])
            keep = np.unique(np.asarray(idx, dtype=np.int64))
            teuk = amp(p, e)[:, keep]
            ylms = self.ylm_gen(amp.l_arr[keep], amp.m_arr[keep], theta, phi)
        else:
            teuk_all = amp(p, e)
            ylms_all = self.ylm_gen(amp.l_arr, amp.m_arr, theta, phi)
            keep = self.mode_selector(teuk_all, ylms_all, None, eps=eps)
            teuk = teuk_all[:, keep]
            K = amp.num_teuk_modes
            ylms = np.concatenate([ylms_all[:K][keep], ylms_all[K:][keep]])
        K = len(keep)
        if not include_minus_m:
            ylms = ylms.copy()
            ylms[K:] = 0.0
        self.last_modes = (amp.l_arr[keep], amp.m_arr[keep], amp.n_arr[keep])
        # orbital frequencies along the trajectory (FEW's get_fundamental_frequencies, as the
        # notebook's F(t) at Tutorial_FD_construction_single_mode.ipynb:227, 280)
        om_phi, _, om_r = get_fundamental_frequencies(0.0, p, e, 0.0)
        return dict(t=t, p=p, e=e, Phi_phi=Phi_phi, Phi_r=Phi_r, teuk=teuk, ylms=ylms,
                    m=amp.m_arr[keep], n=amp.n_arr[keep],
                    f_phi=om_phi / (2.0 * np.pi * M * MTSUN_SI),
                    f_r=om_r / (2.0 * np.pi * M * MTSUN_SI))

    def prefetch(self, calls, wait=True, concurrency=None):
        """Run the host upstream of several sources at once: `calls` are prepare() argument
        tuples (M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, T, eps). The native parts
        release the GIL, so a thread pool works a walker batch in parallel; the results are held
        for the prepare() calls that follow (each taken once).

        wait=False returns at once: each call's upstream runs on the pool (in `calls` order) and
        the prepare() call with its parameters waits for that one result only, so a caller
        working through the batch in groups starts a group's device work as soon as the
        group's own walkers are done, while the pool works on the next groups (the fused
        likelihood's half-step). concurrency (wait=False): at most that many calls run at once,
        started in `calls` order, each with the pool's threads / concurrency OpenMP threads, so
        a caller taking the batch in groups of that size gets its first group early (the
        windowed likelihood's groups then overlap the later walkers' upstream)."""
        calls = [tuple(c) for c in calls]
        # calls whose upstream is already in flight or held (an earlier prefetch of the same
        # batch, e.g. the likelihood's asynchronous one before spectrum_batch's) are not run
        # again: prepare() takes those results. Eviction first, and never of this batch's own
        # entries (which would then be recomputed serially in prepare())
        with self._lock:
            self._evict_inflight({tuple(float(v) for v in c[:11]) + (True,) for c in calls})
            calls = [c for c in calls
                     if (k := tuple(float(v) for v in c[:11]) + (True,)) not in self._inflight
                     and k not in self._prefetched]
        if not calls:
            return 0
        for c in calls:                       # Ylm per viewing angle before the threads start
            self._ylms(c[4], c[5])
        pool = _pool()
        # a batch smaller than the pool gives each walker's mode selection several OpenMP
        # threads (efd_host_set_threads is per calling thread; bitwise the same result)
        limit = len(calls) if (wait or not concurrency) else max(1, min(int(concurrency),
                                                                        len(calls)))
        per = max(1, pool._max_workers // max(1, limit))
        if os.environ.get("EFD_PREFETCH_SPLIT", "1") == "0":
            per = 1
        lib = _lib.load()

        def run(c):
            lib.efd_host_set_threads(per)
            return self._upstream(*c, None, True)

        if limit < len(calls):
            # start the calls in order, `limit` at a time (a task waits for its turn and a
            # free slot; every task releases its slot however it ends)
            cond = threading.Condition()
            state = {"next": 0, "running": 0}

            def run_ordered(i, c):
                with cond:
                    cond.wait_for(lambda: state["next"] == i and state["running"] < limit)
                    state["next"] += 1
                    state["running"] += 1
                    cond.notify_all()
                try:
                    return run(c)
                finally:
                    with cond:
                        state["running"] -= 1
                        cond.notify_all()

            with self._lock:
                for i, c in enumerate(calls):
                    self._inflight[tuple(float(v) for v in c[:11]) + (True,)] = \
                        pool.submit(run_ordered, i, c)
            return len(calls)

        if not wait:
            with self._lock:
                for c in calls:
                    self._inflight[tuple(float(v) for v in c[:11]) + (True,)] = pool.submit(run, c)
            return len(calls)
        res = list(pool.map(run, calls))
        with self._lock:
            # results nobody took (a batch interrupted by an exception, parameters the caller
            # then changed) are dropped once they would hold more than PREFETCH_MAX_BYTES of
            # host memory (each holds the walker's amplitudes, N_t x K complex, and trajectory)
            add = sum(_nbytes(r) for r in res)
            if self._prefetched_bytes + add > self.PREFETCH_MAX_BYTES:
                self._prefetched.clear()
                self._prefetched_bytes = 0
            for c, r in zip(calls, res):
                key = tuple(float(v) for v in c[:11]) + (True,)
                old = self._prefetched.pop(key, None)
                if old is not None:
                    self._prefetched_bytes -= _nbytes(old)
                self._prefetched[key] = r
                self._prefetched_bytes += _nbytes(r)
        return len(res)

    PREFETCH_MAX_BYTES = 1 << 30
    INFLIGHT_MAX = 4096

    def _evict_inflight(self, keep):
        """Drop in-flight entries nobody took (the caller holds self._lock), keeping the keys in
        `keep` (the batch being prefetched): finished ones first once they hold more than
        PREFETCH_MAX_BYTES of host memory or the table exceeds INFLIGHT_MAX entries, then the
        oldest unfinished ones past INFLIGHT_MAX (dropped when they finish)."""
        done = [(k, f) for k, f in self._inflight.items()
                if k not in keep and f.done() and not f.cancelled()]
        held = 0
        for _, f in done:
            try:
                held += _nbytes(f.result())
            except Exception:
                pass
        if held > self.PREFETCH_MAX_BYTES or len(self._inflight) > self.INFLIGHT_MAX:
            for k, _ in done:
                del self._inflight[k]
        over = len(self._inflight) - self.INFLIGHT_MAX
        if over > 0:
            for k in [k for k in self._inflight if k not in keep][:over]:
                del self._inflight[k]

    def spectrum(self, M, mu, p0, e0, theta, phi, dist, Phi_phi0=0.0, Phi_r0=0.0, dt=10.0,
                 T=1.0, eps=1e-5, mode_selection=None, include_minus_m=True, f_arr=None,
                 extra_scale=1.0 + 0.0j, out=None, check=True, **kwargs):
        """Complex FD spectrum S = h+ - i hx (torch, on the GPU), distance-scaled; for
        output_type "td" the complex time series h = h+ - i hx instead. FD: out (complex128
        [N_f] on the device) receives S; check=False queues without the status
        synchronisation (the caller reads the engine's status later)."""
        require_gpu()
        if self.output_type == "td":
            return self.time_series(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, dt, T,
                                    eps, mode_selection, include_minus_m, extra_scale)
        d = self.prepare(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, T, eps,
                         mode_selection, include_minus_m)
        K = len(d["m"])
        scale = complex(extra_scale) * (mu * MRSUN_SI / (dist * Gpc))
        return self.create_waveform.spectrum(d["t"], d["teuk"], d["ylms"][:K], d["ylms"][K:],
                                             d["Phi_phi"], d["Phi_r"], d["m"], d["n"], M, d["p"],
                                             d["e"], dt=dt, T=T, f_arr=f_arr, scale=scale,
                                             f_phi=d["f_phi"], f_r=d["f_r"], out=out,
                                             check=check)

    def submit_channels(self, pipeline, out, M, mu, p0, e0, theta, phi, dist, Phi_phi0=0.0,
                        Phi_r0=0.0, dt=10.0, T=1.0, eps=1e-5, mode_selection=None,
                        include_minus_m=True, f_arr=None, extra_scale=1.0 + 0.0j, order=True,
                        prepare_only=False, **kwargs):
        """Queue [h+, hx] over f >= 0 into out on a WaveformPipeline slot (FD only).
        prepare_only: queue the upload and preparation only and leave the sum's job on the slot
        (out unused; Likelihood's fused batch path)."""
        if self.output_type != "fd":
            raise ValueError("submit_channels is the FD path")
        d = self.prepare(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, T, eps,
                         mode_selection, include_minus_m)
        K = len(d["m"])
        scale = complex(extra_scale) * (mu * MRSUN_SI / (dist * Gpc))
        return self.create_waveform.submit_channels(
            pipeline, out, d["t"], d["teuk"], d["ylms"][:K], d["ylms"][K:], d["Phi_phi"],
            d["Phi_r"], d["m"], d["n"], M, d["p"], d["e"], dt=dt, T=T, f_arr=f_arr, scale=scale,
            f_phi=d["f_phi"], f_r=d["f_r"], order=order, prepare_only=prepare_only)

    def time_series(self, M, mu, p0, e0, theta, phi, dist, Phi_phi0=0.0, Phi_r0=0.0, dt=10.0,
                    T=1.0, eps=1e-5, mode_selection=None, include_minus_m=True,
                    extra_scale=1.0 + 0.0j):
        """Complex TD waveform h = h+ - i hx at t_i = i dt (torch, on the GPU)."""
        require_gpu()
        d = self.prepare(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, T, eps,
                         mode_selection, include_minus_m)
        K = len(d["m"])
        scale = complex(extra_scale) * (mu * MRSUN_SI / (dist * Gpc))
        return self.create_waveform.waveform(d["t"], d["teuk"], d["ylms"][:K], d["ylms"][K:],
                                             d["Phi_phi"], d["Phi_r"], d["m"], d["n"], M, d["p"],
                                             d["e"], dt=dt, T=T, scale=scale)

    def __call__(self, M, mu, p0, e0, theta, phi, dist=1.0, Phi_phi0=0.0, Phi_r0=0.0, dt=10.0,
                 T=1.0, eps=1e-5, show_progress=False, batch_size=-1, mode_selection=None,
                 include_minus_m=True, f_arr=None, mask_positive=False, **kwargs):
        """FEW output: FD stacked [h+, hx] (2, N) in the source frame; TD complex h."""
        torch = require_gpu()
        if self.output_type == "td":
            h = self.time_series(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, dt, T, eps,
                                 mode_selection, include_minus_m)
            return h if self.use_gpu else h.cpu().numpy()
        S = self.spectrum(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, dt, T, eps,
                          mode_selection, include_minus_m, f_arr)
        hp, hc = self.create_waveform.polarizations(S, mask_positive)
        out = torch.stack([hp, hc])
        return out if self.use_gpu else out.cpu().numpy()


def _nbytes(d):
    """Host bytes held by one prepared upstream result (its numpy arrays)."""
    return sum(v.nbytes for v in d.values() if isinstance(v, np.ndarray))


_WAVEFORMS = {"FastSchwarzschildEccentricFlux": FastSchwarzschildEccentricFlux}
_POOL = None


def _pool():
    """Threads for the host upstream of walker batches (its native parts release the GIL):
    one per core of this rank's disjoint host share (hostcpu.threads(): the node's cores split
    over LOCAL_WORLD_SIZE ranks, at most 16; OMP_NUM_THREADS does not decide it)."""
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        from . import hostcpu
        _POOL = ThreadPoolExecutor(max_workers=hostcpu.threads(),
                                   thread_name_prefix="efd-upstream")
    return _POOL


class GenerateEMRIWaveform:
    """Generic EMRI generator with FEW's 14-parameter call (frame handling + list output)."""

    def __init__(self, waveform_class, *args, frame="detector", return_list=False, **kwargs):
        if isinstance(waveform_class, str):
            if waveform_class not in _WAVEFORMS:
                raise ValueError(f"unknown waveform {waveform_class!r}; available: "
                                 f"{sorted(_WAVEFORMS)}")
            waveform_class = _WAVEFORMS[waveform_class]
        if frame not in ("detector", "source"):
            raise ValueError("frame must be 'detector' or 'source'")
        self.waveform_generator = waveform_class(*args, **kwargs)
        self.frame = frame
        self.return_list = return_list
        self._angle_cache = {}

    def _angles(self, qS, phiS, qK, phiK):
        """(theta, phi, rot) of a sky position and spin orientation: the source-frame viewing
        angles and the detector-frame rotation exp(-2 i psi) (1 in the source frame), cached
        per angle set (the drivers' walkers share them, emri_pe.py:161-167)."""
        key = (float(qS), float(phiS), float(qK), float(phiK))
        v = self._angle_cache.get(key)
        if v is None:
            theta, phi = get_viewing_angles(qS, phiS, qK, phiK)
            rot = 1.0 + 0.0j
            if self.frame == "detector":
                rot = complex(np.exp(-2j * polarization_angle(qS, phiS, qK, phiK)))
            if len(self._angle_cache) > 4096:
                self._angle_cache.clear()
            v = self._angle_cache[key] = (theta, phi, rot)
        return v

    @property
    def use_gpu(self):
        return self.waveform_generator.use_gpu

    def _spectrum(self, M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0, Phi_theta0,
                  Phi_r0, **kwargs):
        # a, x0, Phi_theta0 are ignored for Schwarzschild (emri_pe.py:598, 602)
        theta, phi, rot = self._angles(qS, phiS, qK, phiK)
        gen = self.waveform_generator
        return gen.spectrum(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, extra_scale=rot,
                            **kwargs)

    def submit_channels(self, pipeline, out, M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK,
                        Phi_phi0, Phi_theta0, Phi_r0, k0=None, **kwargs):
        """fill_channels on a WaveformPipeline slot: queued, no host synchronisation (the
        walker loop of Likelihood.get_ll keeps several templates in flight). Returns the slot;
        work that reads out belongs on pipeline.stream(slot)."""
        gen = self.waveform_generator
        if k0 is not None and gen.output_type == "fd":
            # checked before anything is queued (the grid is set up from the call's kwargs)
            cw = gen.create_waveform
            cw._grid(kwargs.get("T", 1.0), kwargs.get("dt", 10.0), kwargs.get("f_arr"))
            if k0 != cw.positive_start():
                raise ValueError("positive_frequency_mask does not match the generator's grid")
        theta, phi, rot = self._angles(qS, phiS, qK, phiK)
        return gen.submit_channels(pipeline, out, M, mu, p0, e0, theta, phi, dist, Phi_phi0,
                                   Phi_r0, extra_scale=rot, **kwargs)

    def submit_batch(self, preparer, params, k0=None, T=1.0, dt=10.0, eps=1e-5, f_arr=None,
                     mode_selection=None, include_minus_m=True, **kwargs):
        """submit_channels(prepare_only=True) for every row of params (B x 14) into a
        BatchPreparer: the grid is checked once, the angles come from the per-angle cache and
        the host upstream from prepare() (prefetched results when there are any), so a walker
        costs its dictionary lookups and the preparer's bookkeeping. Same templates, bitwise,
        as B calls of submit_channels."""
        gen = self.waveform_generator
        if gen.output_type != "fd":
            raise ValueError("submit_batch is the FD path")
        cw = gen.create_waveform
        freq, sym = cw._grid(T, dt, f_arr)
        if k0 is not None and k0 != cw.positive_start():
            raise ValueError("positive_frequency_mask does not match the generator's grid")
        if not sym:
            raise ValueError("submit_batch needs a symmetric grid (the fused likelihood's)")
        kc = cw._k0
        submit = preparer.submit
        # the native upstream's walkers go straight onto the preparer's pending list (what
        # submit(d, freq, True, scale, k0=kc, prepare_only=True) appends, without its argument
        # handling per walker)
        pend = getattr(preparer, "_pending", None)
        room = getattr(preparer, "group", 0)
        for prm in np.asarray(params, dtype=np.float64).reshape(-1, 14).tolist():
            M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0, Phi_theta0, Phi_r0 = prm
            theta, phi, rot = self._angles(qS, phiS, qK, phiK)
            d = gen.prepare(M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, T, eps,
                            mode_selection, include_minus_m)
            scale = rot * (mu * MRSUN_SI / (dist * Gpc))   # the spectrum path's rounding
            if "_src" in d:
                # the native upstream recorded its arrays' addresses: the preparer stages them
                # straight from prepare()'s dict
                if pend is not None and len(pend) < room:
                    pend.append((d, freq, True, complex(scale), int(kc), False))
                else:
                    submit(d, freq, True, scale, k0=kc, prepare_only=True)
                continue
            K = len(d["m"])
            y = d["ylms"]
            submit(dict(t=d["t"], amp=d["teuk"], phi_phi=d["Phi_phi"], phi_r=d["Phi_r"],
                        f_phi=d["f_phi"], f_r=d["f_r"], m=d["m"], n=d["n"], ylm_p=y[:K],
                        ylm_m=y[K:], _keep=d), freq, True, scale, k0=kc, prepare_only=True)

    # waveforms per device group of generate_batch: one packed upload, one
    # efd_modesum_prepare_batch and one efd_modesum_sum_batch each (EFD_BATCH_MAX at most)
    BATCH_GROUP = 16

    def generate_batch(self, params, out, T=1.0, dt=10.0, eps=1e-5, f_arr=None, **kwargs):
        """[h+, hx] over f >= 0 of every row of params (B x 14, FEW's order) into out
        (complex128 [B][2][N_pos] on the device): the vectorised form of B calls
        `self(*row, T=T, dt=dt, eps=eps, mask_positive=True)` with return_list=True (bitwise
        the same values), for scans like check_mode_by_mode.py:183-229 and batches of walkers.

        The host upstream of all rows runs at once on the thread pool (prefetch: trajectory,
        amplitudes, selection; this rank's host-core share), then the device work goes in
        groups of BATCH_GROUP: one packed upload and one efd_modesum_prepare_batch per group on
        that group's stream, one efd_modesum_sum_batch writing the group's h+/hx on the same
        stream, two groups in flight. Returns out, ordered after the work on the current stream."""
        torch = require_gpu()
        npos = self._batch_grid(T, dt, f_arr)[1]
        B = len(np.asarray(params, dtype=np.float64).reshape(-1, 14))
        if tuple(out.shape) != (B, 2, npos) or out.dtype != torch.complex128:
            raise ValueError(f"out must be complex128 [{B}][2][{npos}]")
        return self._run_batch(params, out, lambda j: dict(hp=torch.view_as_real(out[j, 0]),
                                                           hc=torch.view_as_real(out[j, 1])),
                               T, dt, eps, f_arr, kwargs)

    def spectrum_batch(self, params, out, T=1.0, dt=10.0, eps=1e-5, f_arr=None, lanes=None,
                       check=True, lanes_host=None, **kwargs):
        """The two-sided spectra S = h+ - i hx of every row of params into the rows of out
        (complex128 [B][N], contiguous rows, on the device): generate_batch's device groups
        with the sum writing S (the windowed templates' input, fdutils.HannConvolution); bitwise
        the spectrum path's S of each row. lanes (int32 [B][2] on the device, optional): each
        row's lane range (efd_modesum_lane_ranges), the bins its terms can reach. check=False
        leaves the device-side status unread (no host synchronisation here): the caller then
        calls check_batch() once its own work on the spectra is queued. lanes_host (pinned int32
        [B][2], with lanes): the lane ranges are gathered right after each group's preparation
        and copied there on a side stream, beside the sum; lanes_ready() waits for those copies
        only, so the host can read them while the sums run."""
        torch = require_gpu()
        n = self._batch_grid(T, dt, f_arr)[0]
        B = len(np.asarray(params, dtype=np.float64).reshape(-1, 14))
        if (out.dim() != 2 or tuple(out.shape) != (B, n) or out.dtype != torch.complex128
                or not out.is_contiguous()):
            raise ValueError(f"out must be contiguous complex128 [{B}][{n}]")
        if lanes is not None and (tuple(lanes.shape) != (B, 2) or lanes.dtype != torch.int32
                                  or not lanes.is_contiguous()):
            raise ValueError(f"lanes must be contiguous int32 [{B}][2]")
        if lanes_host is not None and (lanes is None or tuple(lanes_host.shape) != (B, 2)
                                       or lanes_host.dtype != torch.int32
                                       or not lanes_host.is_pinned()):
            raise ValueError(f"lanes_host must be pinned int32 [{B}][2] beside lanes")
        return self._run_batch(params, out, lambda j: dict(out=torch.view_as_real(out[j])),
                               T, dt, eps, f_arr, kwargs, lanes=lanes, check=check,
                               lanes_host=lanes_host)

    def lanes_ready(self):
        """Wait for the last spectrum_batch's lane-range copies into lanes_host (each group's
        event; the sums behind them keep running)."""
        st = getattr(self, "_gen_batch", None)
        if st is not None:
            for ev in st.get("lanes_ev_used", ()):
                ev.synchronize()

    def check_batch(self):
        """Synchronise the last batch's groups and raise if a workspace reported a device-side
        error (what spectrum_batch(check=False) skipped)."""
        st = getattr(self, "_gen_batch", None)
        if st is not None:
            st["prep"].wait()

    def positive_bins(self, T=1.0, dt=10.0, f_arr=None):
        """N_pos, the f >= 0 bins of the grid generate_batch writes (its out's last dimension)."""
        return self._batch_grid(T, dt, f_arr)[1]

    def _batch_grid(self, T, dt, f_arr):
        gen = self.waveform_generator
        if gen.output_type != "fd":
            raise ValueError("the batched generator is the FD path")
        cw = gen.create_waveform
        freq, sym = cw._grid(T, dt, f_arr)
        if not sym:
            raise ValueError("the batched generator needs a symmetric grid")
        return int(freq.numel()), int(freq.numel()) - cw._k0

    def _run_batch(self, params, out, outputs, T, dt, eps, f_arr, kwargs, lanes=None,
                   check=True, lanes_host=None):
        torch = require_gpu()
        from .summation import BatchPreparer, sum_batch
        cw = self.waveform_generator.create_waveform
        params = np.asarray(params, dtype=np.float64).reshape(-1, 14)
        B = len(params)
        if B == 0:
            return out
        self.prefetch(params, T=T, dt=dt, eps=eps, **kwargs)
        G = min(self.BATCH_GROUP, _lib.EFD_BATCH_MAX)
        st = getattr(self, "_gen_batch", None)
        if (st is None or st["prep"].caustic != cw.caustic or st["device"] != out.device
                or st["prep"].group != G):
            st = self._gen_batch = dict(
                prep=BatchPreparer(group=G, depth=2, caustic=cw.caustic, device=out.device),
                device=out.device,
                ev=[torch.cuda.Event(), torch.cuda.Event()],
                lanes_ev=[torch.cuda.Event(), torch.cuda.Event()],
                prep_ev=[torch.cuda.Event(), torch.cuda.Event()],
                lstream=torch.cuda.Stream(out.device))
        prep = st["prep"]
        cur = torch.cuda.current_stream(out.device)
        prep.order_after_current()
        # each group's sum on the group's own stream, right behind its preparation (no
        # cross-stream wait between the two: ~34 us of idle device a group in the windowed
        # trace, r05zg); group i + 1's preparation on the other stream still runs beside it,
        # and the current stream joins every used group stream at the end
        used = []
        st["lanes_ev_used"] = []
        try:
            for g0 in range(0, B, G):
                rows = params[g0:g0 + G]
                self.submit_batch(prep, rows, T=T, dt=dt, eps=eps, f_arr=f_arr, **kwargs)
                gi, jobs = prep.flush()
                # joined at the end however the rest of the group's queueing ends (its
                # preparation is on the stream already)
                if gi not in used:
                    used.append(gi)
                gs = prep.stream(gi)
                if lanes_host is not None:
                    pev = st["prep_ev"][gi]
                    pev.record(gs)
                sum_batch([(eng, dict(kw, **outputs(g0 + i)))
                           for i, (eng, kw) in enumerate(jobs)], stream=gs.cuda_stream)
                if lanes is not None:   # the preparation's segment ranges
                    # with lanes_host: gathered and copied on a side stream behind the
                    # preparation, beside the sum, so the host has them while the sum runs;
                    # the group's release waits for that stream too
                    ls = st["lstream"] if lanes_host is not None else gs
                    if lanes_host is not None:
                        ls.wait_event(pev)
                    _lib.check(prep.lib.efd_modesum_lane_ranges(
                        prep.groups[gi]["pw"], len(jobs), lanes[g0].data_ptr(),
                        ls.cuda_stream), "efd_modesum_lane_ranges", prep.lib)
                    if lanes_host is not None:
                        _lib.check(prep.lib.efd_download(
                            lanes_host[g0].data_ptr(), lanes[g0].data_ptr(), 8 * len(jobs),
                            ls.cuda_stream), "efd_download", prep.lib)
                        lev = st["lanes_ev"][gi]
                        lev.record(ls)
                        st["lanes_ev_used"].append(lev)
                        gs.wait_event(lev)
                ev = st["ev"][gi]
                ev.record(gs)
                prep.release(gi, ev)
        finally:
            prep._pending = []
            for gi in used:
                cur.wait_stream(prep.stream(gi))
            if lanes_host is not None and used:
                cur.wait_stream(st["lstream"])
        if check:
            prep.wait()   # device-side errors of the groups' workspaces raise here
        return out

    # prefetch(wait=False) is supported (the likelihood's groups then overlap the upstream)
    PREFETCH_ASYNC = True

    def prefetch(self, params, T=1.0, dt=10.0, eps=1e-5, mode_selection=None,
                 include_minus_m=True, wait=True, concurrency=None, **kwargs):
        """The host upstream of a batch of 14-parameter sets at once (thread pool; see
        FastSchwarzschildEccentricFlux.prefetch); later calls with the same parameters and
        kwargs take the results. Only for the FD generator without an explicit mode list."""
        gen = self.waveform_generator
        if gen.output_type != "fd" or mode_selection is not None or not include_minus_m:
            return 0
        calls = []
        # rows as Python floats (one tolist(): unpacking numpy rows costs ~5x more a walker)
        for prm in np.asarray(params, dtype=np.float64).reshape(-1, 14).tolist():
            M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0, Phi_theta0, Phi_r0 = prm
            theta, phi, _ = self._angles(qS, phiS, qK, phiK)
            calls.append((M, mu, p0, e0, theta, phi, dist, Phi_phi0, Phi_r0, T, eps))
        return (gen.prefetch(calls) if wait
                else gen.prefetch(calls, wait=False, concurrency=concurrency))

    def fill_channels(self, out, *params, k0=None, **kwargs):
        """Write [h+, hx] over f >= 0 into the rows of out (complex128 [2][N_pos], device).

        The fused path of fdutils.get_fd_waveform_fromFD: same values as
        `self(*params, mask_positive=True)` with `return_list=True`, without the copies.
        """
        S = self._spectrum(*params, **kwargs)
        cw = self.waveform_generator.create_waveform
        if k0 is not None and k0 != cw.positive_start():
            raise ValueError("positive_frequency_mask does not match the generator's grid")
        cw.polarizations(S, True, out=(out[0], out[1]))
        return out

    def __call__(self, M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0, Phi_theta0,
                 Phi_r0, *add_args, mask_positive=False, **kwargs):
        gen = self.waveform_generator
        if gen.output_type == "td":
            # f_arr / mask_positive are FD options; FEW's TD sum has no use for them
            kwargs.pop("f_arr", None)
            h = self._spectrum(M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0,
                               Phi_theta0, Phi_r0, **kwargs)
            out = list(gen.create_waveform.polarizations(h)) if self.return_list else h
            if self.use_gpu:
                return out
            return [o.cpu().numpy() for o in out] if isinstance(out, list) else out.cpu().numpy()
        S = self._spectrum(M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0, Phi_theta0,
                           Phi_r0, **kwargs)
        cw = gen.create_waveform
        if self.return_list:
            hp, hc = cw.polarizations(S, mask_positive)
            out = [hp, hc]
        else:
            if mask_positive:
                S = S[cw.positive_start():]
            out = S
        if self.use_gpu:
            return out
        return [o.cpu().numpy() for o in out] if isinstance(out, list) else out.cpu().numpy()

"""lisatools-compatible Gaussian likelihood with the reduction on the device.

Mirror of LISAanalysistools/lisatools/sampling/likelihood.py `Likelihood` (:13-334) for the FD
templates the reference drivers use (emri_pe.py:381-414: two channels h+, hx over f >= 0,
noise_fn = FDutils.get_sensitivity, f_arr = frequency[frequency >= 0]):

  inject_signal (:80-234)  data d = inj * sqrt(diff(f)/PSD) and the noise factor
                           w = sqrt(diff(f)/PSD), diff(f)[0] = diff(f)[1]; repeated
                           injections add up; add_noise raises NotImplementedError (as :199)
  get_ll (:236-293)        per walker: template h, ll = -1/2 * 4 * sum |d - h w|^2 over
                           channels and bins, skipping bin 0 when w[0][0] is NaN (:268)
  __call__ (:295-334)      parameter transform, transpose_params, `subset` batching

What changes is where the work happens. Data and noise factor live on the device. On
symmetric grids (FEW's own and the drivers' downsampled f_arr) the walkers' mode sums run a few
at a time in one launch with the likelihood fused into the sum's epilogue
(efd_modesum_sum_loglike): the templates are never written, each walker's logL lands in its slot
of a device result vector, and the batch costs one host synchronisation. Otherwise (or with
fused_likelihood = False) each walker's template is reduced by efd_loglike (HIP) straight from
the template buffer, and the 2 x N_pos residual d - h w is never materialised. When the template is this package's
get_fd_waveform_fromFD around a GenerateEMRIWaveform (the drivers' case), h+ and hx are written
by efd_polarizations directly into one reusable [2][N_pos] buffer (the stream orders reuse), and
non_zero_mask is folded into the template weight (w * mask) instead of zeroing h.
Results are numpy float64 arrays ([B]), or device tensors with use_gpu=True, return_cupy=True.
Time-domain templates (dt only) are not part of this path: get_ll raises NotImplementedError.
"""

import ctypes
import os
import sys

import numpy as np

from . import _lib
from .summation import require_gpu


class Likelihood:
    def __init__(self, template_model, num_channels, dt=None, df=None, f_arr=None,
                 parameter_transforms=None, use_gpu=False, vectorized=False,
                 separate_d_h=False, return_cupy=False, fill_data_noise=False,
                 transpose_params=False, subset=None):
        self.subset = subset
        self.transpose_params = transpose_params
        self.template_model = template_model
        self.parameter_transforms = parameter_transforms
        self.fill_data_noise = fill_data_noise
        self.use_gpu = use_gpu
        self.vectorized = vectorized
        self.num_channels = num_channels
        self.separate_d_h = separate_d_h
        if dt is None and df is None and f_arr is None:
            raise ValueError("Must provide dt, df or f_arr.")
        self.dt, self.df, self.f_arr = dt, df, f_arr
        self.frequency_domain = df is not None or f_arr is not None
        self.return_cupy = return_cupy
        self.noise_has_been_added = False
        self.torch = torch = require_gpu()
        self.device = torch.device("cuda", torch.cuda.current_device())
        from .reductions import Reducer
        self._red = Reducer(self.device)
        self._buf = None
        # walkers whose templates are in flight at once in get_ll (WaveformPipeline slots);
        # one HIP stream each (the box exposes 4 hardware queues per process)
        self.num_streams = 4
        # pipelined templates on symmetric grids: the walkers' mode sums run FUSED_GROUP at a
        # time in one launch with the likelihood in its epilogue (efd_modesum_sum_loglike), so
        # no template is written; False keeps one template buffer + efd_loglike per walker
        self.fused_likelihood = True
        self._fused = None
        self._tile_const = None
        self._specific_likelihood_setup()

    def _specific_likelihood_setup(self):
        if isinstance(self.template_model, list):
            raise ValueError("For single likelihood, template model cannot be a list.")
        if hasattr(self.template_model, "get_ll"):
            self.get_ll = self.template_model.get_ll
            self.like_here = False
        else:
            self.fill_data_noise = False
            self.like_here = True

    # ---------------------------------------------------------------------------------------
    def inject_signal(self, data_stream=None, params=None, waveform_kwargs={}, noise_fn=None,
                      noise_kwargs={}, add_noise=False):
        torch = self.torch
        # the injection's parameters when the data is exactly the template model's output for
        # them (a single injection, no noise): the windowed logL's per-bin data is then made by
        # the logL's own arithmetic (get_fd_waveform_fromFD.hann_local)
        first = not hasattr(self, "injection_channels")
        self._inj_call = None
        if params is not None:
            if self.parameter_transforms is not None:
                key = list(self.parameter_transforms.keys())[0]
                params = self.parameter_transforms[key].both_transforms(params)
            injection_channels = _to_numpy(self.template_model(*params, **waveform_kwargs))
            if first:
                self._inj_call = (np.asarray(params, dtype=np.float64).reshape(-1),
                                  dict(waveform_kwargs))
        elif data_stream is not None:
            if isinstance(data_stream, list) is False:
                raise ValueError("If data_stream is provided, it must be as a list.")
            made_by = getattr(self.template_model, "made_by", None)
            if first and made_by is not None:
                self._inj_call = made_by(data_stream)
            injection_channels = _to_numpy(data_stream)
        else:
            raise ValueError("Must provide data_stream or params kwargs to inject signal.")

        self.injection_length = len(injection_channels[0])
        for inj in injection_channels:
            if len(inj) != self.injection_length:
                raise ValueError("Length of all injection channels must match.")
        if len(injection_channels) != self.num_channels:
            raise ValueError("Number of channels from template_model does not match number of "
                             "channels declare by user.")

        if isinstance(noise_fn, list):
            if len(noise_fn) != 1 and len(noise_fn) != self.num_channels:
                raise ValueError("Number of noise functions does not match number of channels "
                                 "declared by user.")
            elif len(noise_fn) == 1:
                noise_fn = [noise_fn[0] for _ in range(self.num_channels)]
        else:
            noise_fn = [noise_fn for _ in range(self.num_channels)]
        if isinstance(noise_kwargs, list):
            if len(noise_kwargs) != 1 and len(noise_kwargs) != self.num_channels:
                raise ValueError("Number of noise kwargs does not match number of channels "
                                 "declared by user.")
            elif len(noise_kwargs) == 1:
                noise_kwargs = [noise_kwargs[0] for _ in range(self.num_channels)]
        else:
            noise_kwargs = [noise_kwargs for _ in range(self.num_channels)]

        if self.frequency_domain:
            if self.df is not None:
                freqs = np.arange(self.injection_length) * self.df
                can_add_noise = True
            else:
                freqs = _to_numpy(self.f_arr)
                can_add_noise = False
        else:
            freqs = np.fft.rfftfreq(self.injection_length, self.dt)
            can_add_noise = True
        psd = [np.asarray(_to_numpy(fn(freqs, **kw)), dtype=np.float64)
               for fn, kw in zip(noise_fn, noise_kwargs)]
        if self.frequency_domain is False:
            injection_channels = [np.fft.rfft(inj) * self.dt for inj in injection_channels]

        diff_freqs = np.zeros_like(freqs)
        diff_freqs[1:] = np.diff(freqs)
        diff_freqs[0] = diff_freqs[1]
        self.base_injections = injection_channels
        if add_noise and can_add_noise and self.noise_has_been_added is False:
            raise NotImplementedError   # as the reference (likelihood.py:199)

        with np.errstate(invalid="ignore", divide="ignore"):
            nf = np.asarray([(diff_freqs / p) ** 0.5 for p in psd])
        weighted = np.asarray([np.asarray(inj) * w for inj, w in zip(injection_channels, nf)],
                              dtype=np.complex128)
        self.noise_factor = torch.as_tensor(nf, dtype=torch.float64, device=self.device)
        if hasattr(self, "injection_channels") is False:
            self.injection_channels = torch.as_tensor(weighted, device=self.device)
            self.freqs = torch.as_tensor(freqs, dtype=torch.float64, device=self.device)
        else:
            self.injection_channels = self.injection_channels + torch.as_tensor(
                weighted, device=self.device)
        self.data_length = int(self.injection_channels.shape[1])
        self.psd = psd
        self._prepare_reduction()

    def _prepare_reduction(self):
        """Device copies used by efd_loglike: skip bin 0 by zeroing it when w[0][0] is NaN."""
        torch = self.torch
        d = self.injection_channels.contiguous().clone()
        w = self.noise_factor.contiguous().clone()
        self.start_ind = 1 if bool(torch.isnan(self.noise_factor[0, 0]).item()) else 0
        if self.start_ind:
            d[:, 0] = 0.0
            w[:, 0] = 0.0
        self._d, self._w = d, w
        self._w_templ = w
        self._tile_const = None   # (their tile constants are made again on the next call)
        self._hloc = None         # the windowed logL's per-bin data (made on the next call)
        tm = self.template_model
        mask = getattr(tm, "non_zero_mask", None)
        if mask is not None and getattr(tm, "can_fill", False):
            self._w_templ = (w * mask.to(torch.float64)[None, :]).contiguous()

    # ---------------------------------------------------------------------------------------
    def get_ll(self, params, *args, **kwargs):
        torch = self.torch
        if self.frequency_domain is False:
            raise NotImplementedError("time-domain templates are not part of the FD path")
        num_likes = params.shape[0]
        out = torch.empty(num_likes, dtype=torch.float64, device=self.device)
        nch, nb = self._d.shape
        tm = self.template_model
        if self.vectorized:
            h_all = tm(*params, *args, **kwargs)
            for i in range(num_likes):
                h = self._as_channels(h_all[i])
                self._red.loglike(h, self._d, self._w, out=out[i:i + 1])
        elif (getattr(tm, "can_pipeline", False) and self.fused_likelihood
              and (host := self._get_ll_fused(tm, params, args, kwargs, out)) is not None):
            if self.noise_has_been_added:
                raise NotImplementedError
            if self.use_gpu and self.return_cupy:
                return out
            return host
        elif getattr(tm, "can_pipeline", False):
            # several walkers in flight: each pipeline slot has its own template buffer,
            # stream and reduction scratch; walker i's template and logL run on one slot's
            # stream, the batch costs one host synchronisation
            P = self._pipeline_for(tm)
            P.order_after_current()
            _prefetch(tm, params, args, kwargs)
            for i, params_i in enumerate(params):
                j = P.next_slot()
                slot = tm.submit(P, self._pbufs[j], *params_i, *args, order=False, **kwargs)
                with torch.cuda.stream(P.stream(slot)):
                    self._preds[slot].loglike(self._pbufs[slot], self._d, self._w_templ,
                                              out=out[i:i + 1])
            P.wait()
        elif getattr(tm, "can_fill_batch", False) and not args:
            # windowed templates (the drivers' Hann window): groups of WINDOW_GROUP walkers,
            # their spectra in one buffer and the window's transforms batched over them
            # and the windowed templates' logL reduced in place (efd_hann_loglike, at most
            # EFD_HANN_ROWS_MAX rows a call). The batch takes keyword waveform arguments only;
            # extra positional ones go to the per-walker fill below, which forwards them
            G = min(max(1, int(os.environ.get("EFD_WINDOW_GROUP", 0))
                        or int(getattr(tm, "WINDOW_GROUP", 8))), _lib.EFD_HANN_ROWS_MAX)
            scr = getattr(self, "_wscratch", None)
            per_row = max(_lib.EFD_LOGLIKE_SCRATCH, _lib.EFD_HANN_LOCAL_PARTIALS)
            if scr is None or scr.numel() < G * per_row:
                scr = self._wscratch = torch.empty(G * per_row, dtype=torch.float64,
                                                   device=self.device)
            local = self._hann_local(tm, kwargs)
            # the upstream G walkers at a time, in order: the first group's device work then
            # overlaps the later walkers' upstream
            _prefetch(tm, params, args, kwargs, concurrency=G if G < num_likes else None)
            for g0 in range(0, num_likes, G):
                rows = params[g0:g0 + G]
                tm.loglike_batch(out[g0:g0 + len(rows)], rows, self._d, self._w_templ, scr,
                                 *args, local=local, **kwargs)
        elif getattr(tm, "can_fill", False):
            if self._buf is None or tuple(self._buf.shape) != (nch, nb):
                self._buf = torch.empty((nch, nb), dtype=torch.complex128, device=self.device)
            _prefetch(tm, params, args, kwargs)
            for i, params_i in enumerate(params):
                tm.fill(self._buf, *params_i, *args, **kwargs)
                self._red.loglike(self._buf, self._d, self._w_templ, out=out[i:i + 1])
        else:
            for i, params_i in enumerate(params):
                h = self._as_channels(tm(*params_i, *args, **kwargs))
                self._red.loglike(h, self._d, self._w, out=out[i:i + 1])
        if self.noise_has_been_added:
            raise NotImplementedError
        if self.use_gpu and self.return_cupy:
            return out
        return out.cpu().numpy()

    # the windowed logL in its per-bin form, reduced inside the transforms' last pass
    # (efd_hann_loglike_local; False: efd_hann_loglike's mirror-pair form after the transforms)
    HANN_LOCAL = True

    def _hann_local(self, tm, kwargs):
        """The template model's per-bin windowed-logL data for this likelihood's d, w (made once
        per injection), or None."""
        hloc = getattr(self, "_hloc", None)
        if hloc is None:
            make = getattr(tm, "hann_local", None) if self.HANN_LOCAL else None
            inj = getattr(self, "_inj_call", None)
            if make is None:
                hloc = False
            elif inj is not None:
                hloc = make(self._d, self._w_templ, inj=inj[0], **inj[1]) or False
            else:
                hloc = make(self._d, self._w_templ, **kwargs) or False
            self._hloc = hloc
        return hloc or None

    # walkers per fused group (EFD_FUSED_GROUP overrides it: an experiment switch): one
    # efd_modesum_prepare_batch and one efd_modesum_sum_loglike each; FUSED_DEPTH groups rotate so group i+1's preparation runs beside group i's sum.
    # Balanced groups of at most 16 (EFD_BATCH_MAX): config 5's 64-walker half-steps (host-bound,
    # 43-tile grids) ran 54-60 k logL/s in 4 groups against 40-51 k in 8 (5 interleaved rounds);
    # config 4's 8 walkers are one group either way (groups of 4 or 3: -5 to -10%)
    FUSED_GROUP = min(max(1, int(os.environ.get("EFD_FUSED_GROUP", "16"))), 64)
    FUSED_DEPTH = max(1, int(os.environ.get("EFD_FUSED_DEPTH", "2")))
    # each group's sum on the group's own stream, right behind its preparation: no
    # cross-stream wait between the two (~12 us of idle device per group on config 4's chain,
    # tools/chain_timeline.py), and the groups' sums need no common stream (each writes its own
    # slice of out); the streams join once, before the copy out. False: round 3's sum stream.
    FUSED_SUM_OWN_STREAM = os.environ.get("EFD_SUM_STREAM", "0") != "1"
    # a group's staging, upload, preparation and fused sum in one native call
    # (BatchPreparer.flush_loglike, efd_fused_group); False: the Python steps of round 5
    FUSED_NATIVE_GROUP = True

    def _get_ll_fused(self, tm, params, args, kwargs, out):
        """The pipelined path with the likelihood fused into the mode sum: per group of
        FUSED_GROUP walkers, the template chain collects each walker's host inputs
        (BatchPreparer), one upload and one efd_modesum_prepare_batch prepare the group on its
        stream, and one efd_modesum_sum_loglike on a sum stream writes the group's
        log-likelihoods into out (the templates never reach HBM). A group's workspaces are reused
        only after the sum that read them (an event per group). Returns the log-likelihoods on
        the host (copied out in the sum stream's order: one synchronisation per batch), or None,
        before queueing anything, when the template's grid is not symmetric (the caller takes the
        per-walker path). A walker whose preparation or sum raised a device-side error comes
        back NaN from the kernel (efd_modesum_sum_loglike), and only then are the groups'
        status flags read, which raises."""
        torch = self.torch
        from .summation import BatchPreparer
        if not self._fused_grid_ok(tm, kwargs):
            return None
        _prefetch(tm, params, args, kwargs)
        n = len(params)
        if n == 0:
            return np.empty(0, dtype=np.float64)
        ngroups = -(-n // self.FUSED_GROUP)
        G = -(-n // ngroups)                       # balanced groups of at most FUSED_GROUP
        caustic = getattr(getattr(getattr(tm.waveform_generator, "waveform_generator", None),
                                  "create_waveform", None), "caustic", "uniform")
        F = self._fused
        if F is None or F["prep"].caustic != caustic or F["prep"].group < G:
            F = self._fused = dict(prep=BatchPreparer(max(G, self.FUSED_GROUP), self.FUSED_DEPTH,
                                                      caustic=caustic, device=self.device),
                                   stream=torch.cuda.Stream(self.device))
        B, s_sum = F["prep"], F["stream"]
        if "order" not in F:
            # the stream handles the orderings below take (efd_stream_order: one event record
            # and one stream wait each, in C), and one reused release event per group
            vp = ctypes.c_void_p
            F["order"] = (vp * (len(B.groups) + 1))(*[g["stream"].cuda_stream for g in B.groups],
                                                     s_sum.cuda_stream)
            F["gst"] = [g["stream"].cuda_stream for g in B.groups]
            F["sum1"] = (vp * 1)(s_sum.cuda_stream)
            F["ev"] = [torch.cuda.Event() for _ in B.groups]
        lib = B.lib
        cur = torch.cuda.current_stream(self.device)
        curh = cur.cuda_stream
        # the streams this batch uses after the work queued so far on the current one: with the
        # sums on the groups' own streams, only the groups' streams the batch's flushes take
        # (B's rotation from its next group; one stream wait each)
        if self.FUSED_SUM_OWN_STREAM:
            key = ("ord", B._next, min(ngroups, len(B.groups)))
            arr = F.get(key)
            if arr is None:
                gis = [(key[1] + k) % len(B.groups) for k in range(key[2])]
                arr = F[key] = (ctypes.c_void_p * len(gis))(*[F["gst"][g] for g in gis])
            _lib.check(lib.efd_stream_order(curh, arr, len(arr)), "efd_stream_order", lib)
        else:
            _lib.check(lib.efd_stream_order(curh, F["order"], len(F["order"])),
                       "efd_stream_order", lib)
        pin = F.get("pin")
        if pin is None or pin.numel() < n:
            pin = F["pin"] = torch.empty(max(n, 64), dtype=torch.float64, pin_memory=True)
        own = self.FUSED_SUM_OWN_STREAM
        native = self.FUSED_NATIVE_GROUP and hasattr(lib, "efd_fused_group")
        used = []
        try:
            batch = getattr(tm, "submit_batch", None)
            for g0 in range(0, n, G):
                if batch is not None:
                    batch(B, params[g0:g0 + G], *args, **kwargs)
                else:
                    for i in range(g0, min(n, g0 + G)):
                        tm.submit(B, None, *params[i], *args, order=False, prepare_only=True,
                                  **kwargs)
                if own and native:
                    # the group's staging, upload, preparation and fused sum in one native call
                    # on the group's stream (efd_fused_group), the tile constants made on it
                    # first (once per grid)
                    p0 = B._pending[0]
                    sst = B.groups[B._next]["stream"]
                    tc = self._tile_constants({"freq": p0[1], "k0": p0[4]}, sst, F)
                    used.append(B.flush_loglike(self._d, self._w_templ, out, tile_const=tc,
                                                out_off=g0))
                    continue
                gi, jobs = B.flush()
                used.append(gi)
                if own:
                    sst = B.groups[gi]["stream"]
                    tc = self._tile_constants(jobs[0][1], sst, F)
                    B.sum_loglike(gi, self._d, self._w_templ, out[g0:g0 + len(jobs)],
                                  sst.cuda_stream, tile_const=tc)
                    continue   # (the group's next flush is behind this sum on its stream)
                _lib.check(lib.efd_stream_order(F["gst"][gi], F["sum1"], 1), "efd_stream_order",
                           lib)
                tc = self._tile_constants(jobs[0][1], s_sum)
                B.sum_loglike(gi, self._d, self._w_templ, out[g0:g0 + len(jobs)],
                              s_sum.cuda_stream, tile_const=tc)
                ev = F["ev"][gi]   # (flush waited on its previous record before this one)
                ev.record(s_sum)
                B.release(gi, ev)
            if own:
                # the other groups' streams join the last one, which copies out
                last = used[-1]
                vp = ctypes.c_void_p
                for gj in sorted(set(used) - {last}):
                    _lib.check(lib.efd_stream_order(F["gst"][gj], (vp * 1)(F["gst"][last]), 1),
                               "efd_stream_order", lib)
                dl = F["gst"][last]
            else:
                dl = s_sum.cuda_stream
            _lib.check(lib.efd_download(pin.data_ptr(), out.data_ptr(), 8 * n, dl),
                       "efd_download", lib)
        finally:
            B._pending = []
            # `out` belongs to the current stream: nothing may still write it when it is
            # returned, or freed after an exception
            if sys.exc_info()[0] is not None:
                # a failure inside B.flush() (staging, workspace growth, preparation) may leave
                # a group's upload or preparation queued before that group reached `used`: wait
                # for every group stream (and the sum stream), not only the recorded ones
                for g in B.groups:
                    g["stream"].synchronize()
                if not own:
                    s_sum.synchronize()
            elif not own:
                s_sum.synchronize()
            elif used:
                B.groups[used[-1]]["stream"].synchronize()
        host = pin[:n].numpy().copy()
        if np.isnan(host).any():
            B.wait()   # device-side errors of the groups' workspaces (sticky across reuse)
        return host

    # tiles no harmonic reaches take a precomputed partial instead of re-reading d and w
    # (efd_loglike_tile_constants; bitwise the same logL)
    fused_tile_constants = True

    def _tile_constants(self, job, stream, fused=None):
        """The fused sum's per-tile constants for (d, w_templ) on this grid, made once on
        `stream` (ordered after the data's creation: the caller's stream waits on current).
        With `fused` (the sums on the groups' own streams) every stream of fused["order"] is
        then ordered after `stream`, so any group's later sum may read them."""
        if not self.fused_tile_constants:
            return None
        from .summation import loglike_tile_constants
        nf, k0 = int(job["freq"].numel()), int(job.get("k0", 0))
        key = (nf, k0, id(self._d), id(self._w_templ))
        tc = self._tile_const
        if tc is None or tc[0] != key:
            tc = self._tile_const = (key, loglike_tile_constants(
                self._d, self._w_templ, nf, k0, stream.cuda_stream))
            if fused is not None:
                lib = fused["prep"].lib
                _lib.check(lib.efd_stream_order(stream.cuda_stream, fused["order"],
                                                len(fused["order"])), "efd_stream_order", lib)
        return tc[1]

    def _fused_grid_ok(self, tm, kwargs):
        """Whether the template's grid for these kwargs is mirror-symmetric (the fused sum's
        requirement); set up once per grid, without queueing any device work."""
        cw = getattr(getattr(getattr(tm, "waveform_generator", None), "waveform_generator", None),
                     "create_waveform", None)
        if cw is None or not hasattr(cw, "_grid"):
            return False
        _, sym = cw._grid(kwargs.get("T", 1.0), kwargs.get("dt", 10.0), kwargs.get("f_arr"))
        return bool(sym)

    def _pipeline_for(self, tm):
        """The WaveformPipeline (self.num_streams slots) and per-slot buffers of get_ll."""
        torch = self.torch
        from .reductions import Reducer
        from .summation import WaveformPipeline
        nch, nb = self._d.shape
        caustic = getattr(getattr(getattr(tm.waveform_generator, "waveform_generator", None),
                                  "create_waveform", None), "caustic", "uniform")
        P = getattr(self, "_pipe", None)
        if P is None or P.caustic != caustic:
            P = self._pipe = WaveformPipeline(self.num_streams, caustic=caustic,
                                              device=self.device)
            self._pbufs = [None] * P.num_slots
            self._preds = [Reducer(self.device) for _ in range(P.num_slots)]
        for j in range(P.num_slots):
            if self._pbufs[j] is None or tuple(self._pbufs[j].shape) != (nch, nb):
                with torch.cuda.stream(P.stream(j)):
                    self._pbufs[j] = torch.empty((nch, nb), dtype=torch.complex128,
                                                 device=self.device)
        return P

    def _as_channels(self, chans):
        torch = self.torch
        if hasattr(chans, "detach") and chans.dim() == 2:
            h = chans
        else:
            h = torch.stack([torch.as_tensor(c, device=self.device) for c in chans])
        h = h.to(device=self.device, dtype=torch.complex128).contiguous()
        if tuple(h.shape) != tuple(self._d.shape):
            raise ValueError(f"template has shape {tuple(h.shape)}, data {tuple(self._d.shape)}")
        return h

    def __call__(self, params, *args, **kwargs):
        if not isinstance(params, np.ndarray):
            raise ValueError("params must be np.ndarray.")
        if self.parameter_transforms is not None:
            key = list(self.parameter_transforms.keys())[0]
            params = self.parameter_transforms[key].both_transforms(params)
        if self.transpose_params:
            params = params.T
            subset_axis = 1
        else:
            subset_axis = 0
        num_likes = params.shape[subset_axis]
        inds_likes = np.arange(num_likes)
        if self.subset is not None:
            if not isinstance(self.subset, int):
                raise ValueError("Subset must be int.")
            inds_subset = np.split(inds_likes, np.arange(self.subset, num_likes, self.subset))
        else:
            inds_subset = [inds_likes]
        out_ll = []
        for inds in inds_subset:
            args_in = (params[inds],) if subset_axis == 0 else (params[:, inds],)
            args_in += args
            if self.fill_data_noise:
                args_in += (self.injection_channels, self.noise_factor)
            out_ll.append(_to_numpy(self.get_ll(*args_in, **kwargs)))
        return np.concatenate(out_ll, axis=0)


def _prefetch(tm, params, args, kwargs, concurrency=None):
    """The batch's host upstream on the pool. Without waiting when the template supports it
    (PREFETCH_ASYNC): each walker's template then waits for its own upstream only, so the first
    groups' device work runs while the pool computes the later walkers' (concurrency: at most
    that many walkers' upstream at once, in order)."""
    if not hasattr(tm, "prefetch"):
        return
    if getattr(tm, "PREFETCH_ASYNC", False) and os.environ.get("EFD_PREFETCH_ASYNC", "1") != "0":
        if concurrency:
            tm.prefetch(params, *args, wait=False, concurrency=concurrency, **kwargs)
        else:
            tm.prefetch(params, *args, wait=False, **kwargs)
    else:
        tm.prefetch(params, *args, **kwargs)


def _to_numpy(x):
    if isinstance(x, (list, tuple)):
        return [_to_numpy(v) for v in x]
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)

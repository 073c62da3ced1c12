"""The reference's FD template helpers (FDutils.py), on the device.

    get_sensitivity(f)                                             FDutils.py:21-33
    get_convolution(a, b)                                          :35-47
    get_fd_windowed(signal, window, window_in_fd=False)            :66-101
    get_fd_waveform_fromFD(waveform_generator, positive_frequency_mask, dt,
                           non_zero_mask=None, window=None, window_in_fd=False)   :105-139
    get_fft_td_windowed(signal, window, dt)                        :49-64
    get_fd_waveform_fromTD(waveform_generator, positive_frequency_mask, dt,
                           non_zero_mask=None, window=None)        :142-178

get_sensitivity interpolates the drivers' PSD table (LISA_Alloc_Sh.txt, shipped here as a data
file) with a not-a-knot cubic spline, as the reference does with scipy's CubicSpline (:4-5); it
is host-side setup work (once per likelihood), and returns numpy for numpy input and a device
tensor for tensor input.

get_convolution is the reference's scipy/cupy `convolve(hstack((a[1:], a)), b, 'valid')/len(b)`.
For len(a) == len(b) = N that is the circular convolution (a (*) b)[k] = sum_j a[(k-j) mod N]
b[j] / N; the general case is the same 'valid' slice of a linear convolution. Both are evaluated
with FFTs on the device (torch.fft -> rocFFT), O(N log N).

get_fd_waveform_fromFD keeps the reference's call: generator -> optional window convolution ->
positive-frequency mask -> optional zeroing outside non_zero_mask. With no window and the mask
being the f >= 0 suffix of a sorted grid (the drivers' case, emri_pe.py:239-241), `fill` writes
h+ and hx straight into the rows of a caller's [2][N] buffer (no intermediate copies); the
Likelihood uses that.

get_fd_waveform_fromTD is the reference's comparison template: the TD generator's [h+, hx]
(efd_td_modesum on the device), times the window, through rocFFT (torch.fft), shifted and scaled
by dt, then masked like the FD template.
"""

import os

import numpy as np

from .summation import require_gpu

_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "LISA_Alloc_Sh.txt")
_SPLINE = None


def _spline():
    global _SPLINE
    if _SPLINE is None:
        from scipy.interpolate import CubicSpline
        tab = np.genfromtxt(_TABLE)
        _SPLINE = CubicSpline(tab[:, 0], tab[:, 1])
    return _SPLINE


def get_sensitivity(f):
    """PSD S(f) [1/Hz] from the LISA_Alloc_Sh table (FDutils.py:21-33)."""
    if hasattr(f, "detach"):
        torch = require_gpu()
        vals = _spline()(f.detach().cpu().numpy())
        return torch.as_tensor(vals, dtype=torch.float64, device=f.device)
    return _spline()(f)


def get_convolution(a, b):
    """convolve(hstack((a[1:], a)), b, mode='valid') / len(b), on the device."""
    torch = require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())
    a = torch.as_tensor(a, device=dev).to(torch.complex128)
    b = torch.as_tensor(b, device=dev).to(torch.complex128)
    na, nb = int(a.numel()), int(b.numel())
    if na == nb:
        return torch.fft.ifft(torch.fft.fft(a) * torch.fft.fft(b)) / nb
    x = torch.cat((a[1:], a))
    nx = int(x.numel())
    if nb > nx:
        raise ValueError("get_convolution: 'valid' needs len(b) <= 2 len(a) - 1")
    n = nx + nb - 1
    full = torch.fft.ifft(torch.fft.fft(x, n) * torch.fft.fft(b, n))
    return full[nb - 1:nx] / nb


def window_multiplier(window, window_in_fd=False):
    """The window convolution of get_fd_windowed as a multiplier in the DFT's other domain.

    get_convolution(conj(fft(w)), b) is the circular convolution (a (*) b) / N with
    a = conj(fft(w)); by the convolution theorem it equals ifft(fft(a) fft(b)) / N, and
    fft(conj(fft(w))) = N conj(w). So the windowed spectrum is ifft(m * fft(b)) with m = conj(w)
    (= w for the reference's real window: exact, no transform of the window); for a window given
    in FD (window_in_fd), m = fft(conj(window)) / N."""
    torch = require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())
    w = torch.as_tensor(window, device=dev)
    if window_in_fd:
        n = int(w.numel())
        return torch.fft.fft(torch.conj(w.to(torch.complex128))) / n
    return torch.conj(w) if torch.is_complex(w) else w.to(torch.float64)


def windowed_spectrum(S, mult):
    """The two-sided spectrum S = h+ - i hx (rows: one waveform each) convolved with the
    window: ifft(mult * fft(S)) along the last axis (rocFFT, batched over rows).

    The reference convolves h+ and hx separately (FDutils.py:95-96). The window kernel
    a = conj(fft(w)) of a real window is Hermitian (a[-m] = conj(a[m])), so the convolution
    commutes with the mirror-conjugation b[k] -> conj(b[N-1-k]) of the odd two-sided grid; h+ and
    hx are linear in S and its mirror-conjugate (h+ = (S + M S) / 2, hx = i (S - M S) / 2), so
    the windowed h+ and hx are those of the windowed S: one transform pair per waveform instead
    of one per channel."""
    torch = require_gpu()
    return torch.fft.ifft(torch.fft.fft(S.to(torch.complex128), dim=-1) * mult, dim=-1)


def get_fd_windowed(signal, window, window_in_fd=False):
    """[h+, hx] convolved with the window's spectrum (FDutils.py:66-101)."""
    if window is None:
        return [signal[0], signal[1]]
    torch = require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())
    w = torch.as_tensor(window, device=dev)
    fw = w.to(torch.complex128) if window_in_fd else torch.fft.fft(w.to(torch.complex128))
    return [get_convolution(torch.conj(fw), signal[0]),
            get_convolution(torch.conj(fw), signal[1])]


class get_fd_waveform_fromFD:
    """FD template [ch1, ch2] over the positive frequencies (FDutils.py:105-139)."""

    def __init__(self, waveform_generator, positive_frequency_mask, dt, non_zero_mask=None,
                 window=None, window_in_fd=False):
        torch = require_gpu()
        dev = torch.device("cuda", torch.cuda.current_device())
        self.waveform_generator = waveform_generator
        self.positive_frequency_mask = torch.as_tensor(positive_frequency_mask, device=dev)
        self.non_zero_mask = (None if non_zero_mask is None
                              else torch.as_tensor(non_zero_mask, device=dev))
        self.window = window
        self.window_in_fd = window_in_fd
        self.dt = dt
        self._mult = None if window is None else window_multiplier(window, window_in_fd)
        # contiguous-suffix mask (f >= 0 of a sorted grid): the fused fill path applies
        pm = self.positive_frequency_mask
        k0 = int(torch.argmax(pm.to(torch.int8)).item()) if bool(pm.any()) else int(pm.numel())
        self._suffix_k0 = k0 if bool(pm[k0:].all()) and not bool(pm[:k0].any()) else None
        self.num_bins = int(pm.sum().item())

    def _windowed_s_path(self):
        """Windowed templates through the two-sided spectrum (windowed_spectrum): a generator
        with the spectrum entry (GenerateEMRIWaveform) on a symmetric grid whose f >= 0 part is
        the positive mask's suffix."""
        gen = self.waveform_generator
        return (self.window is not None and self._suffix_k0 is not None
                and hasattr(gen, "_spectrum") and hasattr(gen, "waveform_generator")
                and getattr(gen.waveform_generator, "output_type", None) == "fd"
                and self._mult is not None
                and int(self._mult.numel()) == int(self.positive_frequency_mask.numel()))

    def __call__(self, *args, **kwargs):
        torch = require_gpu()
        if self._windowed_s_path():
            out = torch.empty((2, self.num_bins), dtype=torch.complex128,
                              device=self.positive_frequency_mask.device)
            self.fill(out, *args, **kwargs)
            if self.non_zero_mask is not None:
                out[:, ~self.non_zero_mask] = 0.0
            return [out[0], out[1]]
        chans = self.waveform_generator(*args, **kwargs)
        p, c = get_fd_windowed(chans, self.window, window_in_fd=self.window_in_fd)
        p = torch.as_tensor(p)
        c = torch.as_tensor(c)
        ch1 = p[self.positive_frequency_mask]
        ch2 = c[self.positive_frequency_mask]
        if self.non_zero_mask is not None:
            ch1[~self.non_zero_mask] = 0.0
            ch2[~self.non_zero_mask] = 0.0
        return [ch1, ch2]

    @property
    def can_fill(self):
        gen = self.waveform_generator
        if self.window is not None:
            return self._windowed_s_path()
        return self._suffix_k0 is not None and hasattr(gen, "fill_channels")

    @property
    def can_pipeline(self):
        return (self.window is None and self.can_fill
                and hasattr(self.waveform_generator, "submit_channels"))

    def submit(self, pipeline, out, *args, **kwargs):
        """fill, queued on a WaveformPipeline slot (returns the slot; see
        GenerateEMRIWaveform.submit_channels)."""
        return self.waveform_generator.submit_channels(pipeline, out, *args, k0=self._suffix_k0,
                                                       **kwargs)

    def submit_batch(self, preparer, params, *args, **kwargs):
        """Every row of params (walkers x 14) into a BatchPreparer (the fused likelihood's walker
        group): the generator's submit_batch when it has one, else per-walker submits."""
        fn = getattr(self.waveform_generator, "submit_batch", None)
        if fn is not None and not args:
            return fn(preparer, params, k0=self._suffix_k0, **kwargs)
        for prm in params:
            self.submit(preparer, None, *prm, *args, order=False, prepare_only=True, **kwargs)

    def prefetch(self, params, *args, **kwargs):
        """The host upstream of a walker batch in parallel (GenerateEMRIWaveform.prefetch),
        ahead of the per-walker submit/fill calls; a no-op for other generators."""
        fn = getattr(self.waveform_generator, "prefetch", None)
        return fn(params, **kwargs) if fn is not None and not args else 0

    def fill(self, out, *args, **kwargs):
        """Write [ch1, ch2] into out (complex128 [2][num_bins], device) without copies.

        Bins outside non_zero_mask are NOT zeroed here; the Likelihood folds that mask into
        the template's noise weight instead (same result: h * 0).
        """
        if self.window is None:
            self.waveform_generator.fill_channels(out, *args, k0=self._suffix_k0, **kwargs)
            return out
        if not self._windowed_s_path():
            raise ValueError("fill: a windowed template needs the spectrum path")
        gen = self.waveform_generator
        S = gen._spectrum(*args, **kwargs)
        cw = gen.waveform_generator.create_waveform
        if self._suffix_k0 != cw.positive_start():
            raise ValueError("positive_frequency_mask does not match the generator's grid")
        cw.polarizations(windowed_spectrum(S, self._mult), True, out=(out[0], out[1]))
        return out


def get_fft_td_windowed(signal, window, dt):
    """[fftshift(fft(h+ w)) dt, fftshift(fft(hx w)) dt] on the device (FDutils.py:49-64)."""
    torch = require_gpu()
    out = []
    for x in (signal[0], signal[1]):
        x = torch.as_tensor(x, device=torch.device("cuda", torch.cuda.current_device()))
        if window is not None:
            x = x * torch.as_tensor(window, device=x.device)
        out.append(torch.fft.fftshift(torch.fft.fft(x.to(torch.complex128))) * dt)
    return out


class get_fd_waveform_fromTD:
    """DFT of the TD template [ch1, ch2] over the positive frequencies (FDutils.py:142-178)."""

    def __init__(self, waveform_generator, positive_frequency_mask, dt, non_zero_mask=None,
                 window=None):
        torch = require_gpu()
        dev = torch.device("cuda", torch.cuda.current_device())
        self.waveform_generator = waveform_generator
        self.positive_frequency_mask = torch.as_tensor(positive_frequency_mask, device=dev)
        self.dt = dt
        self.non_zero_mask = (None if non_zero_mask is None
                              else torch.as_tensor(non_zero_mask, device=dev))
        # the reference's default window is ones_like(mask) (:165-166): the identity
        self.window = None if window is None else torch.as_tensor(window, device=dev)

    def __call__(self, *args, **kwargs):
        chans = self.waveform_generator(*args, **kwargs)
        p, c = get_fft_td_windowed(chans, self.window, self.dt)
        ch1 = p[self.positive_frequency_mask]
        ch2 = c[self.positive_frequency_mask]
        if self.non_zero_mask is not None:
            ch1[~self.non_zero_mask] = 0.0
            ch2[~self.non_zero_mask] = 0.0
        return [ch1, ch2]

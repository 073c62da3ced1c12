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
import weakref

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


class HannConvolution:
    """The reference's window convolution for its own window, scipy.signal.windows.hann(N)
    (emri_pe.py:261, sym=True: w[n] = 1/2 - 1/2 cos(2 pi n / (N - 1))), without size-N DFTs.

    windowed_spectrum's S_w = ifft(w fft(S)) splits, with theta = 2 pi / (N - 1) = (2 pi / N)
    (1 + e), e = 1 / (N - 1), into 1/2 S minus 1/4 of the trigonometric interpolant
    S~(k) = sum_j S[j] G(k - j), G(u) = (1/N) sum_n exp(2 pi i n u / N), at k +- (1 + e):
      S_w[k] = 1/2 S[k] - 1/4 (S[k+1] + S[k-1]) - 1/4 e (C[k+1] - C[k-1]) + O(e^2),
      C = K (*) S (circular),  K[m] = G'(m) = -i pi / N + (pi / N) cot(pi m / N),
                               K[0] = i pi (N - 1) / N,
    indices mod N. The dropped second-order term is below 1e-13 max|S| at N = 12.6 M (numpy
    check: the first-order form is within 3e-12 of the exact DFT form at N = 1e6, falling as
    1/N^2). The correction term is itself ~1e-6 of max|S|, so C needs ~3 significant digits: it
    is computed in complex64 (rows scaled by their max component) as a linear convolution of
    each row's SUPPORT [first, last) (its nonzero bins: the harmonics reach |f| <= F_max only)
    with the lag kernel, on m-point transforms, m the smallest 2^a or 3 2^a >= N + (last -
    first) - 1 (include/emrifd.h, efd_hann_extent). test.sh's 12.6 M-bin grid with its
    harmonics below ~15% of Nyquist takes m = 2^24, where the full-support form needs 2^25 and
    the size-N DFT form two Bluestein transforms of 2^25 each. The transforms are in place
    (power-of-two m from 2^21 to 2^25: efd_hann_convolve, one four-step FFT pipeline of three
    passes over the rows with the staging and the kernel multiply folded in; other lengths:
    hipFFT plans per (m, rows), _hipfft); efd_hann_loglike then reduces the windowed
    templates' logL without writing them."""

    KEEP_KERNELS = 3   # lag-kernel spectra kept (per m: plain and the logL's differenced one)
    KEEP_PLANS = 2     # hipFFT plans kept (one per (m, rows); the lengths outside the four-step's)
    # The first-order form drops an O(e^2) term, ~3.5-5 / N^2 of max|S| (the test's 5 / N^2 bound:
    # 5e-10 at N = 1e5, 5e-6 at N = 1e3). The likelihood takes this path only where that is below
    # TOL (N >= 2,236,068: every 1-yr or longer grid at dt = 10 s); shorter grids keep the exact
    # size-N DFT form (windowed_spectrum), as the reference's convolution is exact at every N.
    TOL = 1e-12

    @classmethod
    def applies(cls, n):
        """Whether the first-order form is within TOL of max|S| at grid length n."""
        return int(n) >= 3 and 5.0 / float(n) ** 2 <= cls.TOL

    def __init__(self, n, device):
        require_gpu()
        self.n = n = int(n)
        if n < 3:
            raise ValueError("HannConvolution: n >= 3")
        self.eps = 1.0 / (n - 1)
        self.device = device
        self._kf = {}
        self._plans = {}
        self._ybuf = None
        self._info = None

    @staticmethod
    def matches(window):
        """Whether window is scipy.signal.windows.hann(len(window)) (the reference's)."""
        from scipy.signal.windows import hann
        w = np.asarray(window.cpu().numpy() if hasattr(window, "detach") else window)
        return w.ndim == 1 and len(w) >= 3 and np.array_equal(w, hann(len(w)))

    @classmethod
    def size_for(cls, n, support, four_step=True):
        """The transform length for a support of `support` bins: >= n + support - 1, the power
        of two when efd_hann_convolve takes it (three passes over the rows beat hipFFT's ~11 on
        a length up to 4/3 shorter), else the smallest 2^a or 3 2^a."""
        # (one bin more than the linear convolution needs: the fused logL's differenced
        # correction reads Y one place below the window, efd_hann_loglike_local)
        need = int(n) + max(int(support), 1)
        best = None
        for base in (1, 3):
            m = base
            while m < need:
                m *= 2
            if base == 1 and four_step and cls.FOUR_STEP_MIN <= m <= cls.FOUR_STEP_MAX:
                return m
            best = m if best is None else min(best, m)
        return best

    # efd_hann_convolve (one four-step FFT pipeline, 3 passes over the rows) takes power-of-two
    # m in [FOUR_STEP_MIN, FOUR_STEP_MAX]; other lengths go through hipFFT
    FOUR_STEP_MIN, FOUR_STEP_MAX, FOUR_STEP_C = 1 << 21, 1 << 25, 8192
    four_step = True

    def _four(self, m):
        return (self.four_step and m & (m - 1) == 0
                and self.FOUR_STEP_MIN <= m <= self.FOUR_STEP_MAX)

    def kernel_spectrum(self, m, four=False, diff=False):
        """fft(z) / m in complex64, z[t] = K[(t - (m - n)) mod n] (computed in complex128); with
        four=True in efd_hann_convolve's order: [f_r][f_c] = kf[f_r + R f_c], R = m / C with the
        library's C for m (efd_hann_four_step_cols: 8192, or 16384 at m = 2^24). diff=True: times
        2i sin(2 pi f / m), so the transforms give Y[s+1] - Y[s-1] (efd_hann_loglike_local)."""
        kf = self._kf.get((m, four, diff))
        if kf is None:
            torch = require_gpu()
            n = self.n
            t = torch.arange(m, device=self.device, dtype=torch.int64)
            mm = torch.remainder(t - (m - n), n).to(torch.float64)
            zero = mm == 0
            re = torch.where(zero, torch.zeros_like(mm), (np.pi / n) / torch.tan(np.pi * mm / n))
            im = torch.where(zero, torch.full_like(mm, np.pi * (n - 1) / n),
                             torch.full_like(mm, -np.pi / n))
            kf = torch.fft.fft(torch.complex(re, im)) / m
            if diff:
                f = torch.arange(m, device=self.device, dtype=torch.float64)
                kf = kf * torch.complex(torch.zeros_like(f), 2.0 * torch.sin((2.0 * np.pi / m) * f))
            kf = kf.to(torch.complex64)
            if four:
                from . import _lib
                C = int(_lib.load().efd_hann_four_step_cols(m))
                kf = kf.view(C, m // C).t().contiguous()
            while len(self._kf) >= self.KEEP_KERNELS:
                self._kf.pop(next(iter(self._kf)))
            self._kf[(m, four, diff)] = kf
        return kf

    def _rows(self, S):
        torch = require_gpu()
        if S.dim() == 1:
            S = S[None]
        if (S.dtype != torch.complex128 or S.shape[-1] != self.n or not S.is_contiguous()
                or S.device != torch.device(self.device)):
            raise ValueError(f"HannConvolution: contiguous complex128 rows of {self.n} bins on "
                             f"{self.device}")
        return S

    def transform(self, S, lib, lanes=None, support=None):
        """(Y, info, m) for the rows of S ([rows][n], complex128, contiguous): Y complex64
        [rows][m] holds each row's C / scale at ((k - first) mod n) + m - n (efd_hann_stage's
        layout after the transform pair); info int64 [rows][4] (efd_hann_extent). One host
        synchronisation: the rows' supports choose m. lanes: the rows' lane ranges
        (GenerateEMRIWaveform.spectrum_batch), so the extent reads only their bins. support:
        an upper bound of every row's support known on the host (lane_support), which chooses
        m instead: no synchronisation."""
        from . import _hipfft, _lib
        torch = require_gpu()
        S = self._rows(S)
        rows, n = int(S.shape[0]), self.n
        st = torch.cuda.current_stream(S.device).cuda_stream
        sp = torch.view_as_real(S).data_ptr()
        m, info, Y = self._forward_setup(S, lib, lanes, support)
        yp = torch.view_as_real(Y).data_ptr()
        if self._four(m):
            kfp = self.kernel_spectrum(m, four=True)
            _lib.check(lib.efd_hann_convolve(sp, n, n, rows, info.data_ptr(), m,
                                             torch.view_as_real(kfp).data_ptr(), yp, st),
                       "efd_hann_convolve", lib)
            return Y, info, m
        _lib.check(lib.efd_hann_stage(sp, n, n, rows, info.data_ptr(), m, yp, st),
                   "efd_hann_stage", lib)
        plan = self._plans.get((m, rows))
        if plan is None:
            # bounded like the lag kernels: m follows each batch's support and rows the last,
            # partial group, so unbounded plans (each with its work buffer) would pile up
            while len(self._plans) >= self.KEEP_PLANS:
                self._plans.pop(next(iter(self._plans))).destroy()
            plan = self._plans[(m, rows)] = _hipfft.C2CPlan(m, rows)
        plan(yp, _hipfft.FORWARD, st)
        Y.mul_(self.kernel_spectrum(m))
        plan(yp, _hipfft.BACKWARD, st)
        return Y, info, m

    def correction(self, S, lib=None):
        """C = K (*) S (complex128, rows of S along the last axis)."""
        from . import _lib
        torch = require_gpu()
        one = S.dim() == 1
        Y, info, m = self.transform(S, lib or _lib.load())
        n = self.n
        first = info[:, 1].clamp_min(0)
        scale = info[:, 0].contiguous().view(torch.float64)
        k = torch.arange(n, device=Y.device, dtype=torch.int64)
        q = torch.remainder(k[None, :] - first[:, None], n) + (m - n)
        C = torch.gather(Y, 1, q).to(torch.complex128) * scale[:, None]
        return C[0] if one else C

    def polarizations_batch(self, S, outs, k0, lib, lanes=None, support=None):
        """polarizations for every row of S ([B][n], contiguous): one transform pair over the
        rows and one efd_hann_polarizations per row into outs[i] = (hp, hc)."""
        from . import _lib
        torch = require_gpu()
        S = self._rows(S)
        Y, info, m = self.transform(S, lib, lanes, support)
        st = torch.cuda.current_stream(S.device).cuda_stream
        for i, (hp, hc) in enumerate(outs):
            _lib.check(lib.efd_hann_polarizations(
                torch.view_as_real(S[i]).data_ptr(), torch.view_as_real(Y[i]).data_ptr(),
                info[i].data_ptr(), m, self.n, k0, torch.view_as_real(hp).data_ptr(),
                torch.view_as_real(hc).data_ptr(), st), "efd_hann_polarizations", lib)
        return outs

    def polarizations(self, S, hp, hc, k0, lib):
        """h+/hx over bins [k0, n) of the windowed S (one row) into hp, hc."""
        self.polarizations_batch(self._rows(S), [(hp, hc)], k0, lib)
        return hp, hc

    @staticmethod
    def lane_support(lanes_host, n):
        """The largest support any row can have given its lane range (int32 [rows][2] on the
        host): efd_hann_extent scans [min(lo, n - hi), max(hi, n - lo)) of a row with lanes
        [lo, hi), and the row's nonzero bins lie inside it, so its support (last + 1 - first)
        is at most that span; a transform length chosen for the span is long enough."""
        lo = lanes_host[:, 0].astype(np.int64)
        hi = lanes_host[:, 1].astype(np.int64)
        live = hi > lo
        if not live.any():
            return 1
        k_lo = np.maximum(0, np.minimum(lo, n - hi))
        k_hi = np.minimum(n, np.maximum(hi, n - lo))
        return int((k_hi - k_lo)[live].max())

    def loglike_batch(self, S, d, w, k0, out, scratch, lib, lanes=None, support=None):
        """efd_hann_loglike: the logL of every row's windowed template against d, w
        (efd_loglike's [2][n - k0] layout) into out (float64 device [rows]); scratch holds
        rows * EFD_LOGLIKE_SCRATCH doubles."""
        from . import _lib
        torch = require_gpu()
        S = self._rows(S)
        rows = int(S.shape[0])
        Y, info, m = self.transform(S, lib, lanes, support)
        st = torch.cuda.current_stream(S.device).cuda_stream
        _lib.check(lib.efd_hann_loglike(
            torch.view_as_real(S).data_ptr(), self.n, torch.view_as_real(Y).data_ptr(),
            info.data_ptr(), m, rows, self.n, k0, torch.view_as_real(d).data_ptr(),
            w.data_ptr(), out.data_ptr(), scratch.data_ptr(), st), "efd_hann_loglike", lib)
        return out

    # local logL data (efd_hann_loglike_local) --------------------------------------------
    def local_ok(self, d, w, k0):
        """Whether the windowed logL against d, w ([2][n - k0]) can take the per-bin form of
        efd_hann_loglike_local: the same weight on both channels at every bin and every mirror
        n-1-k of a kept bin k >= k0 outside the kept bins (or k itself)."""
        torch = require_gpu()
        n = self.n
        return (2 * int(k0) >= n - 1 and tuple(d.shape) == (2, n - k0)
                and tuple(w.shape) == (2, n - k0) and bool(torch.equal(w[0], w[1])))

    def local_data(self, d, w, k0):
        """(dl, wl, kself) of efd_hann_loglike_local from d, w ([2][n - k0], efd_loglike's
        layout): dl complex128 [n + 1] with d0 - i d1 at each kept bin k, conj(d0 + i d1) at its
        mirror n-1-k (at dl[n] when the mirror is k itself, kself = k), wl float64 [n] the
        weight at both; bins neither kept nor mirrored hold 0 (no term)."""
        require_gpu()
        return self.local_layout(self.n, d, w, k0)

    @staticmethod
    def local_layout(n, d, w, k0):
        """local_data's arithmetic for a grid of n bins, on d's device (any torch device: the
        CPU tests pin the layout and the recombination identity with it)."""
        import torch
        n, k0 = int(n), int(k0)
        dev = d.device
        dl = torch.zeros(n + 1, dtype=torch.complex128, device=dev)
        wl = torch.zeros(n, dtype=torch.float64, device=dev)
        k = torch.arange(k0, n, device=dev)
        j = (n - 1) - k
        d0, d1 = d[0], d[1]
        a = torch.complex(d0.real + d1.imag, d0.imag - d1.real)       # d0 - i d1
        b = torch.complex(d0.real - d1.imag, -(d0.imag + d1.real))    # conj(d0 + i d1)
        kself = n - 1 - k0 if 2 * k0 == n - 1 else -1
        dl[j] = b
        wl[j] = w[0]
        if kself >= 0:
            dl[n] = b[0]
        dl[k] = a
        wl[k] = w[0]
        return dl, wl, kself

    def local_emit(self, S, wl, kself, lib, lanes=None, support=None):
        """dl = wl S_w over the grid (and dl[n] = dl[kself]) for one row S: the local data of an
        injection made with this arithmetic (efd_hann_loglike_local's emit), whose logL against
        a template of the same spectrum and transform length is exactly 0."""
        from . import _lib
        torch = require_gpu()
        S = self._rows(S)
        if S.shape[0] != 1:
            raise ValueError("local_emit: one row")
        m, info, Y = self._forward_setup(S, lib, lanes, support)
        if not self._four(m):
            return None
        dl = torch.zeros(self.n + 1, dtype=torch.complex128, device=S.device)
        st = torch.cuda.current_stream(S.device).cuda_stream
        _lib.check(lib.efd_hann_loglike_local(
            torch.view_as_real(S).data_ptr(), self.n, self.n, 1, info.data_ptr(), m,
            torch.view_as_real(self.kernel_spectrum(m, four=True, diff=True)).data_ptr(),
            torch.view_as_real(Y).data_ptr(), None, wl.data_ptr(), int(kself), None, None,
            torch.view_as_real(dl).data_ptr(), st), "efd_hann_loglike_local", lib)
        return dl

    def _forward_setup(self, S, lib, lanes, support):
        """efd_hann_extent, the transform length m and the Y buffer for the rows of S."""
        from . import _lib
        torch = require_gpu()
        rows, n = int(S.shape[0]), self.n
        st = torch.cuda.current_stream(S.device).cuda_stream
        if self._info is None or self._info.shape[0] < rows:
            self._info = torch.empty((rows, 4), dtype=torch.int64, device=S.device)
        info = self._info[:rows]
        lp = None
        if lanes is not None:
            if tuple(lanes.shape) != (rows, 2) or lanes.dtype != torch.int32:
                raise ValueError("lanes: int32 [rows][2]")
            lp = lanes.data_ptr()
        _lib.check(lib.efd_hann_extent(torch.view_as_real(S).data_ptr(), n, n, rows, lp,
                                       info.data_ptr(), st), "efd_hann_extent", lib)
        if support is None:
            ext = info[:, 1:3].cpu().numpy()          # first (-1: empty row), last + 1
            live = ext[:, 1] > 0
            support = int((ext[live, 1] - ext[live, 0]).max()) if live.any() else 1
        m = self.size_for(n, max(int(support), 1), self.four_step)
        need = rows * m
        if self._ybuf is None or self._ybuf.numel() < need:
            self._ybuf = None
            self._ybuf = torch.empty(need, dtype=torch.complex64, device=S.device)
        return m, info, self._ybuf[:need].view(rows, m)

    def loglike_local(self, S, local, out, scratch, lib, lanes=None, support=None):
        """efd_hann_loglike_local: every row's windowed logL against local = (dl, wl, kself)
        into out (float64 device [rows]), the correction reduced inside the inverse column pass
        (no correction array written or read back); scratch holds rows *
        EFD_HANN_LOCAL_PARTIALS doubles. Returns False (nothing done) when the transform length
        is not the four-step's: the caller takes loglike_batch."""
        from . import _lib
        torch = require_gpu()
        S = self._rows(S)
        rows = int(S.shape[0])
        m, info, Y = self._forward_setup(S, lib, lanes, support)
        if not self._four(m):
            return False
        dl, wl, kself = local
        st = torch.cuda.current_stream(S.device).cuda_stream
        _lib.check(lib.efd_hann_loglike_local(
            torch.view_as_real(S).data_ptr(), self.n, self.n, rows, info.data_ptr(), m,
            torch.view_as_real(self.kernel_spectrum(m, four=True, diff=True)).data_ptr(),
            torch.view_as_real(Y).data_ptr(), torch.view_as_real(dl).data_ptr(), wl.data_ptr(),
            int(kself), out.data_ptr(), scratch.data_ptr(), None, st),
            "efd_hann_loglike_local", lib)
        return True

    def __call__(self, S):
        torch = require_gpu()
        C = self.correction(S)
        Sp, Sm = torch.roll(S, -1, dims=-1), torch.roll(S, 1, dims=-1)
        Cd = torch.roll(C, -1, dims=-1) - torch.roll(C, 1, dims=-1)
        return 0.5 * S - 0.25 * (Sp + Sm) - (0.25 * self.eps) * Cd


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
        # the reference's own window (hann(N), emri_pe.py:261) takes HannConvolution
        # when the first-order form is within HannConvolution.TOL at this length (applies(N));
        # shorter grids keep the exact transform pair (windowed_spectrum)
        self._hann = (HannConvolution(len(window), dev)
                      if window is not None and not window_in_fd
                      and HannConvolution.applies(len(window)) and HannConvolution.matches(window)
                      else None)
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
            chans = [out[0], out[1]]
            # what made these channels (made_by): weak references, the template is the caller's
            try:
                self._made = (np.asarray(args, dtype=np.float64).reshape(-1), dict(kwargs),
                              [weakref.ref(c) for c in chans], out._version)
            except (TypeError, ValueError):
                self._made = None
            return chans
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
        ahead of the per-walker submit/fill calls; a no-op for other generators. wait=False
        (PREFETCH_ASYNC generators) returns before the upstream is done."""
        fn = getattr(self.waveform_generator, "prefetch", None)
        return fn(params, **kwargs) if fn is not None and not args else 0

    @property
    def PREFETCH_ASYNC(self):
        return bool(getattr(self.waveform_generator, "PREFETCH_ASYNC", False))

    # walkers per windowed group (fill_batch): their spectra share one batched transform pair
    WINDOW_GROUP = 8

    @property
    def can_fill_batch(self):
        return self._hann is not None and self._windowed_s_path()

    def _spectra(self, params, **kwargs):
        """Every walker's two-sided spectrum in one [B][N] buffer; returns (rows,
        create_waveform, whether the per-walker path ran: its device status is still unread,
        the rows' lane ranges or None)."""
        torch = require_gpu()
        if not self.can_fill_batch:
            raise ValueError("the Hann-window spectrum path only")
        gen = self.waveform_generator
        B = len(params)
        n = int(self.positive_frequency_mask.numel())
        dev = self.positive_frequency_mask.device
        buf = getattr(self, "_sbuf", None)
        if buf is None or buf.shape[0] < B or buf.shape[1] != n:
            self._sbuf = None
            buf = self._sbuf = torch.empty((B, n), dtype=torch.complex128, device=dev)
        single = not (hasattr(gen, "spectrum_batch") and
                      gen.waveform_generator.output_type == "fd")
        lanes = None
        if not single:
            # packed uploads, batched preparation and one sum launch per group of walkers
            # (device-side errors raise in there); each row's lane range for the extent scan
            lb = getattr(self, "_lanes", None)
            if lb is None or lb.shape[0] < B or lb.device != dev:
                lb = self._lanes = torch.empty((max(B, 16), 2), dtype=torch.int32, device=dev)
            lanes = lb[:B]
            lh = getattr(self, "_lanes_host", None)
            if lh is None or lh.shape[0] < B:
                lh = self._lanes_host = torch.empty((max(B, 16), 2), dtype=torch.int32,
                                                    pin_memory=True)
            # the status is read once the caller's window work is queued (_status), and the
            # lane ranges come to the host while the sums run (support): no host
            # synchronisation between the mode sum and the transforms
            gen.spectrum_batch(params, buf[:B], lanes=lanes, check=False, lanes_host=lh[:B],
                               **kwargs)
        else:
            for i, p in enumerate(params):
                gen._spectrum(*p, out=buf[i], check=False, **kwargs)
        cw = gen.waveform_generator.create_waveform
        if self._suffix_k0 != cw.positive_start():
            raise ValueError("positive_frequency_mask does not match the generator's grid")
        return buf[:B], cw, single, lanes

    def _status(self, cw, single):
        if not single:
            self.waveform_generator.check_batch()
        elif not cw.engine.status():
            from . import _lib
            raise _lib.EFDError(f"efd_modesum: {_lib.last_error(cw.engine.lib)}")

    def fill_batch(self, outs, params, **kwargs):
        """fill for a batch of walkers (rows of params, FEW's 14) into outs[i] (complex128
        [2][num_bins] each): the walkers' spectra in one [B][N] buffer, then the Hann window
        for all of them (one transform pair over the rows, HannConvolution.polarizations_batch).
        Same values as B fill calls up to the batched transform's rounding (the correction term
        carries ~1e-6 of max|S|; it enters at <= 1e-12). The engine's device-side status is
        checked once, at the end."""
        if len(params) == 0:
            return outs
        S, cw, single, lanes = self._spectra(params, **kwargs)
        self._hann.polarizations_batch(S, [(o[0], o[1]) for o in outs], self._suffix_k0,
                                       cw.engine.lib, lanes, self._lane_support(S, lanes))
        self._status(cw, single)
        return outs

    def _lane_support(self, S, lanes):
        """The rows' support bound from their lane ranges, on the host as soon as the copies
        _spectra queued are done (the sums may still run), or None without lane ranges."""
        if lanes is None:
            return None
        self.waveform_generator.lanes_ready()
        return self._hann.lane_support(self._lanes_host[:S.shape[0]].numpy(), S.shape[1])

    def loglike_batch(self, out, params, d, w, scratch, local=None, **kwargs):
        """The windowed templates' log-likelihoods of a batch of walkers into out (float64
        device [B]) against d, w (efd_loglike's operands, [2][num_bins]): the spectra as in
        fill_batch, then HannConvolution.loglike_batch (efd_hann_loglike: no template is
        written). The same logL as fill_batch + efd_loglike up to the reduction order.
        local: hann_local's data for d, w: the logL reduced inside the transforms' last pass
        (HannConvolution.loglike_local) where the transform length allows it."""
        if len(params) == 0:
            return out
        S, cw, single, lanes = self._spectra(params, **kwargs)
        support = self._lane_support(S, lanes)
        if local is None or not self._hann.loglike_local(S, local, out, scratch, cw.engine.lib,
                                                         lanes, support):
            self._hann.loglike_batch(S, d, w, self._suffix_k0, out, scratch, cw.engine.lib,
                                     lanes, support)
        self._status(cw, single)
        return out

    def made_by(self, channels):
        """(FEW parameters, waveform kwargs) of this model's call that returned `channels`, if
        they are those very tensors, unmodified since (the drivers inject data = gen(*truth),
        emri_pe.py:276), else None."""
        made = getattr(self, "_made", None)
        if made is None or not isinstance(channels, (list, tuple)) or len(channels) != 2:
            return None
        params, kw, refs, version = made
        if any(r() is not c for r, c in zip(refs, channels)) or channels[0]._version != version:
            return None
        return params, kw

    def hann_local(self, d, w, inj=None, **kwargs):
        """The per-bin logL data of d, w (HannConvolution.local_data: the same weight on both
        channels) for loglike_batch, or None where the windowed logL cannot take that form.
        inj: the injection's FEW parameters when d is this model's template of them times w:
        the data is then emitted by the logL's own arithmetic (HannConvolution.local_emit),
        so the injection's logL against itself is exactly 0 as with efd_hann_loglike."""
        if (self._hann is None or not self._windowed_s_path()
                or not self._hann.local_ok(d, w, self._suffix_k0)):
            return None
        dl, wl, kself = self._hann.local_data(d, w, self._suffix_k0)
        if inj is not None:
            S, cw, single, lanes = self._spectra(np.asarray(inj, dtype=np.float64)[None, :],
                                                 **kwargs)
            e = self._hann.local_emit(S, wl, kself, cw.engine.lib, lanes,
                                      self._lane_support(S, lanes))
            self._status(cw, single)
            if e is not None:
                dl = e
        return dl, wl, kself

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
        if self._hann is not None:
            self._hann.polarizations(S.contiguous(), out[0], out[1], self._suffix_k0,
                                     cw.engine.lib)
            return out
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

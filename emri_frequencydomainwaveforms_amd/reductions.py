"""Device reductions of the likelihood side: thin wrappers of efd_loglike / efd_inner_product.

Both run in libemrifd.so (HIP, gfx950) as fixed-partition two-pass reductions, so results are
bitwise reproducible. They read the channels in place: h, d complex128 [nchan][nbin], w float64
[nchan][nbin] (all contiguous, on one device); the result stays on the device until the caller
asks for it, so a batch of walkers costs one host synchronisation.
"""

import ctypes

from . import _lib
from .summation import require_gpu


class Reducer:
    """Per-device scratch + entry points (one instance per device/stream user)."""

    def __init__(self, device=None):
        self.torch = torch = require_gpu()
        self.lib = _lib.load()
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        self._scr_ll = torch.empty(_lib.EFD_LOGLIKE_SCRATCH, dtype=torch.float64,
                                   device=self.device)
        self._scr_ip = torch.empty(_lib.EFD_INNER_SCRATCH, dtype=torch.float64,
                                   device=self.device)

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, x, name, dtype, shape):
        torch = self.torch
        if x.dtype != dtype or not x.is_contiguous() or x.device != self.device:
            raise ValueError(f"{name}: expected contiguous {dtype} on {self.device}, got "
                             f"{x.dtype} on {x.device}")
        if tuple(x.shape) != tuple(shape):
            raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(x.shape)}")
        return torch.view_as_real(x).data_ptr() if x.is_complex() else x.data_ptr()

    def loglike(self, h, d, w, out=None):
        """-1/2 * 4 * sum |d - h w|^2 over all channels and bins (likelihood.py:257-274).

        h may be None (data-only term). Returns a 1-element float64 device tensor (or writes
        into `out`, a 1-element view, e.g. one slot of a batch result).
        """
        torch = self.torch
        nchan, nbin = int(d.shape[0]), int(d.shape[1])
        pd = self._check(d, "d", torch.complex128, (nchan, nbin))
        pw = self._check(w, "w", torch.float64, (nchan, nbin))
        ph = None if h is None else self._check(h, "h", torch.complex128, (nchan, nbin))
        if out is None:
            out = torch.empty(1, dtype=torch.float64, device=self.device)
        _lib.check(self.lib.efd_loglike(ph, pd, pw, nchan, nbin, out.data_ptr(),
                                        self._scr_ll.data_ptr(), self._stream()),
                   "efd_loglike", self.lib)
        return out

    def inner(self, a, b, w=None):
        """4 * sum conj(a) b w as a complex128 device scalar (diagnostic.py:95-110)."""
        torch = self.torch
        nchan, nbin = int(a.shape[0]), int(a.shape[1])
        pa = self._check(a, "a", torch.complex128, (nchan, nbin))
        pb = self._check(b, "b", torch.complex128, (nchan, nbin))
        pw = None if w is None else self._check(w, "w", torch.float64, (nchan, nbin))
        out = torch.empty(1, dtype=torch.complex128, device=self.device)
        _lib.check(self.lib.efd_inner_product(pa, pb, pw, nchan, nbin,
                                              torch.view_as_real(out).data_ptr(),
                                              self._scr_ip.data_ptr(), self._stream()),
                   "efd_inner_product", self.lib)
        return out

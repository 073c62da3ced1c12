"""lisatools-compatible inner products on the device (LISAanalysistools/lisatools/diagnostic.py).

    inner_product(sig1, sig2, dt=None, df=None, f_arr=None, PSD="lisasens", PSD_args=(),
                  PSD_kwargs={}, normalize=False, use_gpu=False, complex=False)   :14-157
    snr(sig1, *args, data=None, use_gpu=False, **kwargs)                         :160-171

Same arguments, rules and errors as the reference:
  - signals are one channel or a list of channels (equal counts, else ValueError);
  - dt: time-domain signals, rfft * dt with the DC bin dropped (:57-73);
  - df: frequencies (arange(N) + 1) * df (:79-80); f_arr: the given grid (:82-83);
  - PSD: an array (the drivers' usage, emri_pe.py:281-292), or a string naming a sensitivity
    function: "cornish_lisa_psd" (the notebooks' mismatch weighting, sensitivity.py) or
    "LISA_Alloc_Sh" / "lisa_alloc" (the drivers' table, FDutils.py:4-5); other lisatools curves
    raise NotImplementedError;
    PSD=None raises TypeError exactly like the reference (len() of a float at :97);
  - right-sum rule: x = diff(f) with the first spacing repeated (:97-100); out = 4 sum
    Re(conj(a) b) / PSD * x, or the complex sum with complex=True (:103-110);
  - normalize: True -> / sqrt(<a,a><b,b>); "sig1"/"sig2" -> / <s,s> (:112-154).
The reduction runs in libemrifd.so (efd_inner_product); the weights x/PSD are formed once per
call on the device. Inputs may be numpy arrays or torch tensors; the result is a Python float
(complex with complex=True), like the reference's numpy scalar.
"""

import numpy as np

from .summation import require_gpu

_REDUCERS = {}


def _reducer(device):
    from .reductions import Reducer
    key = str(device)
    if key not in _REDUCERS:
        _REDUCERS[key] = Reducer(device)
    return _REDUCERS[key]


def _as_channels(sig, torch, device):
    if not isinstance(sig, list):
        sig = [sig]
    return [torch.as_tensor(s, device=device) for s in sig]


def _psd_array(PSD, freqs, PSD_args, PSD_kwargs, torch, device):
    if isinstance(PSD, str):
        fh = freqs.detach().cpu().numpy() if hasattr(freqs, "detach") else np.asarray(freqs)
        if PSD in ("LISA_Alloc_Sh", "lisa_alloc"):
            from .fdutils import get_sensitivity
            vals = get_sensitivity(fh, *PSD_args, **PSD_kwargs)
        else:   # lisatools' named curves (diagnostic.py:81-82): sensitivity.get_sensitivity
            from .sensitivity import get_sensitivity
            with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
                vals = get_sensitivity(fh, PSD, *PSD_args, **PSD_kwargs)
        return torch.as_tensor(vals, device=device, dtype=torch.float64)
    if PSD is None:
        # the reference evaluates len(1.0) here (diagnostic.py:97) and fails the same way
        raise TypeError("object of type 'float' has no len()")
    if isinstance(PSD, (np.ndarray,)) or hasattr(PSD, "detach"):
        return torch.as_tensor(PSD, device=device, dtype=torch.float64)
    raise ValueError("PSD must be a string giving the sens_fn or a predetermimed array or None "
                     "if noise weighting is included in a signal.")


def inner_product(sig1, sig2, dt=None, df=None, f_arr=None, PSD="lisasens", PSD_args=(),
                  PSD_kwargs={}, normalize=False, use_gpu=False, complex=False):
    torch = require_gpu()
    if df is None and dt is None and f_arr is None:
        raise ValueError("Must provide either df, dt or f_arr keyword arguments.")
    dev = torch.device("cuda", torch.cuda.current_device())
    s1 = _as_channels(sig1, torch, dev)
    s2 = _as_channels(sig2, torch, dev)
    if len(s1) != len(s2):
        raise ValueError("Signal 1 has {} channels. Signal 2 has {} channels. Must be "
                         "equal.".format(len(s1), len(s2)))
    if dt is not None:
        n = max(len(s1[0]), len(s2[0]))
        s1 = [torch.nn.functional.pad(s, (0, n - len(s))) for s in s1]
        s2 = [torch.nn.functional.pad(s, (0, n - len(s))) for s in s2]
        freqs = torch.fft.rfftfreq(n, dt, dtype=torch.float64, device=dev)[1:]
        f1 = [torch.fft.rfft(s.to(torch.float64))[1:] * dt for s in s1]
        f2 = [torch.fft.rfft(s.to(torch.float64))[1:] * dt for s in s2]
    else:
        f1 = [s.to(torch.complex128) for s in s1]
        f2 = [s.to(torch.complex128) for s in s2]
        if df is not None:
            freqs = (torch.arange(len(f1[0]), dtype=torch.float64, device=dev) + 1) * df
        else:
            freqs = torch.as_tensor(f_arr, dtype=torch.float64, device=dev)
    psd = _psd_array(PSD, freqs, PSD_args, PSD_kwargs, torch, dev)
    nbin = len(f1[0])
    x = torch.empty(nbin, dtype=torch.float64, device=dev)
    x[1:] = torch.diff(freqs)
    x[0] = x[1]
    w = (x / psd).expand(len(f1), nbin).contiguous()
    a = torch.stack(f1).contiguous()
    b = torch.stack(f2).contiguous()
    val = _reducer(dev).inner(a, b, w).item()
    out = val if complex else val.real

    norm = 1.0
    kw = dict(dt=dt, df=df, f_arr=f_arr, PSD=PSD, PSD_args=PSD_args, PSD_kwargs=PSD_kwargs)
    if normalize is True:
        n1 = inner_product(sig1, sig1, use_gpu=use_gpu, normalize=False, **kw)
        n2 = inner_product(sig2, sig2, use_gpu=use_gpu, normalize=False, **kw)
        norm = np.sqrt(n1 * n2)
    elif isinstance(normalize, str):
        if normalize == "sig1":
            ref = sig1
        elif normalize == "sig2":
            ref = sig2
        else:
            raise ValueError("If normalizing with respect to sig1 or sig2, normalize kwarg must "
                             "either be 'sig1' or 'sig2'.")
        norm = inner_product(ref, ref, normalize=False, **kw)
    elif normalize is not False:
        raise ValueError("Normalize must be True, False, 'sig1', or 'sig2'.")
    return out / norm


def snr(sig1, *args, data=None, use_gpu=False, **kwargs):
    sig2 = sig1 if data is None else data
    return np.sqrt(inner_product(sig1, sig2, *args, use_gpu=use_gpu, **kwargs))

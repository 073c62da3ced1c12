"""lisatools-compatible analytic LISA sensitivity (LISAanalysistools/lisatools/sensitivity.py).

    cornish_lisa_psd(f, sky_averaged=False, use_gpu=False)                    :1227-1286
    get_sensitivity(f, sens_fn="lisasens", return_type="PSD", *args, **kwargs) :1289-1325

The reference's notebooks weight their FD-vs-TD mismatches with `cornish_lisa_psd`
(Tutorial_FrequencyDomain_Waveforms.ipynb:258, 416, through inner_product(..., PSD=
"cornish_lisa_psd")). The PSD is host setup work (one evaluation per grid), so it is numpy;
with use_gpu=True the result is a device tensor. Of the named curves only "cornish_lisa_psd" is
built; the drivers' own table is fdutils.get_sensitivity (LISA_Alloc_Sh.txt).
"""

import numpy as np

# the other curves lisatools resolves by name (its tdi.py / MLDC sensitivities): not built here
_NOT_BUILT = ("lisasens", "noisepsd_AE", "noisepsd_T", "noisepsd_XYZ", "lisanoises", "SGal",
              "GalConf", "WDconfusionX", "WDconfusionAE", "LISASensitivity")


def cornish_lisa_psd(f, sky_averaged=False, use_gpu=False):
    """Cornish & Robson (arXiv:1803.01944) PSD with the 1-yr galactic foreground, as
    lisatools/sensitivity.py:1227-1286 (same constants, same operation order)."""
    fh = f.detach().cpu().numpy() if hasattr(f, "detach") else np.asarray(f, dtype=np.float64)
    c = 20 / 3 if sky_averaged else 1.0
    L = 2.5 * 10 ** 9                                   # arm length (m)
    f0 = 19.09 * 10 ** (-3)                             # transfer frequency (Hz)
    Poms = ((1.5e-11) * (1.5e-11)) * (1 + np.power((2e-3) / fh, 4))
    Pacc = (3e-15) * (3e-15) * (1 + (4e-4 / fh) * (4e-4 / fh)) * (1 + np.power(fh / (8e-3), 4))
    alpha, beta, k, gamma, f_k = 0.171, 292, 1020, 1680, 0.00215
    Sc = (9e-45 * np.power(fh, -7 / 3) * np.exp(-np.power(fh, alpha) + beta * fh * np.sin(k * fh))
          * (1 + np.tanh(gamma * (f_k - fh))))
    psd = c * ((10 / (3 * L * L)) * (Poms + (4 * Pacc) / (np.power(2 * np.pi * fh, 4)))
               * (1 + 0.6 * (fh / f0) * (fh / f0)) + Sc)
    if use_gpu:
        from .summation import require_gpu
        torch = require_gpu()
        return torch.as_tensor(psd, device=torch.device("cuda", torch.cuda.current_device()))
    return psd


_CURVES = {"cornish_lisa_psd": cornish_lisa_psd}


def get_sensitivity(f, sens_fn="lisasens", return_type="PSD", *args, **kwargs):
    """Named sensitivity curve as PSD, ASD or characteristic strain (sensitivity.py:1289-1325)."""
    if sens_fn in _NOT_BUILT:
        raise NotImplementedError(f"{sens_fn} sensitivity is not built here; use "
                                  "'cornish_lisa_psd' or pass a PSD array")
    try:
        sensitivity = _CURVES[sens_fn]
    except KeyError:
        raise ValueError("{} sensitivity is not available.".format(sens_fn)) from None
    PSD = sensitivity(f, *args, **kwargs)
    if return_type == "PSD":
        return PSD
    elif return_type == "ASD":
        return PSD ** (1 / 2)
    elif return_type == "char_strain":
        fh = f.detach().cpu().numpy() if hasattr(f, "detach") else np.asarray(f)
        if hasattr(PSD, "detach"):
            import torch
            return (torch.as_tensor(fh, device=PSD.device) * PSD) ** (1 / 2)
        return (fh * PSD) ** (1 / 2)
    else:
        raise ValueError("return_type must be PSD, ASD, or char_strain.")

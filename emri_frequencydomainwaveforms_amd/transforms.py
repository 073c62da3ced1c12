"""Sampler-to-waveform parameter mapping used on every likelihood call of the drivers.

emri_pe.py samples a 6-vector (ln M, ln(mu/M), p0, e0, Phi_phi0, Phi_r0) and hands the
likelihood an Eryn `TransformContainer` (Eryn/eryn/utils/transform.py:10-226) built from
  fill_dict = {"ndim_full": 14, "fill_inds": [2, 5, 6, 7, 8, 9, 10, 12], "fill_values": [...]}
  parameter_transforms = {(0, 1): transform_mass_ratio}          emri_pe.py:95-96, 161-206
`both_transforms` first scatters the sampled columns into the 14-column waveform vector (the
fixed ones from fill_values), then applies single-index transforms, then multi-index ones.
This module restates that contract for the host side of Likelihood.__call__ (SURVEY.md section 2
row 13: the semantics must be reproduced by the build's driver); it is plain numpy.
"""

import numpy as np


def transform_mass_ratio(logM, logeta):
    """(ln M, ln q) -> (M, mu = q M)   (emri_pe.py:95-96)."""
    M = np.exp(logM)
    return [M, M * np.exp(logeta)]


class TransformContainer:
    """fill + transform of sampled parameters (Eryn TransformContainer semantics)."""

    def __init__(self, parameter_transforms=None, fill_dict=None):
        self.single, self.multi = {}, {}
        for key, fn in (parameter_transforms or {}).items():
            if isinstance(key, (int, np.integer)):
                self.single[int(key)] = fn
            elif isinstance(key, tuple):
                self.multi[key] = fn
            else:
                raise ValueError(f"parameter transform keys must be int or tuple of int, got {key!r}")
        self.fill_dict = None
        if fill_dict is not None:
            if not isinstance(fill_dict, dict):
                raise ValueError("fill_dict must be a dictionary.")
            for k in ("ndim_full", "fill_inds", "fill_values"):
                if k not in fill_dict:
                    raise ValueError(f"If providing fill_inds, dictionary must have {k} as a key.")
            nfull = fill_dict["ndim_full"]
            if not isinstance(nfull, int):
                raise ValueError("fill_dict['ndim_full'] must be an int.")
            inds = np.asarray(fill_dict["fill_inds"])
            self.fill_dict = dict(fill_dict)
            self.fill_dict["test_inds"] = np.setdiff1d(np.arange(nfull), inds)

    def transform_base_parameters(self, params, copy=True, return_transpose=False):
        cols = (np.array(params, dtype=np.float64) if copy else params).T
        for i, fn in self.single.items():
            cols[i] = fn(cols[i])
        for inds, fn in self.multi.items():
            vals = fn(*[cols[i] for i in inds])
            for i, v in zip(inds, vals):
                cols[i] = v
        return cols if return_transpose else cols.T

    def fill_values(self, params):
        if self.fill_dict is None:
            return params
        params = np.asarray(params, dtype=np.float64)
        out = np.zeros(params.shape[:-1] + (self.fill_dict["ndim_full"],))
        out[..., self.fill_dict["test_inds"]] = params
        out[..., np.asarray(self.fill_dict["fill_inds"])] = np.asarray(self.fill_dict["fill_values"])
        return out

    def both_transforms(self, params, copy=True, return_transpose=False, reverse=False):
        if reverse:
            return self.fill_values(self.transform_base_parameters(params, copy=copy))
        return self.transform_base_parameters(self.fill_values(params), copy=copy,
                                              return_transpose=return_transpose)

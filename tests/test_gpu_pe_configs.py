"""GPU parity at BASELINE.json configs 4 and 5: the emri_pe.py likelihood, full size.

config 4  emri_pe.py -Tobs 2 -eps 1e-2 -injectFD 1 -template fd -nwalkers 16 -ntemps 1 on the
          full 6,311,631-bin grid (emri_pe.py:399-417): 16 walkers from the reference's own
          start, multivariate_normal(truth, cov(covariance.npy) / (2.4 * 6)) (:440-444),
          evaluated as Eryn's two red-blue half-steps of 8 through Likelihood.__call__ (6 sampled
          parameters -> TransformContainer -> 14, red_blue.py:149-156);
config 5  -downsample 100 -Tobs 4 -nwalkers 128: one half-step of 64 walkers on the
          downsampled grid (emri_pe.py:322-374).
Each walker's logL (fused into the mode sum, and through template buffers + efd_loglike) is
compared with likelihood_oracle.loglike on the oracle's C-restatement spectra of the same
walker (same host upstream). Tolerance, written out: the oracle's spectra are trusted to the
per-bin split bound of tests/helpers.split_check (1e-9 max|R| off the folds, 2 D_k on fold
bins); with r = d - h w and e = ||tol_d w|| + ||tol_h w|| (the bound on ||Delta r||),
|ll_gpu - ll_oracle| <= 4 ||r|| e + 2 e^2 (Cauchy-Schwarz on -2 sum |r|^2). The GPU templates
of the first walkers are also held to split_check bin by bin.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from emri_frequencydomainwaveforms_amd import pe  # noqa: E402
from emri_frequencydomainwaveforms_amd.fdutils import get_sensitivity  # noqa: E402
from oracle import likelihood_oracle as lo  # noqa: E402
from tests.helpers import (channel_tolerance, channels, oracle_spectra, record_parity,  # noqa: E402
                           split_check)


def _oracle_ll(s, walkers6, check_templates=2):
    """Oracle logL per walker, its tolerance, and per-bin template checks of the first ones."""
    f = s.f_like
    w = lo.noise_factor(f, [get_sensitivity(f)] * 2)
    R, Rps, grid, E = oracle_spectra(s.few, s.truth14, s.kwargs, perturb_seeds=(1, 999))
    ok, st, tolS = split_check(R, R, Rps, E=E)   # the injection's own tolerance vector
    d = channels(R, grid) * w
    e_d = np.sqrt(np.sum((channel_tolerance(tolS, grid) * w) ** 2))
    params14 = s.transform.both_transforms(walkers6)
    ll, bound, stats = [], [], []
    for i, p in enumerate(params14):
        seeds = (2 + i, 1000 + i) if i < check_templates else (2 + i,)
        Ri, Rpi, _, Ei = oracle_spectra(s.few, p, s.kwargs, perturb_seeds=seeds)
        h = channels(Ri, grid)
        ll.append(lo.loglike(h, d, w))
        _, _, tol_i = split_check(Ri, Ri, Rpi, E=Ei)
        e = e_d + np.sqrt(np.sum((channel_tolerance(tol_i, grid) * w) ** 2))
        rn = np.sqrt(np.sum(np.abs(d - h * w) ** 2))
        bound.append(4.0 * rn * e + 2.0 * e * e)
        if i < check_templates:
            # the GPU template of this walker, bin by bin against the oracle
            S = s.few._spectrum(*p, **s.kwargs).cpu().numpy()
            ok_i, st_i, _ = split_check(S, Ri, Rpi, E=Ei)
            assert ok_i, st_i
            np.testing.assert_array_equal(S != 0, Ri != 0)
            stats.append(st_i)
    return np.array(ll), np.array(bound), stats


def _run(s, name, half_steps=2):
    like = s.like
    batches = s.half_steps()[:half_steps]
    like.fused_likelihood = True
    llf = np.concatenate([like(b, **s.kwargs) for b in batches])
    assert np.array_equal(np.concatenate([like(b, **s.kwargs) for b in batches]), llf)
    like.fused_likelihood = False
    llu = np.concatenate([like(b, **s.kwargs) for b in batches])
    like.fused_likelihood = True
    np.testing.assert_allclose(llf, llu, rtol=1e-12, atol=0.0)   # reduction order differs
    # the injection itself (sampled coordinates of the truth): logL = 0 exactly
    assert like(s.truth6[None, :], **s.kwargs)[0] == 0.0
    walkers = np.concatenate(batches)
    ref, bound, tstats = _oracle_ll(s, walkers)
    err = np.abs(llf - ref)
    rec = {"config": name, "walkers": int(len(walkers)), "ll_gpu": llf.tolist(),
           "ll_oracle": ref.tolist(), "abs_err": err.tolist(), "bound": bound.tolist(),
           "max_err_over_bound": float(np.max(err / bound)), "template_checks": tstats,
           "info": s.info}
    record_parity(name, rec)
    assert np.all(err <= bound), rec
    assert np.all(llf < 0.0)
    return rec


def test_config4_emri_pe_likelihood_full_grid():
    s = pe.setup(Tobs=2.0, dt=10.0, eps=1e-2, nwalkers=16, ntemps=1)
    assert s.info["N_f"] == 6311631 and s.half_step == 8 and s.like.subset == 24
    _run(s, "config4")


def test_config5_emri_pe_downsampled_likelihood():
    s = pe.setup(Tobs=4.0, dt=10.0, eps=1e-2, downsample=100, nwalkers=128, ntemps=1)
    assert s.half_step == 64 and s.kwargs.get("f_arr") is not None
    f = s.kwargs["f_arr"]
    assert np.array_equal(f, -f[::-1]) and len(f) < s.info["N_f"] // 50
    _run(s, "config5", half_steps=1)      # one half-step of 64 walkers

"""Shared test helpers: synthetic multi-harmonic inputs of the hot path."""

import numpy as np

from emri_frequencydomainwaveforms_amd.amplitude import ModeSelector, SyntheticTeukolskyAmplitude
from emri_frequencydomainwaveforms_amd.constants import Gpc, MRSUN_SI, MTSUN_SI
from emri_frequencydomainwaveforms_amd.frequencies import get_fundamental_frequencies
from emri_frequencydomainwaveforms_amd.summation import fd_grid
from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
from emri_frequencydomainwaveforms_amd.ylm import GetYlms


def source_inputs(M=3e5, mu=10.0, e0=0.35, T=0.02, dt=20.0, eps=1e-2, p0=None, modes=None,
                  theta=np.pi / 3, phi=-np.pi / 2, dist=1.0):
    """Stand-in trajectory + amplitudes + Ylm for one source; returns a dict of hot-path inputs."""
    traj = EMRIInspiral()
    if p0 is None:
        p0 = get_p_at_t(traj, 0.99 * T, [M, mu, 0.0, e0, 1.0])
    t, p, e, x, pp, pt, pr = traj(M, mu, 0.0, p0, e0, 1.0, T=T)
    amp = SyntheticTeukolskyAmplitude()
    yg = GetYlms(assume_positive_m=True)
    A = amp(p, e)
    ylms = yg(amp.l_arr, amp.m_arr, theta, phi)
    Kall = amp.num_teuk_modes
    if modes is None:
        keep = ModeSelector(amp.m0mask)(A, ylms, None, eps=eps)
    else:
        keep = np.array([amp.lmn_indices[tuple(md)] for md in modes])
    op, _, orr = get_fundamental_frequencies(0.0, p, e, 0.0)
    return dict(t=t, amp=A[:, keep].T.copy(), phi_phi=pp, phi_r=pr,
                f_phi=op / (2 * np.pi * M * MTSUN_SI), f_r=orr / (2 * np.pi * M * MTSUN_SI),
                m=amp.m_arr[keep].astype(np.int32), n=amp.n_arr[keep].astype(np.int32),
                l=amp.l_arr[keep].astype(np.int32),
                ylm_p=ylms[:Kall][keep], ylm_m=ylms[Kall:][keep],
                prefactor=mu * MRSUN_SI / (dist * Gpc), freq=fd_grid(T, dt), p=p, e=e, M=M,
                mu=mu, p0=p0, e0=e0, T=T, dt=dt)


# ---------------------------------------------------------------------------------------------
# Full-size parity: the split tolerance and the oracle on the drivers' own parameters
# ---------------------------------------------------------------------------------------------

# The oracle's conditioning is probed with PERTURB_ULPS-ulp random changes of its trajectory
# inputs. The kernel differs from the oracle by more than 1 ulp of input: its spline solves use
# a reciprocal estimate + Newton steps and a different evaluation order, so its coefficients
# carry a few ulps of rounding of their own. Measured at config 2's folds (round 3, 1-ulp
# probe): |S - R| reached 4.8 x the 1-ulp response; the response is linear in the probe size
# there, so a 4-ulp probe (and the 2 D bound) covers an effective 8 ulps.
PERTURB_ULPS = 4


def ulp_perturbation(seed, ulps=PERTURB_ULPS):
    """x -> x (1 +- ulps 2^-52) elementwise: a random `ulps`-ulp change of a trajectory array."""
    rng = np.random.default_rng(seed)
    return lambda x: x * (1.0 + rng.choice([-1.0, 1.0], len(x)) * ulps * 2.0 ** -52)


def split_check(S, R, Rps, rel=1e-9, dilate=8, E=None, Rps1=None):
    """Per-bin parity of a spectrum S against the oracle's R.

    D_k = max over the perturbed oracle runs Rps (PERTURB_ULPS ulps of the trajectory arrays) of
    |Rp_k - R_k|, dilated by a running max over +-dilate bins: the oracle's own conditioning
    at bin k. The inverse spline t(F) is ill-conditioned near turning points of F (folds),
    where 1 ulp of input moves bins by up to ~3e-5 of a harmonic's peak. Fold bins are those with D_k > rel max|R|; there the bound is
    |S_k - R_k| <= 2 D_k. Every other bin must meet |S_k - R_k| <= rel max|R|, so an error in
    a smooth bin cannot hide under the folds' floor.

    E (optional, fd_oracle_c.modesum(..., extrap=True)): per bin, the magnitude of the terms
    whose t(g) the splines extrapolate outside the trajectory (the inverse spline of a nearly
    flat run overshoots its times; scipy's CubicSpline, which the notebook uses, extrapolates).
    Their phase comes from cubics evaluated far outside their intervals, so two faithful
    evaluations agree in magnitude only: those bins get + 2 E_k. Returns (ok, stats, tol[k]).

    Rps1 (optional): the oracle perturbed by ONE ulp instead. Not part of the pass rule; it adds
    D1 (the same dilated response at 1 ulp) and err / D1 at the bins where D1 > rel max|R| to the
    stats: how the kernel's fold error compares with the reference construction's own rounding
    sensitivity."""
    from scipy.ndimage import maximum_filter1d
    mx = float(np.abs(R).max())
    D = np.zeros(len(R))
    for Rp in Rps:
        D = np.maximum(D, np.abs(Rp - R))
    if dilate:
        D = maximum_filter1d(D, size=2 * dilate + 1, mode="nearest")
    fold = D > rel * mx
    tol = np.where(fold, 2.0 * D, rel * mx)
    ext = np.zeros(len(R), dtype=bool) if E is None else E > 0.0
    if E is not None:
        tol = tol + 2.0 * E
    err = np.abs(S - R)
    ok = bool(np.all(err <= tol))
    off = err[~fold & ~ext]
    stats = {"bins": int(len(R)), "max_abs_R": mx,
             "max_err_rel": float(err.max() / mx) if mx > 0 else 0.0,
             "max_err_off_fold_rel": float(off.max() / mx) if off.size and mx > 0 else 0.0,
             "fold_bins": int(fold.sum()),
             "D_max_rel": float(D.max() / mx) if mx > 0 else 0.0,
             "max_err_over_D_at_folds": float((err[fold] / D[fold]).max()) if fold.any() else 0.0,
             "extrapolated_bins": int(ext.sum()),
             "max_err_over_E_at_extrapolated": (float((err[ext] / E[ext]).max())
                                                if ext.any() else 0.0),
             "tolerance": f"|S-R| <= {rel:g} max|R| off the folds, <= 2 D_k at the "
                          f"{int(fold.sum())} fold bins (D: {PERTURB_ULPS}-ulp oracle response, "
                          f"+-{dilate}-bin running max), + 2 E_k at the {int(ext.sum())} bins "
                          f"with extrapolated terms",
             "ok": ok}
    # the tolerance a user can rely on, per bin class, relative to max|R|: off the folds the
    # 1e-9 rule; at the folds the measured worst error (the bound there is 2 D_k)
    stats["tol_rel_by_class"] = {"off_fold": rel,
                                 "fold_measured_max": float(err[fold].max() / mx)
                                 if fold.any() and mx > 0 else 0.0,
                                 "fold_bound_max": float(2.0 * D.max() / mx) if mx > 0 else 0.0}
    if Rps1:
        D1 = np.zeros(len(R))
        for Rp in Rps1:
            D1 = np.maximum(D1, np.abs(Rp - R))
        if dilate:
            D1 = maximum_filter1d(D1, size=2 * dilate + 1, mode="nearest")
        f1 = (D1 > rel * mx) & ~ext
        stats["D1_fold_bins"] = int(f1.sum())
        stats["max_err_over_D1_at_folds"] = float((err[f1] / D1[f1]).max()) if f1.any() else 0.0
        stats["D1_max_rel"] = float(D1.max() / mx) if mx > 0 else 0.0
    if not ok:
        k = int(np.argmax(err - tol))
        stats["worst_bin"] = {"k": k, "err_rel": float(err[k] / mx), "tol_rel": float(tol[k] / mx),
                              "fold": bool(fold[k])}
    return ok, stats, tol


def record_parity(name, stats):
    """Write a parity record to $EFD_PARITY_OUT/<name>.json (collated into profiles/ by
    tools/collect_parity.py); a no-op when the variable is unset."""
    import json
    import os
    out = os.environ.get("EFD_PARITY_OUT")
    if not out:
        return
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"{name}.json"), "w") as fh:
        json.dump(stats, fh, indent=1, default=float)


def oracle_spectra(few, params14, kw, perturb_seeds=(), threads=None, caustic="uniform"):
    """C-oracle spectra for the 14 FEW parameters through the same host upstream as the
    generator (trajectory, amplitudes, Ylm, mode selection: stand-ins) on the generator's grid.

    Returns (R, [R with every trajectory array (t, f_phi, Phi_phi, f_r, Phi_r) perturbed by
    PERTURB_ULPS ulps, per seed], grid, E = the extrapolated terms' magnitude per bin)."""
    import os
    from emri_frequencydomainwaveforms_amd.waveform import get_viewing_angles, polarization_angle
    from oracle import fd_oracle_c
    threads = threads or min(16, len(os.sched_getaffinity(0)))
    wg = few.waveform_generator
    M, mu, _a, p0, e0, _x0, dist, qS, phiS, qK, phiK, pp0, _pt0, pr0 = (float(v) for v in params14)
    theta, phi = get_viewing_angles(qS, phiS, qK, phiK)
    rot = np.exp(-2j * polarization_angle(qS, phiS, qK, phiK)) if few.frame == "detector" else 1.0
    d = wg.prepare(M, mu, p0, e0, theta, phi, dist, pp0, pr0, kw["T"], kw["eps"])
    scale = complex(rot) * (mu * MRSUN_SI / (dist * Gpc))
    grid = np.asarray(kw["f_arr"]) if kw.get("f_arr") is not None else fd_grid(kw["T"], kw["dt"])
    K = len(d["m"])

    def run(t, fphi, pphi, fr, pr, extrap=False):
        return fd_oracle_c.modesum(t, d["teuk"].T, pphi, pr, fphi, fr, d["m"], d["n"],
                                   d["ylms"][:K], d["ylms"][K:], grid, scale, caustic=caustic,
                                   nthreads=threads, extrap=extrap)

    R, E = run(d["t"], d["f_phi"], d["Phi_phi"], d["f_r"], d["Phi_r"], extrap=True)
    Rps = []
    for s in perturb_seeds:
        p = ulp_perturbation(s)
        Rps.append(run(p(d["t"]), p(d["f_phi"]), p(d["Phi_phi"]), p(d["f_r"]), p(d["Phi_r"])))
    return R, Rps, grid, E


def channels(S, grid):
    """[h+, hx] over f >= 0 (FEW list output with mask_positive) from a two-sided S."""
    Sf = S[::-1]
    keep = np.asarray(grid) >= 0.0
    return np.stack([0.5 * (S + np.conj(Sf))[keep], 0.5j * (S - np.conj(Sf))[keep]])


def channel_tolerance(tolS, grid):
    """Per-bin bound on each channel from a per-bin bound on S (h = (S(f) +- conj S(-f)) / 2)."""
    keep = np.asarray(grid) >= 0.0
    return 0.5 * (tolS + tolS[::-1])[keep]

"""emri_pe.py-shaped likelihood setup (BASELINE.json configs 4 and 5) on the MI355X path.

Mirrors run_emri_pe's preamble (emri_pe.py:125-450) with this package's drop-ins:
  source and fixed angles                     emri_pe.py:590-635 (p0 re-solved for 0.99 Tobs)
  sampled 6-vector, fill_dict, transforms     :161-206 (TransformContainer, transform_mass_ratio)
  FD injection [h+, hx] over f >= 0           :203, 238-241, 276 (get_fd_waveform_fromFD)
  downsampled grid to 1.01 x the last non-zero bin, len/downsample points   :322-364
  Likelihood(..., subset=24) + inject_signal with LISA_Alloc_Sh noise         :381-417
  walker start multivariate_normal(truth, cov(covariance.npy) / (2.4 ndim))   :437-444
The covariance is shipped as data (data/walker_cov.npy, from tools/make_walker_cov.py). The
start uses numpy's Generator seeded with the reference's SEED = 2601996 (emri_pe.py:65), so the
walkers are reproducible, not the reference's own draws. One Eryn red-blue half-step evaluates
ntemps * nwalkers / 2 walkers in one Likelihood call (red_blue.py:149-156, ensemble.py:1283-1318).
"""

import os
from dataclasses import dataclass, field

import numpy as np

from .transforms import TransformContainer, transform_mass_ratio

SUM_KW = dict(pad_output=True, output_type="fd", odd_len=True)
SEED = 2601996
FILL_INDS = np.array([2, 5, 6, 7, 8, 9, 10, 12])
_COV = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "walker_cov.npy")


@dataclass
class PESetup:
    few: object              # GenerateEMRIWaveform(..., return_list=True)
    gen: object              # get_fd_waveform_fromFD template
    like: object             # Likelihood with the "emri" TransformContainer
    transform: object
    truth14: np.ndarray      # injection parameters (14, FEW order)
    truth6: np.ndarray       # sampled coordinates of the injection
    start: np.ndarray        # [ntemps * nwalkers, 6] walker start
    kwargs: dict             # waveform kwargs of every likelihood call (T, dt, eps[, f_arr])
    f_like: np.ndarray       # the likelihood's frequencies (f >= 0 of the template grid)
    half_step: int           # walkers per Likelihood call (ntemps * nwalkers / 2)
    info: dict = field(default_factory=dict)

    def half_steps(self):
        """The start's walker batches, one per red-blue half-step."""
        B = self.half_step
        return [self.start[i:i + B] for i in range(0, len(self.start), B)]


def setup(Tobs=2.0, dt=10.0, eps=1e-2, M=1e6, mu=10.0, e0=0.35, downsample=None, nwalkers=16,
          ntemps=1, seed=SEED, caustic="uniform", subset=24, window_flag=False, freeze_gc=True):
    """window_flag: the templates and the injection convolved with a Hann window of the grid's
    length (emri_pe.py:259-263, -window_flag 1 in test.sh: scipy.signal.windows.hann(N), N the
    TD/FD length, odd_len); not with downsampling (emri_pe.py:330-331).
    freeze_gc: collect, then move every object alive after the setup (torch's and scipy's
    modules, the likelihood, its grids) out of the cyclic collector's reach (gc.freeze), as a
    sampler process would once its setup is done: a full collection otherwise walks ~200 k
    objects, 35 ms (130 ms with a dropped setup's garbage), inside whichever likelihood call
    happens to trigger it (tools/api_trace.py, tools/gc_cycles.py)."""
    from .fdutils import get_fd_waveform_fromFD, get_sensitivity
    from .likelihood import Likelihood
    from .trajectory import EMRIInspiral, get_p_at_t
    from .waveform import GenerateEMRIWaveform

    a, x0, Phi_theta0 = 0.1, 1.0, 0.0           # a, x0 ignored for Schwarzschild (:598, :602)
    qK = phiK = qS = phiS = np.pi / 3
    dist = 2.4539054256
    Phi_phi0 = Phi_r0 = np.pi / 3
    p0 = float(get_p_at_t(EMRIInspiral(), Tobs * 0.99, [M, mu, 0.0, e0, 1.0]))
    truth14 = np.array([M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0, Phi_theta0,
                        Phi_r0], dtype=np.float64)
    fill = {"ndim_full": 14, "fill_values": np.array([0.0, x0, dist, qS, phiS, qK, phiK,
                                                      Phi_theta0]),
            "fill_inds": FILL_INDS.copy()}
    tc = TransformContainer({(0, 1): transform_mass_ratio}, fill)
    truth6 = np.delete(truth14.copy(), FILL_INDS)
    truth6[1] = np.log(truth6[1] / truth6[0])
    truth6[0] = np.log(truth6[0])
    injection = tc.both_transforms(truth6[None, :])[0]

    few = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux", sum_kwargs=SUM_KW,
                               use_gpu=True, return_list=True, caustic=caustic)
    kw = dict(T=Tobs, dt=dt, eps=eps)
    sig = few(*injection, mask_positive=True, **kw)
    frequency = few.waveform_generator.create_waveform.frequency
    frequency = frequency.cpu().numpy() if hasattr(frequency, "detach") else np.asarray(frequency)
    pos = frequency >= 0.0
    info = {"p0": p0, "N_f": int(len(frequency))}
    like_subset = subset
    window = None
    if window_flag:
        if downsample:
            raise ValueError("Cannot run downsampling with windowing")   # emri_pe.py:331
        from scipy.signal.windows import hann
        window = hann(len(frequency))
        info["window"] = "hann"
    if downsample:
        fixed = frequency[pos]
        nz = np.abs(sig[0].cpu().numpy()) > 1e-50                    # emri_pe.py:245
        num = int(nz.sum() / downsample)
        p_freq = np.linspace(0.0, fixed[nz].max() * 1.01, num=num)
        newfreq = np.hstack((-p_freq[::-1][:-1], p_freq))
        kw["f_arr"] = newfreq
        pos = newfreq >= 0.0
        f_like = newfreq[pos]
        like_subset = None                                           # like_ds (:366-374)
        info.update(downsample=downsample, N_f_downsampled=int(len(newfreq)))
    else:
        f_like = frequency[pos]
    gen = get_fd_waveform_fromFD(few, pos, dt, window=window)
    like = Likelihood(gen, 2, parameter_transforms={"emri": tc}, vectorized=False,
                      transpose_params=False, subset=like_subset, f_arr=f_like, use_gpu=True)
    data = gen(*injection, **kw)
    like.inject_signal(data_stream=data, noise_fn=[get_sensitivity, get_sensitivity],
                       noise_kwargs=[{}, {}])
    cov = np.load(_COV, allow_pickle=False) / (2.4 * 6)
    rng = np.random.default_rng(seed)
    start = rng.multivariate_normal(truth6, cov, size=nwalkers * ntemps)
    if freeze_gc:
        import gc
        gc.collect()
        gc.freeze()
    return PESetup(few=few, gen=gen, like=like, transform=tc, truth14=injection,
                   truth6=truth6, start=start, kwargs=kw, f_like=f_like,
                   half_step=max(1, nwalkers * ntemps // 2), info=info)


class MemoizedUpstream:
    """Memoise a generator's host upstream (trajectory, amplitudes, Ylm, mode selection: the
    stand-ins of trajectory.py / amplitude.py) per parameter set, so repeated likelihood calls on
    the same walkers time the device path alone ("inputs resident"). Installed on the instance;
    `remove()` restores it. Arrays in kwargs (f_arr) are keyed by identity."""

    def __init__(self, wg):
        import time
        self._time = time.perf_counter
        self.wg = wg
        self.orig = wg.prepare
        self.memo = {}
        self.host_s = 0.0
        wg.prepare = self
        if hasattr(wg, "prefetch"):
            wg.prefetch = lambda calls, wait=True, concurrency=None: 0   # the memo holds it

    def __call__(self, *args, **kwargs):
        # submit_batch calls positionally with plain floats (and None / bool flags): the args
        # tuple is the key, as prepare()'s own prefetch lookup keys on them
        key = args if not kwargs else (
            tuple(float(a) if isinstance(a, (float, int, np.floating)) else a for a in args),
            tuple(sorted((k, ("id", id(v)) if hasattr(v, "shape") else v)
                         for k, v in kwargs.items())))
        hit = self.memo.get(key)
        if hit is None:
            t0 = self._time()
            hit = self.memo[key] = self.orig(*args, **kwargs)
            self.host_s += self._time() - t0
        return hit

    def remove(self):
        for name in ("prepare", "prefetch"):
            if name in self.wg.__dict__:
                delattr(self.wg, name)   # back to the class's methods

"""Teukolsky-amplitude STAND-IN and mode selection (host side, upstream of the hot path).

The reference evaluates `RomanAmplitude` (ROMAN network, 3843 complex modes l<=10, 0<=m<=l,
|n|<=30) and keeps modes with `ModeSelector(eps)` (Tutorial_FD_construction_single_mode.ipynb:32,
:37, :125-127; `eps` kwarg emri_pe.py:659-663). The network weights are absent offline (SURVEY.md
section 2, row 1c), so `SyntheticTeukolskyAmplitude` returns seeded, smooth complex amplitudes
with the same mode list, ordering and call surface. Magnitudes fall off geometrically in l, l-m
and |n - n_peak(e)| (eccentric orbits spread power over n), and grow as p shrinks, tuned so that
eps = 1e-5 keeps ~3000 modes and eps = 1e-2 keeps ~10^2 at e ~ 0.35 like the reference's
BASELINE configs. NOT FEW physics: only the workload shape (modes, supports) is meaningful.

`ModeSelector` restates FEW's power-based selection [FEW-ext, from the FEW 1.x sources as
recalled in SURVEY.md]: per trajectory point, sort |A Y|^2 over the m>=0 and partner -m
branches, keep the modes needed to reach (1 - eps) of the power, fold -m picks onto +m, take
the union over time.
"""

import ctypes

import numpy as np

LMAX = 10
NMAX = 30
_SEED = 2601996  # the reference's SEED (check_mode_by_mode.py:47, emri_pe.py:65)


def mode_list(lmax=LMAX, nmax=NMAX):
    l_arr, m_arr, n_arr = [], [], []
    for l in range(2, lmax + 1):
        for m in range(0, l + 1):
            for n in range(-nmax, nmax + 1):
                l_arr.append(l)
                m_arr.append(m)
                n_arr.append(n)
    return (np.asarray(l_arr, dtype=np.int32), np.asarray(m_arr, dtype=np.int32),
            np.asarray(n_arr, dtype=np.int32))


class SyntheticTeukolskyAmplitude:
    """Seeded smooth complex A_lmn(p, e) over FEW's 3843-mode list (stand-in for RomanAmplitude)."""

    def __init__(self, lmax=LMAX, nmax=NMAX, seed=_SEED, use_gpu=False, **kwargs):
        self.l_arr, self.m_arr, self.n_arr = mode_list(lmax, nmax)
        self.num_teuk_modes = len(self.l_arr)
        self.m0mask = self.m_arr != 0
        self.num_m_zero_up = self.num_teuk_modes
        self.num_m0 = int(np.sum(~self.m0mask))
        self.num_m_1_p = self.num_teuk_modes  # index offset of the -m partners in power arrays
        self.lmn_indices = {(int(l), int(m), int(n)): i
                            for i, (l, m, n) in enumerate(zip(self.l_arr, self.m_arr, self.n_arr))}
        lm = np.stack([self.l_arr, self.m_arr], axis=1)
        unique_lm, self.inverse_lm = np.unique(lm, axis=0, return_inverse=True)
        self.inverse_lm = self.inverse_lm.reshape(-1)
        self.unique_l, self.unique_m = unique_lm[:, 0], unique_lm[:, 1]
        rng = np.random.default_rng(seed)
        self._phase0 = rng.uniform(0.0, 2.0 * np.pi, self.num_teuk_modes)
        self._jitter = rng.uniform(-0.15, 0.15, self.num_teuk_modes)

    def _log10_mag(self, p, e):
        l = self.l_arr[None, :].astype(np.float64)
        m = self.m_arr[None, :].astype(np.float64)
        n = self.n_arr[None, :].astype(np.float64)
        p = np.asarray(p, dtype=np.float64)[:, None]
        e = np.asarray(e, dtype=np.float64)[:, None]
        n_peak = m * 1.4 * e
        width = 0.35 + 2.2 * e        # eccentric orbits spread power over many n
        decay = 0.42 * (l - 2.0) + 0.30 * (l - m) + 0.60 * np.abs(n - n_peak) / width
        # a steep core holding ~99% of the power over a slowly decaying tail: eps = 1e-2 keeps
        # ~10^2 modes, eps = 1e-5 reaches into the tail and keeps ~3000
        core = -1.0 - decay
        tail = -3.6 - 0.085 * decay
        return (np.log10(10.0 ** core + 10.0 ** tail)
                + 0.5 * (l + 2.0) * np.log10(10.0 / p) + self._jitter[None, :])

    def __call__(self, p, e, *args, specific_modes=None, **kwargs):
        p = np.atleast_1d(np.asarray(p, dtype=np.float64))
        e = np.atleast_1d(np.asarray(e, dtype=np.float64))
        mag = 10.0 ** self._log10_mag(p, e)
        # slow, smooth phase drift along the inspiral keeps Re/Im splines non-trivial
        drift = 0.2 * (self.l_arr[None, :] - self.m_arr[None, :] + 1) * (10.0 / p[:, None]) \
            + 0.1 * self.n_arr[None, :] * e[:, None]
        amps = mag * np.exp(1j * (self._phase0[None, :] + drift))
        if specific_modes is None:
            return amps
        out = {}
        for lmn in specific_modes:
            l, m, n = (int(v) for v in lmn)
            if m >= 0:
                out[(l, m, n)] = amps[:, self.lmn_indices[(l, m, n)]]
            else:  # FEW symmetry A_{l,-m,-n} = (-1)^l conj(A_{l,m,n})
                out[(l, m, n)] = (-1.0) ** l * np.conj(amps[:, self.lmn_indices[(l, -m, -n)]])
        return out


    def select(self, p, e, ylms, eps, lib=None):
        """(keep, teuk): ModeSelector(eps) over this model's modes and the kept modes' complex
        amplitudes [N_t][K], in one native call (csrc/emrifd_host.cpp: efd_host_modes) when the
        library is available, else through __call__ + ModeSelector (numpy). ylms: the GetYlms
        output [Y_lm..., (-1)^l Y_l-m...] over the whole mode list."""
        if lib is None or not hasattr(lib, "efd_host_modes"):
            A = self(p, e)
            keep = ModeSelector(self.m0mask)(A, ylms, None, eps=eps)
            return keep, np.ascontiguousarray(A[:, keep])
        p = np.ascontiguousarray(p, dtype=np.float64)
        e = np.ascontiguousarray(e, dtype=np.float64)
        K = self.num_teuk_modes
        yp = np.ascontiguousarray(ylms[:K], dtype=np.complex128)
        ym = np.ascontiguousarray(ylms[K:], dtype=np.complex128)
        keep = np.empty(K, dtype=np.int32)
        nkeep = ctypes.c_int32(0)
        nt = len(p)
        cap = 2 * nt * K   # np.empty: untouched pages cost nothing
        for _ in range(2):
            teuk = np.empty(cap // 2, dtype=np.complex128)
            rc = lib.efd_host_modes(p.ctypes.data, e.ctypes.data, nt, self.l_arr.ctypes.data,
                                    self.m_arr.ctypes.data, self.n_arr.ctypes.data,
                                    self._phase0.ctypes.data, self._jitter.ctypes.data, K,
                                    yp.ctypes.data, ym.ctypes.data, float(eps), keep.ctypes.data,
                                    ctypes.byref(nkeep), teuk.ctypes.data, cap)
            if rc == 0:
                k = nkeep.value
                return keep[:k].astype(np.int64), teuk[:nt * k].reshape(nt, k)
            if rc != -3:
                raise RuntimeError(f"efd_host_modes failed ({rc})")
            cap = 2 * nt * nkeep.value
        raise RuntimeError("efd_host_modes: amplitude buffer")


# FEW-compatible name used by the reference notebooks
RomanAmplitude = SyntheticTeukolskyAmplitude


class ModeSelector:
    """Keep the modes carrying (1 - eps) of the power (few.utils.modeselector.ModeSelector)."""

    def __init__(self, m0mask, use_gpu=False):
        self.m0mask = np.asarray(m0mask, dtype=bool)
        self.num_m_1_p = len(self.m0mask)

    def __call__(self, teuk_modes, ylms, modeinds, eps=1e-5):
        """teuk_modes [N_t, K]; ylms [K + K] (+m then partner); returns kept mode indices."""
        K = teuk_modes.shape[1]
        ylm_p, ylm_m = ylms[:K], ylms[K:]
        # m = 0 modes have no separate partner branch (their +-n mirrors are separate modes)
        partner = np.conj(teuk_modes[:, self.m0mask]) * ylm_m[self.m0mask][None, :]
        power = np.abs(np.concatenate([teuk_modes * ylm_p[None, :], partner], axis=1)) ** 2
        partner_idx = np.nonzero(self.m0mask)[0]
        inds_sort = np.argsort(power, axis=1)[:, ::-1]
        power = np.take_along_axis(power, inds_sort, axis=1)
        cumsum = np.cumsum(power, axis=1)
        keep = np.ones(cumsum.shape, dtype=bool)
        keep[:, 1:] = cumsum[:, :-1] < cumsum[:, -1][:, None] * (1.0 - eps)
        picked = inds_sort[keep]
        # fold partner picks back onto their +m mode
        picked = np.where(picked < K, picked, partner_idx[np.clip(picked - K, 0, None)])
        return np.unique(picked)

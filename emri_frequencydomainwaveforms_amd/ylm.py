"""Spin-weight -2 spherical harmonics (host side; replaces `few.utils.ylm.GetYlms`).

Call surface follows the reference notebooks: ``GetYlms(assume_positive_m=True, use_gpu=False)``
then ``ylm_gen(l_arr, m_arr, theta, phi)`` (Tutorial_FD_construction_single_mode.ipynb:87, :130,
:597). With ``assume_positive_m=True`` the output is ``[Y_lm ..., (-1)^l Y_{l,-m} ...]``: the
second half is the partner factor used for the -m branch (notebook :611 multiplies the
conjugated amplitude by ``ylms[1]``).

Formula: Goldberg et al. (1967),
  sY_lm = (-1)^m sqrt((l+m)!(l-m)!(2l+1) / (4 pi (l+s)!(l-s)!)) sin^{2l}(th/2)
          * sum_r C(l-s, r) C(l+s, r+s-m) (-1)^{l-r-s} e^{i m phi} cot^{2r+s-m}(th/2)
with s = -2, written with explicit sin/cos powers so theta = 0, pi are finite.
The overall sign/phase convention of FEW's ylm module is [FEW-ext] and not checkable offline
(SURVEY.md section 0.2); this one matches the LAL convention, e.g.
-2Y_22 = sqrt(5/(64 pi)) (1 + cos th)^2 e^{2 i phi}.
"""

from math import comb, factorial, sqrt, pi

import numpy as np


def _swsh_m2(l, m, theta, phi):
    s = -2
    if l < 2 or abs(m) > l:
        return 0.0 + 0.0j
    pref = (-1.0) ** m * sqrt(
        factorial(l + m) * factorial(l - m) * (2 * l + 1)
        / (4.0 * pi * factorial(l + s) * factorial(l - s)))
    sh = np.sin(theta / 2.0)
    ch = np.cos(theta / 2.0)
    acc = 0.0
    for r in range(0, l - s + 1):
        k2 = r + s - m
        if k2 < 0 or k2 > l + s:
            continue
        c = comb(l - s, r) * comb(l + s, k2) * (-1.0) ** (l - r - s)
        pw = 2 * r + s - m                       # power of cot(theta/2)
        acc += c * (ch ** pw) * (sh ** (2 * l - pw))
    return pref * acc * np.exp(1j * m * phi)


class GetYlms:
    """-2 spin-weighted spherical harmonics, FEW-compatible call surface."""

    def __init__(self, assume_positive_m=False, use_gpu=False):
        self.assume_positive_m = assume_positive_m
        self.use_gpu = use_gpu  # host-only: Ylm cost is O(K), off the hot path

    def __call__(self, l_in, m_in, theta, phi):
        l_in = np.atleast_1d(np.asarray(l_in, dtype=np.int64))
        m_in = np.atleast_1d(np.asarray(m_in, dtype=np.int64))
        if l_in.shape != m_in.shape:
            raise ValueError("l and m arrays must have the same shape")
        # cache per unique (l, m): the mode list repeats (l, m) for every n
        cache = {}

        def y(l, m):
            key = (int(l), int(m))
            if key not in cache:
                cache[key] = _swsh_m2(key[0], key[1], theta, phi)
            return cache[key]

        plus = np.array([y(l, m) for l, m in zip(l_in, m_in)], dtype=np.complex128)
        if not self.assume_positive_m:
            return plus
        minus = np.array([(-1.0) ** int(l) * y(l, -m) for l, m in zip(l_in, m_in)],
                         dtype=np.complex128)
        return np.concatenate([plus, minus])

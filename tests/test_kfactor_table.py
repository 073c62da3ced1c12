"""The uniform-SPA factor table (csrc/kfactor_table.inc) against scipy's K_{1/3}.

The general path of k_modesum evaluates G(y) = Q / Q_spa (notebook
Tutorial_FD_construction_single_mode.ipynb:599-608: Q = i F'/|F''| K_{1/3}(z) e^z 2/sqrt(3),
z = -i y) from a piecewise-polynomial table in w = 1/|y| for 2^-10 < |y| <= 256. This test
re-evaluates the table exactly as kfactor_tab does (interval from the bits of w, x = 8 m - (9 + 2k),
Horner in double) and compares it with G computed from scipy.special.kv (AMOS, what the notebook
calls) on random points of every interval, and with the Hankel series the fast path uses above
|y| = 153.
"""

import os
import re

import numpy as np
from scipy import special

INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "emri_frequencydomainwaveforms_amd", "csrc", "kfactor_table.inc")


def load_table():
    txt = open(INC).read()
    e_lo = int(re.search(r"#define KTAB_E_LO \((-?\d+)\)", txt).group(1))
    e_hi = int(re.search(r"#define KTAB_E_HI \((-?\d+)\)", txt).group(1))
    deg = int(re.search(r"#define KTAB_DEG (\d+)", txt).group(1))
    body = txt[txt.index("= {") + 3:]
    nums = [float(v) for v in re.findall(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?", body)]
    tab = np.array(nums).reshape(-1, deg + 1, 2)
    assert tab.shape[0] == 4 * (e_hi - e_lo)
    return tab, e_lo, e_hi, deg


def table_G(tab, e_lo, ww):
    """kfactor_tab, vectorised: (R, I) for y = 1/ww > 0."""
    bits = ww.view(np.uint64)
    hi = (bits >> np.uint64(32)).astype(np.int64)
    k = (hi >> 18) & 3
    idx = np.clip(4 * ((hi >> 20) - 1023 - e_lo) + k, 0, tab.shape[0] - 1)
    m = ((bits & np.uint64(0x000FFFFFFFFFFFFF)) | np.uint64(0x3FF0000000000000)).view(np.float64)
    x = 8.0 * m - (9 + 2 * k)
    c = tab[idx]
    r = np.zeros_like(ww)
    im = np.zeros_like(ww)
    for j in range(c.shape[1] - 1, -1, -1):
        r = r * x + c[:, j, 0]
        im = im * x + c[:, j, 1]
    return r + 1j * im


def scipy_G(y):
    """G(y) = e^{-i pi/4} sqrt(2y/pi) K_{1/3}(-iy) e^{-iy} for y > 0 (-> 1 as y -> inf)."""
    return (np.exp(-0.25j * np.pi) * np.sqrt(2.0 * y / np.pi) *
            special.kv(1.0 / 3.0, -1j * y) * np.exp(-1j * y))


def test_table_matches_scipy_kv():
    tab, e_lo, e_hi, _ = load_table()
    rng = np.random.default_rng(2601996)
    # 64 random points in each of the 4 quarters of every binade of w, plus both ends
    ws = []
    for e in range(e_lo, e_hi):
        for k in range(4):
            lo, hi = 2.0 ** e * (1 + k / 4), 2.0 ** e * (1 + (k + 1) / 4)
            ws.append(rng.uniform(lo, hi, 64))
            ws.append(np.array([lo, np.nextafter(hi, 0.0)]))
    ww = np.concatenate(ws)
    g_tab = table_G(tab, e_lo, ww)
    g_ref = scipy_G(1.0 / ww)
    err = np.abs(g_tab - g_ref)
    assert np.all(np.isfinite(g_ref))
    assert err.max() < 5e-15, f"max |G_table - G_scipy| = {err.max():.3e}"


def test_table_meets_fast_path_series():
    """Above |y| = 153 the fast path uses the Hankel series (KB, KC); the table must agree
    where both hold (153 <= |y| <= 256), so the split between the paths is seamless."""
    tab, e_lo, _, _ = load_table()
    # a_k of K_{1/3}: a_k = a_{k-1} (4/9 - (2k-1)^2) / (8k); G = sum a_k (i w)^k
    y = np.linspace(153.0, 256.0, 257)
    w = 1.0 / y
    a, g = 1.0, np.ones_like(y, dtype=complex)
    for k in range(1, 9):
        a *= (4.0 / 9.0 - (2 * k - 1) ** 2) / (8.0 * k)
        g = g + a * (1j * w) ** k
    g_tab = table_G(tab, e_lo, w)
    assert np.abs(g_tab - g).max() < 5e-16

"""The windowed logL's per-bin form (efd_hann_loglike_local) on the CPU: the
data layout fdutils.HannConvolution.local_layout builds, and the identity it rests on.

With h+ = (a + conj b)/2, hx = i (a - conj b)/2 for a = S_w[k], b = S_w[n-1-k] (the odd
two-sided grid's split, efd_polarizations) and the same weight w on both channels,
    |d0 - w h+|^2 + |d1 - w hx|^2 = (|(d0 - i d1) - w a|^2 + |(d0 + i d1) - w conj b|^2) / 2,
so the mirror-pair sum over the kept bins k >= k0 equals (1/2) sum_j |dl[j] - wl[j] S_w[j]|^2
over the grid, the self-mirror bin's second term from dl[n]. Checked in float64 at 1e-12
relative on random data, odd and even grids, with a masked (w = 0) bin. No GPU needed."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution  # noqa: E402


def _pair_form(Sw, d, w, k0):
    n = len(Sw)
    k = np.arange(k0, n)
    a, b = Sw[k], Sw[n - 1 - k]
    hp = 0.5 * (a + np.conj(b))
    hc = 0.5j * (a - np.conj(b))
    return float(np.sum(np.abs(d[0] - w[0] * hp) ** 2 + np.abs(d[1] - w[1] * hc) ** 2))


@pytest.mark.parametrize("n,k0", [(101, 50), (1001, 500), (100, 50), (11, 5)])
def test_local_layout_equals_pair_form(n, k0):
    rng = np.random.default_rng(n)
    nb = n - k0
    Sw = rng.normal(size=n) + 1j * rng.normal(size=n)
    d = rng.normal(size=(2, nb)) + 1j * rng.normal(size=(2, nb))
    w1 = rng.uniform(0.5, 2.0, size=nb)
    w1[0] = 0.0
    w = np.stack([w1, w1])
    dl, wl, kself = HannConvolution.local_layout(n, torch.as_tensor(d), torch.as_tensor(w), k0)
    dl, wl = dl.numpy(), wl.numpy()
    assert dl.shape == (n + 1,) and wl.shape == (n,)
    assert kself == (k0 if 2 * k0 == n - 1 else -1)
    local = 0.5 * float(np.sum(np.abs(dl[:n] - wl * Sw) ** 2))
    if kself >= 0:
        local += 0.5 * float(abs(dl[n] - wl[kself] * Sw[kself]) ** 2)
    pair = _pair_form(Sw, d, w, k0)
    assert abs(local - pair) <= 1e-12 * pair
    # bins neither kept nor mirrored carry no term
    k = np.arange(k0, n)
    live = np.zeros(n, dtype=bool)
    live[k] = live[n - 1 - k] = True
    assert np.all(dl[:n][~live] == 0) and np.all(wl[~live] == 0)


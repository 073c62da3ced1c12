"""Transform lengths of the Hann window's correction (fdutils.HannConvolution.size_for): the
smallest 2^a or 3 2^a that holds the linear convolution of a row's support with the lag kernel
(n + support - 1 points), so a spectrum whose harmonics stay below ~1/3 of Nyquist transforms at
about half the full-support length. No GPU needed."""

import pytest

from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution


@pytest.mark.parametrize("n,support,m", [
    (12623261, 12623261, 2 ** 25),          # full support: >= 2n - 1
    (12623261, 1800000, 2 ** 24),           # test.sh's harmonics (~14% of the grid)
    (12623261, 4153956, 2 ** 24),           # the most 2^24 holds
    (12623261, 4153957, 3 * 2 ** 23),
    (100001, 1, 2 ** 17),
    (100001, 0, 2 ** 17),                   # an all-zero batch
    (3, 3, 6),
])
def test_size_for(n, support, m):
    got = HannConvolution.size_for(n, support)
    assert got == m
    assert got >= n + max(support, 1) - 1
    # no smaller length of either family would do
    for base in (1, 3):
        k = base
        while k < got:
            assert k < n + max(support, 1) - 1
            k *= 2

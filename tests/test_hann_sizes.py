"""Transform lengths of the Hann window's correction (fdutils.HannConvolution.size_for): a
length that holds the linear convolution of a row's support with the lag kernel (n + support - 1
points): the power of two in efd_hann_convolve's range [2^21, 2^25] (its four-step pipeline),
else the smallest 2^a or 3 2^a (hipFFT). A spectrum whose harmonics stay below ~1/3 of Nyquist
transforms at about half the full-support length. No GPU needed."""

import pytest

from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution


@pytest.mark.parametrize("n,support,m", [
    (12623261, 12623261, 2 ** 25),          # full support: >= 2n - 1
    (12623261, 1800000, 2 ** 24),           # test.sh's harmonics (~14% of the grid)
    (12623261, 4153956, 2 ** 24),           # the most 2^24 holds
    (12623261, 4153957, 2 ** 25),           # four-step range: the power of two
    (1000001, 500000, 2 ** 21),             # (3 2^19 would hold it, on hipFFT)
    (16777217, 16777217, 3 * 2 ** 24),      # past 2^25: hipFFT's lengths
    (100001, 1, 2 ** 17),
    (100001, 0, 2 ** 17),                   # an all-zero batch
    (3, 3, 6),
])
def test_size_for(n, support, m):
    got = HannConvolution.size_for(n, support)
    assert got == m
    need = n + max(support, 1) - 1
    assert got >= need
    if not HannConvolution.FOUR_STEP_MIN <= got <= HannConvolution.FOUR_STEP_MAX:
        # no smaller length of either family would do
        for base in (1, 3):
            k = base
            while k < got:
                assert k < need
                k *= 2
    # without the four-step pipeline: the smallest of either family
    alt = HannConvolution.size_for(n, support, four_step=False)
    assert alt >= need and alt <= got

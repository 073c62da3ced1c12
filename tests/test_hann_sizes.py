"""Transform lengths of the Hann window's correction (fdutils.HannConvolution.size_for): a
length that holds the linear convolution of a row's support with the lag kernel (n + support - 1
points) and one point more (the fused logL reads the differenced correction one place below the
output window, efd_hann_loglike_local): the power of two in efd_hann_convolve's range [2^21, 2^25] (its four-step pipeline),
else the smallest 2^a or 3 2^a (hipFFT). A spectrum whose harmonics stay below ~1/3 of Nyquist
transforms at about half the full-support length. No GPU needed."""

import pytest

from emri_frequencydomainwaveforms_amd.fdutils import HannConvolution


@pytest.mark.parametrize("n,support,m", [
    (12623261, 12623261, 2 ** 25),          # full support: >= 2n - 1
    (12623261, 1800000, 2 ** 24),           # test.sh's harmonics (~14% of the grid)
    (12623261, 4153955, 2 ** 24),           # the most 2^24 holds
    (12623261, 4153956, 2 ** 25),           # four-step range: the power of two
    (1000001, 500000, 2 ** 21),             # (3 2^19 would hold it, on hipFFT)
    (16777217, 16777217, 3 * 2 ** 24),      # past 2^25: hipFFT's lengths
    (100001, 1, 2 ** 17),
    (100001, 0, 2 ** 17),                   # an all-zero batch
    (3, 3, 6),
    (3, 2, 6),
])
def test_size_for(n, support, m):
    got = HannConvolution.size_for(n, support)
    assert got == m
    need = n + max(support, 1)
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


def test_lane_support_bounds_the_support():
    """HannConvolution.lane_support (the host's transform-length input from the rows' lane
    ranges, no synchronisation): for random paired-grid rows whose nonzero bins lie in
    {l, n-1-l : lo <= l < hi}, the bound is at least every row's support (last + 1 - first) and
    the span the extent scan covers; empty rows count as support 1; one all-empty batch gives 1."""
    import numpy as np
    rng = np.random.default_rng(7)
    n = 100001
    lanes = []
    worst = 0
    for _ in range(64):
        lo = int(rng.integers(0, n // 2))
        hi = int(rng.integers(lo, n // 2 + 1))
        lanes.append((lo, hi))
        if hi > lo:
            # nonzero bins: a random subset of the lanes and their mirrors
            ls = rng.integers(lo, hi, size=5)
            bins = np.concatenate([ls, n - 1 - ls])
            worst = max(worst, int(bins.max()) + 1 - int(bins.min()))
            span = min(n, max(hi, n - lo)) - max(0, min(lo, n - hi))
            assert HannConvolution.lane_support(np.array([(lo, hi)], dtype=np.int32), n) == span
    bound = HannConvolution.lane_support(np.array(lanes, dtype=np.int32), n)
    assert bound >= worst
    assert HannConvolution.lane_support(np.array([(5, 5), (9, 3)], dtype=np.int32), n) == 1

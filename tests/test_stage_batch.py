"""efd_stage_batch (host C, no GPU): the batched likelihood's packing of walker inputs.

Each walker's ten arrays must land 256-B aligned, in order, byte-exact in the staging buffer,
and its argument struct must carry the template's grid fields, its own nt, K and scale, and
dev_base + the array's offset; a short buffer is refused with the size it needs.
"""

import ctypes

import numpy as np

from emri_frequencydomainwaveforms_amd import _lib


def _walker(rng, nt, K):
    f = lambda n: rng.standard_normal(n)  # noqa: E731
    c = lambda *s: rng.standard_normal(s) + 1j * rng.standard_normal(s)  # noqa: E731
    return [f(nt), f(nt), f(nt), f(nt), f(nt), c(nt, K),
            rng.integers(-10, 10, K).astype(np.int32), rng.integers(-30, 30, K).astype(np.int32),
            c(K), c(K)]


def test_stage_batch_layout_and_args():
    lib = _lib.load()
    rng = np.random.default_rng(0)
    shapes = [(7, 3), (130, 41), (2, 1)]
    walkers = [_walker(rng, nt, K) for nt, K in shapes]
    src = np.array([[a.ctypes.data for a in w] for w in walkers], dtype=np.uint64)
    shape = np.array(shapes, dtype=np.int32)
    scale = np.array([[1.5, -0.25], [2.0, 0.0], [-1.0, 3.0]])
    tmpl = _lib.ModesumArgs(freq=0x1234, nf=999, grid_symmetric=1, caustic=1, k0=499)
    args = (_lib.ModesumArgs * 3)()
    total = ctypes.c_size_t(0)
    base = 1 << 40
    assert lib.efd_stage_batch(None, 0, base, 3, src.ctypes.data, shape.ctypes.data,
                               scale.ctypes.data, ctypes.byref(tmpl), args,
                               ctypes.byref(total)) == _lib.EFD_ERR_WORKSPACE
    need = total.value
    pin = np.zeros(need + 256, dtype=np.uint8)
    assert lib.efd_stage_batch(pin.ctypes.data, need - 1, base, 3, src.ctypes.data,
                               shape.ctypes.data, scale.ctypes.data, ctypes.byref(tmpl), args,
                               ctypes.byref(total)) == _lib.EFD_ERR_WORKSPACE
    assert lib.efd_stage_batch(pin.ctypes.data, pin.nbytes, base, 3, src.ctypes.data,
                               shape.ctypes.data, scale.ctypes.data, ctypes.byref(tmpl), args,
                               ctypes.byref(total)) == _lib.EFD_OK
    off = 0
    names = ("t", "phi_phi", "phi_r", "f_phi", "f_r", "amp", "m", "n", "ylm_p", "ylm_m")
    for i, w in enumerate(walkers):
        a = args[i]
        assert (a.nt, a.K) == shapes[i]
        assert (a.scale_re, a.scale_im) == tuple(scale[i])
        assert (a.freq, a.nf, a.grid_symmetric, a.caustic, a.k0) == (0x1234, 999, 1, 1, 499)
        for name, arr in zip(names, w):
            assert getattr(a, name) == base + off
            assert off % 256 == 0
            np.testing.assert_array_equal(pin[off:off + arr.nbytes], arr.reshape(-1).view(np.uint8))
            off = (off + arr.nbytes + 255) // 256 * 256
    assert off == need


def test_stage_batch_rejects_bad_input():
    lib = _lib.load()
    tmpl = _lib.ModesumArgs()
    args = (_lib.ModesumArgs * 1)()
    total = ctypes.c_size_t(0)
    src = np.zeros((1, 10), dtype=np.uint64)
    shape = np.array([[5, 2]], dtype=np.int32)
    scale = np.zeros((1, 2))
    pin = np.zeros(1 << 16, dtype=np.uint8)
    assert lib.efd_stage_batch(pin.ctypes.data, pin.nbytes, 0, 1, src.ctypes.data,
                               shape.ctypes.data, scale.ctypes.data, ctypes.byref(tmpl), args,
                               ctypes.byref(total)) == _lib.EFD_ERR_ARG      # NULL source
    shape[0] = (1, 2)
    assert lib.efd_stage_batch(pin.ctypes.data, pin.nbytes, 0, 1, src.ctypes.data,
                               shape.ctypes.data, scale.ctypes.data, ctypes.byref(tmpl), args,
                               ctypes.byref(total)) == _lib.EFD_ERR_ARG      # nt < 2
    assert lib.efd_stage_batch(pin.ctypes.data, pin.nbytes, 0, 0, src.ctypes.data,
                               shape.ctypes.data, scale.ctypes.data, ctypes.byref(tmpl), args,
                               ctypes.byref(total)) == _lib.EFD_ERR_ARG      # empty batch

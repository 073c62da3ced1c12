"""The windowed template model's injection provenance (fdutils.get_fd_waveform_fromFD.made_by),
on CPU tensors: the likelihood emits the windowed logL's per-bin data by its own arithmetic only
when the data stream is the very pair of channels a template call returned, unmodified
(emri_pe.py:276 injects data = gen(*truth)); anything else converts from (d0, d1).
"""
import weakref

import numpy as np
import torch

from emri_frequencydomainwaveforms_amd.fdutils import get_fd_waveform_fromFD


class _Model:
    """made_by's state as get_fd_waveform_fromFD.__call__ records it (no GPU needed)."""
    made_by = get_fd_waveform_fromFD.made_by

    def call(self, params, **kw):
        out = torch.zeros((2, 16), dtype=torch.complex128)
        chans = [out[0], out[1]]
        self._made = (np.asarray(params, dtype=np.float64).reshape(-1), dict(kw),
                      [weakref.ref(c) for c in chans], out._version)
        return chans


def test_made_by_same_channels():
    m = _Model()
    truth = np.arange(14, dtype=np.float64)
    chans = m.call(truth, T=2.0, dt=10.0)
    got = m.made_by(chans)
    assert got is not None
    np.testing.assert_array_equal(got[0], truth)
    assert got[1] == dict(T=2.0, dt=10.0)
    assert m.made_by(tuple(chans)) is not None


def test_made_by_rejects_other_data():
    m = _Model()
    chans = m.call(np.zeros(14))
    # copies, a single channel, the channels swapped, plain arrays: not this call's output
    assert m.made_by([c.clone() for c in chans]) is None
    assert m.made_by([chans[0]]) is None
    assert m.made_by([chans[1], chans[0]]) is None
    assert m.made_by([c.numpy() for c in chans]) is None
    assert m.made_by(None) is None
    # a later call's output replaces the record
    later = m.call(np.ones(14))
    assert m.made_by(chans) is None
    assert m.made_by(later) is not None
    assert _Model().made_by(later) is None   # a model that made nothing


def test_made_by_rejects_modified_channels():
    m = _Model()
    chans = m.call(np.zeros(14))
    chans[1][3] = 1.0 + 2.0j   # an in-place edit (noise added to the injection, say)
    assert m.made_by(chans) is None

"""Shared test helpers: synthetic multi-harmonic inputs of the hot path."""

import numpy as np

from emri_frequencydomainwaveforms_amd.amplitude import ModeSelector, SyntheticTeukolskyAmplitude
from emri_frequencydomainwaveforms_amd.constants import Gpc, MRSUN_SI, MTSUN_SI
from emri_frequencydomainwaveforms_amd.frequencies import get_fundamental_frequencies
from emri_frequencydomainwaveforms_amd.summation import fd_grid
from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
from emri_frequencydomainwaveforms_amd.ylm import GetYlms


def source_inputs(M=3e5, mu=10.0, e0=0.35, T=0.02, dt=20.0, eps=1e-2, p0=None, modes=None,
                  theta=np.pi / 3, phi=-np.pi / 2, dist=1.0):
    """Stand-in trajectory + amplitudes + Ylm for one source; returns a dict of hot-path inputs."""
    traj = EMRIInspiral()
    if p0 is None:
        p0 = get_p_at_t(traj, 0.99 * T, [M, mu, 0.0, e0, 1.0])
    t, p, e, x, pp, pt, pr = traj(M, mu, 0.0, p0, e0, 1.0, T=T)
    amp = SyntheticTeukolskyAmplitude()
    yg = GetYlms(assume_positive_m=True)
    A = amp(p, e)
    ylms = yg(amp.l_arr, amp.m_arr, theta, phi)
    Kall = amp.num_teuk_modes
    if modes is None:
        keep = ModeSelector(amp.m0mask)(A, ylms, None, eps=eps)
    else:
        keep = np.array([amp.lmn_indices[tuple(md)] for md in modes])
    op, _, orr = get_fundamental_frequencies(0.0, p, e, 0.0)
    return dict(t=t, amp=A[:, keep].T.copy(), phi_phi=pp, phi_r=pr,
                f_phi=op / (2 * np.pi * M * MTSUN_SI), f_r=orr / (2 * np.pi * M * MTSUN_SI),
                m=amp.m_arr[keep].astype(np.int32), n=amp.n_arr[keep].astype(np.int32),
                l=amp.l_arr[keep].astype(np.int32),
                ylm_p=ylms[:Kall][keep], ylm_m=ylms[Kall:][keep],
                prefactor=mu * MRSUN_SI / (dist * Gpc), freq=fd_grid(T, dt), p=p, e=e, M=M,
                mu=mu, p0=p0, e0=e0, T=T, dt=dt)

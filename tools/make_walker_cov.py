"""Derive the emri_pe.py walker-start covariance (6 x 6) from the reference's covariance.npy.

    python tools/make_walker_cov.py        # writes emri_frequencydomainwaveforms_amd/data/walker_cov.npy

emri_pe.py:440-444 starts the walkers at multivariate_normal(truth, cov) with
cov = np.cov(np.load("covariance.npy"), rowvar=False) / (2.4 * ndim), ndim = 6. The 34240 x 6
chain (1.6 MB) is not shipped to the GPU box; its 6 x 6 sample covariance (undivided) is, as
data. Run here, where /root/reference exists.
"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
chain = np.load("/root/reference/covariance.npy", allow_pickle=False)
cov = np.cov(chain, rowvar=False)
out = os.path.join(ROOT, "emri_frequencydomainwaveforms_amd", "data", "walker_cov.npy")
np.save(out, cov)
print(out, cov.shape, np.sqrt(np.diag(cov / (2.4 * 6))))

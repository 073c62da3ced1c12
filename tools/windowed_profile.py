"""The windowed likelihood at test.sh's shape (Tobs 4 yr, M 3.67e6, 12.6 M bins, Hann window;
emri_pe.py:259-263, FDutils.py:66-101) for kernel-trace and PMC attribution (GPU box).

    python tools/windowed_profile.py [STEPS]

Device path (host upstream memoised after the warm-up), STEPS timed half-steps of 8 walkers
between two marker launches (efd_polarizations on a 3-bin grid: k_polarizations, which the
windowed path never launches otherwise), so a rocprofv3 --kernel-trace CSV of this command can
be cut to the timed region (tools/windowed_summary.py). Prints one JSON line: ms per half-step
and a hash of the batch's logL (variants that must agree bitwise compare it).
"""

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def marker(lib, buf, st):
    from emri_frequencydomainwaveforms_amd import _lib
    _lib.check(lib.efd_polarizations(buf[0].data_ptr(), 3, 1, buf[1].data_ptr(),
                                     buf[2].data_ptr(), st), "efd_polarizations", lib)


def main():
    import torch
    from emri_frequencydomainwaveforms_amd import _lib, pe
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    s = pe.setup(Tobs=4.0, dt=10.0, eps=1e-2, M=3670041.7362535275, mu=292.0583167470244,
                 e0=0.5794130830706371, nwalkers=16, ntemps=1, window_flag=True)
    like = s.like
    batch = s.half_steps()[0]
    like(batch, **s.kwargs)
    memo = pe.MemoizedUpstream(s.few.waveform_generator)
    like(batch, **s.kwargs)
    like(batch, **s.kwargs)
    lib = _lib.load()
    buf = [torch.zeros(12, dtype=torch.float64, device="cuda") for _ in range(3)]
    st = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    marker(lib, buf, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        like(batch, **s.kwargs)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    marker(lib, buf, st)
    torch.cuda.synchronize()
    ll = np.asarray(like(batch, **s.kwargs), dtype=np.float64)
    memo.remove()
    print(json.dumps({"config": "test.sh windowed, 8 walkers per half-step", "steps": steps,
                      "ms_per_half_step": el / steps * 1e3, "N_f": s.info["N_f"],
                      "loglikes_per_s": len(batch) * steps / el,
                      "ll_sha16": hashlib.sha256(ll.tobytes()).hexdigest()[:16]}))


if __name__ == "__main__":
    main()

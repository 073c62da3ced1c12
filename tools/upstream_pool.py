"""Parallel efficiency of the host upstream at config 4 (GPU box host): one walker's
_upstream on the calling thread (1 and 2 OpenMP threads) against the pool's prefetch of 8
walkers (2 threads each and 1), and 8 plain threads running _upstream with 1 thread each.
Medians of REPS, ms.   python tools/upstream_pool.py [REPS]
"""

import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from emri_frequencydomainwaveforms_amd import _lib, hostcpu
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    from emri_frequencydomainwaveforms_amd.waveform import FastSchwarzschildEccentricFlux
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    share = hostcpu.pin()
    M, mu, e0 = 1e6, 10.0, 0.35
    p0 = float(get_p_at_t(EMRIInspiral(), 2.0 * 0.99, [M, mu, 0.0, e0, 1.0]))
    g = FastSchwarzschildEccentricFlux()
    rng = np.random.default_rng(3)
    calls = [(M * (1 + 1e-4 * rng.normal()), mu, p0 + 1e-3 * rng.normal(), e0, 0.8, 1.2, 1.0,
              0.1, 0.2, 2.0, 1e-2) for _ in range(8)]
    lib = _lib.load()
    out = {"cores": len(share)}

    def med(f):
        f()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            f()
            ts.append((time.perf_counter() - t0) * 1e3)
        return float(np.median(ts))

    for nth in (1, 2):
        lib.efd_host_set_threads(nth)
        out[f"one_walker_{nth}thr"] = med(lambda: g._upstream(*calls[0], None, True))
    out["one_walker_traj"] = med(lambda: g.inspiral_generator.with_frequencies(
        M, mu, 0.0, p0, e0, 1.0, Phi_phi0=0.1, Phi_r0=0.2, T=2.0))

    def pool8():
        g._prefetched.clear()
        g._prefetched_bytes = 0
        g.prefetch(calls)
    out["pool8_default"] = med(pool8)
    os.environ["EFD_PREFETCH_SPLIT"] = "0"
    out["pool8_1thr"] = med(pool8)
    os.environ.pop("EFD_PREFETCH_SPLIT")

    def threads8():
        def w(c):
            lib.efd_host_set_threads(1)
            g._upstream(*c, None, True)
        ts = [threading.Thread(target=w, args=(c,)) for c in calls]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    out["threads8_1thr"] = med(threads8)

    def traj8():
        def w(c):
            g.inspiral_generator.with_frequencies(c[0], c[1], 0.0, c[2], c[3], 1.0,
                                                  Phi_phi0=0.1, Phi_r0=0.2, T=2.0)
        ts = [threading.Thread(target=w, args=(c,)) for c in calls]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    out["threads8_traj_only"] = med(traj8)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

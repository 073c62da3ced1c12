"""The host upstream of one test.sh walker (windowed config: Tobs 4, M 3.67e6, eps 1e-2) by
OpenMP thread count, on the calling thread: median ms of REPS calls per count.

    python tools/upstream_threads.py [REPS]
"""

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from emri_frequencydomainwaveforms_amd import _lib, hostcpu
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    from emri_frequencydomainwaveforms_amd.waveform import FastSchwarzschildEccentricFlux
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    hostcpu.pin()
    M, mu, e0 = 3670041.7362535275, 292.0583167470244, 0.5794130830706371
    p0 = float(get_p_at_t(EMRIInspiral(), 4.0 * 0.99, [M, mu, 0.0, e0, 1.0]))
    g = FastSchwarzschildEccentricFlux()
    args = (M, mu, p0, e0, 0.8, 1.2, 1.0, 0.1, 0.2, 4.0, 1e-2, None, True)
    lib = _lib.load()
    out = {"host_threads": hostcpu.threads()}
    for nth in (1, 2, 4, 8, 16):
        lib.efd_host_set_threads(nth)
        for _ in range(2):
            g._upstream(*args)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            d = g._upstream(*args)
            ts.append((time.perf_counter() - t0) * 1e3)
        out[f"ms_{nth}"] = float(np.median(ts))
    t0 = time.perf_counter()
    for _ in range(reps):
        g.inspiral_generator.with_frequencies(M, mu, 0.0, p0, e0, 1.0, Phi_phi0=0.1, Phi_r0=0.2,
                                              T=4.0)
    out["trajectory_ms"] = (time.perf_counter() - t0) / reps * 1e3
    out["N_t"], out["K"] = len(d["t"]), len(d["m"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Host thread scaling on this box (the upstream pool's ceiling).

    python tools/host_scaling.py

For each job -- numpy sin over a 200k array (releases the GIL), the native stand-in trajectory
(efd_host_trajectory), the native mode selection (efd_host_modes, config 5's source), and one
config-5 walker's whole upstream (_upstream) -- the time of 16 calls on one thread against 8
calls on each of N threads (N = 2, 4, 8, 16): speedup = N x t(1 call) / t(N threads, 8 calls
each). Also the affinity set, the cgroup's cpuset and CPU quota. One JSON line.
"""

import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def read(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


def scaling(fn, counts=(2, 4, 8, 16), per=8):
    fn()
    t0 = time.perf_counter()
    for _ in range(2 * per):
        fn()
    one = (time.perf_counter() - t0) / (2 * per)
    out = {"ms_per_call": one * 1e3}
    for n in counts:
        def w():
            for _ in range(per):
                fn()
        ts = [threading.Thread(target=w) for _ in range(n)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        out[f"speedup_{n}"] = n * per * one / (time.perf_counter() - t0)
    return out


def main():
    from emri_frequencydomainwaveforms_amd import _lib, hostcpu
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    from emri_frequencydomainwaveforms_amd.waveform import FastSchwarzschildEccentricFlux
    lib = _lib.load()
    res = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
           "cgroup_cpuset": read("/sys/fs/cgroup/cpuset.cpus.effective")
           or read("/sys/fs/cgroup/cpuset/cpuset.effective_cpus"),
           "cgroup_cpu_max": read("/sys/fs/cgroup/cpu.max")
           or read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"),
           "host_threads": hostcpu.threads(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    x = np.random.rand(200000)
    res["numpy_sin"] = scaling(lambda: np.sin(x))
    M, mu, e0, T = 1e6, 10.0, 0.35, 4.0
    p0 = float(get_p_at_t(EMRIInspiral(), T * 0.99, [M, mu, 0.0, e0, 1.0]))
    L = 1000

    def traj():
        bufs = np.empty((7, L))
        n = ctypes.c_int32(0)
        p = lambda i: bufs[i].ctypes.data  # noqa: E731
        lib.efd_host_trajectory(M, mu, p0, e0, 0.1, 0.2, T, 1e-10, 1e-10, L, p(0), p(1), p(2),
                                p(3), p(4), p(5), p(6), ctypes.byref(n))
    res["trajectory"] = scaling(traj)
    g = FastSchwarzschildEccentricFlux()
    lib.efd_host_set_threads(1)
    pe = g.inspiral_generator.with_frequencies(M, mu, 0.0, p0, e0, 1.0, Phi_phi0=0.1,
                                               Phi_r0=0.2, T=T)
    yl = g._ylms(0.8, 1.2)

    def sel():
        lib.efd_host_set_threads(1)
        g.amplitude_generator.select(pe[1], pe[2], yl, 1e-2, lib=lib)
    res["mode_selection"] = scaling(sel)

    def up():
        lib.efd_host_set_threads(1)
        g._upstream(M, mu, p0, e0, 0.8, 1.2, 1.0, 0.1, 0.2, T, 1e-2, None, True)
    res["upstream"] = scaling(up)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

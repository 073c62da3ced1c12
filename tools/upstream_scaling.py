"""How the host stand-in upstream (trajectory + amplitudes + selection, C++) scales over the
upstream thread pool for a walker half-step (config 4: 8 walkers, Tobs 2 yr, eps 1e-2).

    python tools/upstream_scaling.py [B]

Prints one JSON line: the serial time per walker (1 and all OpenMP threads), the pooled
prefetch of B walkers with and without the per-walker OpenMP split, and each walker's start /
end inside the pooled call (relative to its start), so serialisation shows up as staggered
windows. Host only (no GPU needed)."""

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
    from emri_frequencydomainwaveforms_amd import waveform as wf
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    g = wf.FastSchwarzschildEccentricFlux(
        sum_kwargs=dict(pad_output=True, output_type="fd", odd_len=True))
    T, eps, M, mu, e0 = 2.0, 1e-2, 1e6, 10.0, 0.35
    p0 = float(get_p_at_t(EMRIInspiral(), 0.99 * T, [M, mu, 0.0, e0, 1.0]))
    rng = np.random.default_rng(1)

    def calls():
        return [(M * (1 + 1e-4 * rng.normal()), mu * (1 + 1e-4 * rng.normal()),
                 p0 + 1e-4 * rng.normal(), e0 + 1e-4 * rng.normal(), 1.0, 0.5, 2.45, 1.0, 2.0,
                 T, eps) for _ in range(B)]
    lib = _lib.load()
    out = {"B": B, "pool_threads": wf._pool()._max_workers, "host_share": len(hostcpu.pin())}
    for th in (1, out["pool_threads"]):
        lib.efd_host_set_threads(th)
        g.prepare(*calls()[0])
        ts = []
        for _ in range(3):
            cs = calls()
            t0 = time.perf_counter()
            for c in cs:
                g.prepare(*c)
            ts.append((time.perf_counter() - t0) / B)
        out[f"serial_ms_per_walker_omp{th}"] = min(ts) * 1e3
    # pooled, with per-walker windows
    orig = g.prepare
    win = []
    lock = threading.Lock()

    def timed(*a, **k):
        t0 = time.perf_counter()
        r = orig(*a, **k)
        with lock:
            win.append((t0, time.perf_counter(), threading.get_ident()))
        return r
    for split in ("0", "1"):
        os.environ["EFD_PREFETCH_SPLIT"] = split
        ts = []
        for rep in range(5):
            cs = calls()
            win.clear()
            g.prepare = timed
            t0 = time.perf_counter()
            g.prefetch(cs)
            el = time.perf_counter() - t0
            g.prepare = orig
            ts.append(el)
            for c in cs:
                g.prepare(*c)
            if rep == 4:
                out[f"windows_split{split}_ms"] = [
                    [round((a - t0) * 1e3, 3), round((b - t0) * 1e3, 3)] for a, b, _ in
                    sorted(win)]
        out[f"prefetch_split{split}_ms"] = float(np.median(ts)) * 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Where a likelihood half-step's time goes with the host upstream in the loop.

    python tools/api_trace.py config5|config4|config4,config5 [CALLS]

Sets up emri_pe's likelihood as tools/configs.py does and times CALLS get_ll calls over the first
half-step's walkers with the stand-in upstream recomputed each call. Each walker's upstream
(_upstream: start, end, thread) and each prepare() lookup (hit in flight / held / recomputed,
how long the main thread waited) are recorded. Per call: wall ms, the pool's busy share
(sum of upstream durations / (threads x wall)), the mean upstream ms in the pool, the main
thread's waits, and recomputed misses. One JSON line per call, then a summary line.
"""

import gc
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "config5"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    gc.callbacks.append(_gc_cb)
    for w in which.split(","):   # several in one process (tools/configs.py's order)
        trace(w, calls)


GC = []       # (generation, seconds) of every collection
_gc_t0 = [0.0]


def _gc_cb(phase, info):
    if phase == "start":
        _gc_t0[0] = time.perf_counter()
    else:
        GC.append((info["generation"], time.perf_counter() - _gc_t0[0]))


def trace(which, calls):
    import torch
    from emri_frequencydomainwaveforms_amd import pe
    from emri_frequencydomainwaveforms_amd.waveform import _pool
    cfg = dict(config4=dict(Tobs=2.0, eps=1e-2, nwalkers=16),
               config5=dict(Tobs=4.0, eps=1e-2, nwalkers=128, downsample=100))[which]
    st = pe.setup(**cfg)
    walkers = st.transform.both_transforms(st.half_steps()[0])
    like, kw = st.like, st.kwargs
    g = st.few.waveform_generator
    rec, lock = [], threading.Lock()
    orig_up, orig_prep = g._upstream, g.prepare

    def up(*a, **k):
        t0 = time.perf_counter()
        r = orig_up(*a, **k)
        with lock:
            rec.append(("up", threading.get_ident(), t0, time.perf_counter()))
        return r

    def prep(*a, **k):
        t0 = time.perf_counter()
        inflight = bool(g._inflight)
        r = orig_prep(*a, **k)
        with lock:
            rec.append(("prep", inflight, t0, time.perf_counter()))
        return r
    g._upstream, g.prepare = up, prep
    nthr = _pool()._max_workers
    for _ in range(3):
        like.get_ll(walkers, **kw)
    torch.cuda.synchronize()
    out = []
    if os.environ.get("TRACE_GC_FREEZE"):
        gc.freeze()
    print(json.dumps({"setup": which, "gc_tracked_objects": len(gc.get_objects()),
                      "gc_frozen": gc.get_freeze_count(), "gc_counts": gc.get_count()}), flush=True)
    for c in range(calls):
        rec.clear()
        GC.clear()
        t0 = time.perf_counter()
        like.get_ll(walkers, **kw)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ups = [r for r in rec if r[0] == "up"]
        main_ups = [r for r in ups if r[1] == threading.main_thread().ident]
        preps = [r for r in rec if r[0] == "prep"]
        busy = sum(r[3] - r[2] for r in ups)
        line = {"call": c, "walkers": len(walkers), "wall_ms": wall * 1e3,
                "pool_threads": nthr, "upstreams": len(ups),
                "upstream_mean_ms": 1e3 * busy / max(1, len(ups)),
                "pool_busy_share": busy / (nthr * wall),
                "recomputed_on_main": len(main_ups),
                "main_wait_in_prepare_ms": 1e3 * sum(r[3] - r[2] for r in preps),
                "last_upstream_end_ms": 1e3 * (max(r[3] for r in ups) - t0) if ups else None,
                "first_prepare_ms": 1e3 * (min(r[2] for r in preps) - t0) if preps else None,
                "gc": [[g, round(1e3 * d, 3)] for g, d in GC]}
        out.append(line)
        print(json.dumps(line), flush=True)
    w = [x["wall_ms"] for x in out]
    print(json.dumps({"summary": which, "wall_ms_median": float(np.median(w)),
                      "wall_ms_min": min(w), "wall_ms_max": max(w),
                      "loglikes_per_s_median": len(walkers) / (float(np.median(w)) * 1e-3)}))


if __name__ == "__main__":
    main()

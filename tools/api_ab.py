"""Paired A/B of the likelihood API path's host options at configs 4 and 5 (GPU box).

    python tools/api_ab.py ROUNDS REPS

One process, one emri_pe setup per configuration (tools/configs.py's), the host stand-in
upstream in the loop (not memoised). Each round runs every mode in rotated order, REPS half-steps
each, and records ms per half-step; prints one JSON line per configuration with the per-mode
medians, the ratios to the first mode and every round's values. Modes: the upstream prefetch
asynchronous (EFD_PREFETCH_ASYNC, read per call) or waited for, and the fused group size
(Likelihood.FUSED_GROUP on the instance). The logL of every mode must equal the first's bitwise.
"""

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

MODES = [("async_g16", "1", 16), ("sync_g16", "0", 16), ("async_g4", "1", 4), ("sync_g4", "0", 4),
         ("async_g8", "1", 8)]


def main():
    import torch
    from configs import _likelihood_setup
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    for name, T, eps, ds, nw in (("config4", 2.0, 1e-2, 1, 16), ("config5", 4.0, 1e-2, 100, 128)):
        few, like, walkers, kw, nbins = _likelihood_setup(T, eps, ds, nw)
        like.fused_likelihood = True
        ref = None
        times = {m[0]: [] for m in MODES}
        for r in range(rounds):
            order = MODES[r % len(MODES):] + MODES[:r % len(MODES)]
            for mname, asyn, group in order:
                os.environ["EFD_PREFETCH_ASYNC"] = asyn
                like.FUSED_GROUP = group
                ll = like.get_ll(walkers, **kw)   # warm-up of this mode's group shapes
                torch.cuda.synchronize()
                if ref is None:
                    ref = ll
                assert np.array_equal(ll, ref), mname
                t0 = time.perf_counter()
                for _ in range(reps):
                    like.get_ll(walkers, **kw)
                torch.cuda.synchronize()
                times[mname].append((time.perf_counter() - t0) / reps * 1e3)
        med = {k: float(np.median(v)) for k, v in times.items()}
        base = med[MODES[0][0]]
        print(json.dumps({"config": name, "walkers_per_half_step": len(walkers),
                          "ms_per_half_step_median": med,
                          "loglikes_per_s_median": {k: len(walkers) / v * 1e3
                                                    for k, v in med.items()},
                          "ratio_to_" + MODES[0][0]: {k: base / v for k, v in med.items()},
                          "rounds": times}), flush=True)
    os.environ.pop("EFD_PREFETCH_ASYNC", None)


if __name__ == "__main__":
    main()

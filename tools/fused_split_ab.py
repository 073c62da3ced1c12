"""Paired A/B of Likelihood.FUSED_SPLIT_LAST (the batch's last fused group in two halves) on the
device rate of configs 4 and 5 (host upstream memoised), one process per configuration, rotated
rounds; the logL of both modes must agree bitwise.   python tools/fused_split_ab.py ROUNDS REPS
"""

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from configs import _likelihood_setup
    from emri_frequencydomainwaveforms_amd.pe import MemoizedUpstream
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    for name, T, ds, nw in (("config5", 4.0, 100, 128), ("config4", 2.0, None, 16)):
        few, like, walkers, kw, nbins = _likelihood_setup(T, 1e-2, ds, nw)
        like.fused_likelihood = True
        MemoizedUpstream(few.waveform_generator)
        ref = None
        times = {False: [], True: []}
        for r in range(rounds):
            for mode in ((False, True) if r % 2 == 0 else (True, False)):
                like.FUSED_SPLIT_LAST = mode
                ll = like.get_ll(walkers, **kw)
                torch.cuda.synchronize()
                if ref is None:
                    ref = ll
                assert np.array_equal(ll, ref), mode
                t0 = time.perf_counter()
                for _ in range(reps):
                    like.get_ll(walkers, **kw)
                torch.cuda.synchronize()
                times[mode].append((time.perf_counter() - t0) / reps * 1e3)
        med = {str(k): float(np.median(v)) for k, v in times.items()}
        print(json.dumps({"config": name, "walkers": len(walkers), "ms_per_half_step": med,
                          "device_loglikes_per_s": {k: len(walkers) / v * 1e3
                                                    for k, v in med.items()},
                          "rounds": {str(k): v for k, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()

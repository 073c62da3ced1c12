"""Host-side cost of the pipelined likelihood path (config 5 shape) under cProfile.

    python tools/host_overhead.py [--config 5] [--reps 3]

Runs Likelihood.get_ll over config 5's walker batch with the host upstream memoised (as
tools/configs.py's "device" rate) and prints the wall time per walker, the host time spent
inside get_ll before the final synchronisation, and the top cProfile entries, to tell a
host-launch-bound batch from a device-bound one.
"""

import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="5", choices=["4", "5"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--slots", type=int, default=4)
    args = ap.parse_args()
    import torch
    import configs
    if args.config == "5":
        few, like, walkers, kw, nb = configs._likelihood_setup(4.0, 1e-2, 100, 128)
    else:
        few, like, walkers, kw, nb = configs._likelihood_setup(2.0, 1e-2, None, 16)
    like.num_streams = args.slots
    configs.PrepareCache(few.waveform_generator)
    like.get_ll(walkers, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        like.get_ll(walkers, **kw)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.reps
    # host time up to the batch's synchronisation: time the loop with the final wait stubbed
    fused = getattr(like, "_fused", None)
    P = fused["prep"] if fused else like._pipe
    real_wait = P.wait
    P.wait = lambda: None
    real_sync = torch.cuda.Stream.synchronize
    if fused:   # the fused path also synchronises its sum stream
        torch.cuda.Stream.synchronize = lambda self: None
    t0 = time.perf_counter()
    like.get_ll(walkers, **kw)
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    P.wait = real_wait
    torch.cuda.Stream.synchronize = real_sync
    pr = cProfile.Profile()
    pr.enable()
    like.get_ll(walkers, **kw)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(os.environ.get("HO_SORT", "tottime")).print_stats(int(os.environ.get("HO_N", "18")))
    B = len(walkers)
    print(json.dumps({"config": args.config, "walkers": B, "slots": args.slots,
                      "fused_likelihood": bool(fused),
                      "wall_ms_per_walker": wall / B * 1e3,
                      "host_ms_per_walker_before_sync": host / B * 1e3}))
    print(s.getvalue())


if __name__ == "__main__":
    main()

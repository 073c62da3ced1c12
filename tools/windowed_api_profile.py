"""Where the windowed likelihood's API half-step spends its host time (GPU box).

    python tools/windowed_api_profile.py [REPS] [windowed|config4]

test.sh's windowed setup (or config 4's; tools/configs.py's), the host stand-in upstream in the loop: the
upstream of one walker on the calling thread, the pool's prefetch of the 8 walkers (wait=True),
then cProfile over REPS get_ll calls (top functions by cumulative time to stderr) and the
mean ms per half-step as one JSON line.
"""

import cProfile
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from configs import _likelihood_setup
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    which = sys.argv[2] if len(sys.argv) > 2 else "windowed"
    if which == "config4":
        few, like, walkers, kw, nbins = _likelihood_setup(2.0, 1e-2, None, 16)
        like.fused_likelihood = True
    else:
        few, like, walkers, kw, nbins = _likelihood_setup(
            4.0, 1e-2, None, 16, M=3670041.7362535275, mu=292.0583167470244,
            e0=0.5794130830706371, window_flag=True)
    for _ in range(3):
        like.get_ll(walkers, **kw)
    torch.cuda.synchronize()
    tm = like.template_model
    gen = getattr(tm, "waveform_generator", tm)
    up = getattr(gen, "_upstream", None)
    out = {"walkers": len(walkers)}
    # the pool's prefetch of the batch, waited for
    if hasattr(tm, "prefetch"):
        t0 = time.perf_counter()
        tm.prefetch(walkers, wait=True, **kw)
        out["prefetch_wait_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    for _ in range(reps):
        like.get_ll(walkers, **kw)
    torch.cuda.synchronize()
    out["api_ms_per_half_step"] = (time.perf_counter() - t0) / reps * 1e3
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(reps):
        like.get_ll(walkers, **kw)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(45)
    out["upstream_attr"] = up is not None
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Per-tile work of the fused sparse sum at config 4 / 5 (a -DEFD_EXP build: record evaluations
per tile and each tile's wall-clock duration, the last writer's), to see what sets the sum.

    EFD_LIB=exp/libemrifd_exp.so python tools/sparse_tiles.py config4

(build the variant first: python tools/exp_variants.py build exp:-DEFD_EXP). Prints one JSON
line: the visited tiles, the duration distribution (us; s_memrealtime ticks of 10 ns), the
slowest tiles with their evaluation counts, and the evaluation-count distribution.
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from emri_frequencydomainwaveforms_amd import _lib, pe  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config4"
s = pe.setup(**bench.LIKE_CONFIGS[cfg])
batches = s.half_steps()
for i in range(4):
    s.like(batches[i % len(batches)], **s.kwargs)
torch.cuda.synchronize()
lib = _lib.load()
if not hasattr(lib, "efd_exp_tiles"):
    raise SystemExit("not a -DEFD_EXP build (set EFD_LIB)")
lib.efd_exp_tiles.restype = ctypes.c_int
lib.efd_exp_tiles.argtypes = [ctypes.c_void_p, ctypes.c_void_p]   # (pointers, not C ints)
ev = np.zeros(16384, dtype=np.uint32)
clk = np.zeros(16384, dtype=np.uint64)
lib.efd_exp_tiles(ev.ctypes.data, clk.ctypes.data)
dur = (clk & np.uint64(0xffffffff)).astype(np.float64) * 0.01   # us
seen = np.nonzero(dur > 0)[0]
d = dur[seen]
order = seen[np.argsort(-dur[seen])][:12]
out = {"config": cfg, "tiles_timed": int(seen.size),
       "us": {"max": float(d.max()), "p90": float(np.percentile(d, 90)),
              "median": float(np.median(d)), "mean": float(d.mean())},
       "slowest": [{"tile": int(t), "us": round(float(dur[t]), 2), "evals": int(ev[t])}
                   for t in order],
       "evals_per_tile": {"max": int(ev.max()), "median_nonzero": float(np.median(ev[ev > 0]))
                          if (ev > 0).any() else 0.0, "tiles_nonzero": int((ev > 0).sum())}}
print(json.dumps(out))

"""GPU box: the tile extent of configs 4 / 5's walkers (the union [lane_lo, lane_hi) of the
segments' lane ranges that k_segment_compact writes into each workspace header), against the
grid's tile count.   python tools/tile_extent.py"""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from emri_frequencydomainwaveforms_amd import pe
TL = 768   # lanes per tile: emrifd.hip's TILE * BPL (512 up to round 3)
for cfg in (dict(Tobs=2.0, dt=10.0, eps=1e-2, nwalkers=16, ntemps=1),
            dict(Tobs=4.0, dt=10.0, eps=1e-2, nwalkers=128, ntemps=1, downsample=100)):
    s = pe.setup(**cfg)
    b = s.half_steps()[0]
    s.like(b, **s.kwargs)
    torch.cuda.synchronize()
    B = s.like._fused["prep"]
    G = B.groups[0]
    for eng in G["engines"][:4]:
        h = eng._ws[:64].cpu().numpy().view(np.int32)
        a = eng._last_args
        nl = (a.nf + 1) // 2
        print(cfg["Tobs"], "nf", a.nf, "K", a.K, "nt", a.nt, "lanes", nl, "ntiles", -(-nl // TL),
              "lane_lo", h[10], "lane_hi", h[11], "tiles_hit", (h[11] - 1) // TL - h[10] // TL + 1,
              flush=True)

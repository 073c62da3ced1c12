"""Which objects of a likelihood setup are left to the cyclic garbage collector (VERDICT r5 item 5:
a generation-2 collection that frees a dropped setup's cycles stalled a later API call by
~130 ms, tools/api_trace.py).

    python tools/gc_cycles.py [config4|config5]

Sets up emri_pe's likelihood (tools/configs.py's way), runs two get_ll calls, drops every
reference, and collects with gc.DEBUG_SAVEALL: prints the collection's time, the count of
unreachable objects by type, and for the few types that own device or host resources the
referrers that close their cycles.
"""

import collections
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from emri_frequencydomainwaveforms_amd import pe
    which = sys.argv[1] if len(sys.argv) > 1 else "config4"
    cfg = dict(config4=dict(Tobs=2.0, eps=1e-2, nwalkers=16),
               config5=dict(Tobs=4.0, eps=1e-2, nwalkers=128, downsample=100))[which]
    gc.collect()
    st = pe.setup(**cfg)
    walkers = st.transform.both_transforms(st.half_steps()[0])
    for _ in range(2):
        st.like.get_ll(walkers, **st.kwargs)
    torch.cuda.synchronize()
    gc.collect()
    # a full collection with the setup alive: its traversal cost, and the largest containers
    # it walks (len > 10k) with the attribute names that hold them
    t0 = time.perf_counter()
    gc.collect()
    full_ms = (time.perf_counter() - t0) * 1e3
    big = []
    for o in gc.get_objects():
        try:
            n = len(o)
        except Exception:
            continue
        if n > 10000 and isinstance(o, (list, dict, set, tuple, collections.deque)):
            holders = []
            for r in gc.get_referrers(o)[:6]:
                if isinstance(r, dict):
                    holders += [k for k, v in r.items() if v is o][:2]
                else:
                    holders.append(type(r).__qualname__)
            sample = type(next(iter(o.values() if isinstance(o, dict) else o))).__qualname__
            big.append((type(o).__qualname__, n, sample, holders[:6]))
    big.sort(key=lambda t: -t[1])
    print(json.dumps({"config": which, "full_collect_ms": full_ms,
                      "tracked": len(gc.get_objects()), "big_containers": big[:25]}), flush=True)
    gc.set_debug(gc.DEBUG_SAVEALL)
    del st, walkers
    t0 = time.perf_counter()
    n = gc.collect()
    dt = time.perf_counter() - t0
    gc.set_debug(0)
    kinds = collections.Counter(type(o).__module__ + "." + type(o).__qualname__ for o in gc.garbage)
    ours = [o for o in gc.garbage
            if type(o).__module__.startswith("emri_frequencydomainwaveforms_amd")]
    print(json.dumps({"config": which, "collected": n, "collect_ms": dt * 1e3,
                      "garbage_types": kinds.most_common(40),
                      "package_objects": sorted({type(o).__qualname__ for o in ours})}),
          flush=True)
    # the attributes of our objects that point back into the garbage (cycle edges)
    ids = {id(o) for o in gc.garbage}
    edges = collections.Counter()
    for o in ours:
        d = getattr(o, "__dict__", {})
        for k, v in d.items():
            if id(v) in ids:
                edges[f"{type(o).__qualname__}.{k} -> {type(v).__qualname__}"] += 1
    print(json.dumps({"edges": edges.most_common(60)}), flush=True)
    gc.garbage.clear()


if __name__ == "__main__":
    main()

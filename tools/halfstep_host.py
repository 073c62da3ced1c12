"""Host time of one fused-likelihood half-step by phase (config 4 / 5, memoised upstream).

    python tools/halfstep_host.py config4|config5 [python]

("python": the groups' host steps in Python, Likelihood.FUSED_NATIVE_GROUP = False)

Runs bench.py's likelihood setup (pe.setup) with a copy of Likelihood._get_ll_fused that adds
timers between its phases (grid check and prefetch, stream setup, submit_batch, flush,
sum_loglike and events, the final synchronisation, the status check) and prints microseconds
per half-step. Keep the copy in step with likelihood.py when that changes.
"""
import sys, time, json, collections, ctypes
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import numpy as np, torch
import bench
from emri_frequencydomainwaveforms_amd import pe, likelihood as L
from emri_frequencydomainwaveforms_amd.summation import BatchPreparer
cfg = bench.LIKE_CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "config5"]
if "python" in sys.argv[2:]:
    L.Likelihood.FUSED_NATIVE_GROUP = False
s = pe.setup(**cfg)
batches = s.half_steps()
memo = pe.MemoizedUpstream(s.few.waveform_generator)
acc = collections.defaultdict(float)
pc = time.perf_counter
def fused(self, tm, params, args, kwargs, out):
    t0 = pc()
    if not self._fused_grid_ok(tm, kwargs):
        return False
    if hasattr(tm, "prefetch"):
        tm.prefetch(params, *args, **kwargs)
    t1 = pc(); acc["grid+prefetch"] += t1 - t0
    n = len(params)
    ngroups = -(-n // self.FUSED_GROUP)
    G = -(-n // ngroups)
    caustic = "uniform"
    F = self._fused
    if F is None:
        F = self._fused = dict(prep=BatchPreparer(max(G, self.FUSED_GROUP), self.FUSED_DEPTH, caustic=caustic, device=self.device), stream=torch.cuda.Stream(self.device))
    B, s_sum = F["prep"], F["stream"]
    if "order" not in F:
        vp = ctypes.c_void_p
        F["order"] = (vp * (len(B.groups) + 1))(*[g["stream"].cuda_stream for g in B.groups],
                                                 s_sum.cuda_stream)
        F["gst"] = [g["stream"].cuda_stream for g in B.groups]
        F["sum1"] = (vp * 1)(s_sum.cuda_stream)
        F["ev"] = [torch.cuda.Event() for _ in B.groups]
    lib = B.lib
    cur = torch.cuda.current_stream(self.device)
    key = ("ord", B._next, min(ngroups, len(B.groups)))
    arr = F.get(key)
    if arr is None:
        gis = [(key[1] + k) % len(B.groups) for k in range(key[2])]
        arr = F[key] = (ctypes.c_void_p * len(gis))(*[F["gst"][g] for g in gis])
    lib.efd_stream_order(cur.cuda_stream, arr, len(arr))
    pin = F.get("pin")
    if pin is None or pin.numel() < n:
        pin = F["pin"] = torch.empty(max(n, 64), dtype=torch.float64, pin_memory=True)
    t2 = pc(); acc["setup"] += t2 - t1
    batch = tm.submit_batch
    used = []
    for g0 in range(0, n, G):
        ta = pc()
        batch(B, params[g0:g0 + G], *args, **kwargs)
        tb = pc(); acc["submit_batch"] += tb - ta
        if self.FUSED_NATIVE_GROUP:
            # one native call per group (efd_fused_group), as Likelihood._get_ll_fused
            p0 = B._pending[0]
            sst = B.groups[B._next]["stream"]
            tcon = self._tile_constants({"freq": p0[1], "k0": p0[4]}, sst, F)
            used.append(B.flush_loglike(self._d, self._w_templ, out, tile_const=tcon,
                                        out_off=g0))
            acc["flush+sum (native)"] += pc() - tb
            continue
        gi, jobs = B.flush()
        used.append(gi)
        tc = pc(); acc["flush"] += tc - tb
        # each group's sum on its own stream (Likelihood.FUSED_SUM_OWN_STREAM)
        sst = B.groups[gi]["stream"]
        tcon = self._tile_constants(jobs[0][1], sst, F)
        B.sum_loglike(gi, self._d, self._w_templ, out[g0:g0 + len(jobs)], sst.cuda_stream,
                      tile_const=tcon)
        td = pc(); acc["sum+events"] += td - tc
    last = used[-1]
    for gj in sorted(set(used) - {last}):
        lib.efd_stream_order(F["gst"][gj], (ctypes.c_void_p * 1)(F["gst"][last]), 1)
    lib.efd_download(pin.data_ptr(), out.data_ptr(), 8 * n, F["gst"][last])
    t3 = pc()
    B._pending = []
    B.groups[last]["stream"].synchronize()
    t4 = pc(); acc["sync"] += t4 - t3
    host = pin[:n].numpy().copy()
    if np.isnan(host).any():
        B.wait()
    t5 = pc(); acc["status"] += t5 - t4
    return host
L.Likelihood._get_ll_fused = fused
orig_get_ll = L.Likelihood.get_ll
def get_ll(self, *a, **k):
    t0 = pc(); r = orig_get_ll(self, *a, **k); acc["get_ll_total"] += pc() - t0; return r
L.Likelihood.get_ll = get_ll
for i in range(5):
    s.like(batches[i % len(batches)], **s.kwargs)
torch.cuda.synchronize()
acc.clear()
ft = BatchPreparer.FLUSH_TIMERS = {}
N = 40
t0 = pc()
for i in range(N):
    s.like(batches[i % len(batches)], **s.kwargs)
wall = pc() - t0
print(json.dumps({"cfg": sys.argv[1:], "walkers": s.half_step, "ms_per_half_step": wall / N * 1e3,
                  "us_per_half_step": {k: v / N * 1e6 for k, v in acc.items()},
                  "flush_us_per_half_step": {k: v / N * 1e6 for k, v in ft.items()}}, indent=1))

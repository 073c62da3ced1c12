"""Walker sharding across GPUs: one process per GPU, torch.distributed (RCCL on ROCm).

SURVEY.md section 8(e): every walker's waveform and log-likelihood is independent, so a batch
of B walkers (ntemps * nwalkers / 2 per Eryn half-step, red_blue.py:149-156; the drivers'
Likelihood.__call__, emri_pe.py:381-414) splits as rank r of G taking walkers
[r B / G, (r + 1) B / G). Each rank holds its own replica of the data and noise weights
(injected once per rank). The data path has no collective; the only exchanges are the
parameter block (B x ndim float64, <= a few KB) broadcast from the driving rank and an
all-gather of the B float64 log-likelihoods -- both latency-bound, so their size never matters
on xGMI.

Two ways to drive it:
  - SPMD: every rank calls `sharded(params)` with the same params (e.g. identically seeded
    samplers), broadcast=False skips the parameter broadcast;
  - driver/servers: rank `src` calls `sharded(params)`; the other ranks sit in
    `sharded.serve()` until the driver calls `sharded.close()`.
Backend "nccl" (RCCL) uses device tensors of the current GPU; "gloo" (CPU tests) host tensors.

Parameter scans (config 3, check_mode_by_mode.py:183-229) shard the same way through
ShardedScan: the points go round-robin over the ranks, each rank runs the batched generator on
its own points and the per-point records (not the spectra) are all-gathered.
"""

import numpy as np


def shard_range(n, rank, world):
    """[lo, hi) of the n walkers owned by `rank` of `world` (balanced, contiguous, in order)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    return n * rank // world, n * (rank + 1) // world


class ShardedLikelihood:
    """Evaluate a batch of walkers' log-likelihoods across ranks.

    like: this package's Likelihood (called as Eryn calls it, `like(params, **call_kwargs)`:
    parameter transforms, subset batching, get_ll; emri_pe.py:399-417 with Eryn's
    vectorize=True, ensemble.py:1283-1318, and its _FunctionWrapper kwargs, :1539-1583), or any
    callable params[b, ndim] -> array[b]; an object without __call__ is used through get_ll.
    call_kwargs: the waveform kwargs of every call (T, dt, eps[, f_arr]).
    """

    _STOP = -1

    def __init__(self, like, group=None, src=0, broadcast=True, call_kwargs=None):
        import torch
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("ShardedLikelihood needs torch.distributed to be initialised")
        self.torch, self.dist = torch, dist
        self.like = like
        self.group = group
        self.src = src
        self.broadcast = broadcast
        self.call_kwargs = dict(call_kwargs or {})
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if dist.get_backend(group) == "nccl":
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")
        self.evaluated = 0      # walkers this rank evaluated (for accounting / tests)

    def _local(self, params):
        fn = self.like if callable(self.like) else self.like.get_ll
        if len(params) == 0:
            return np.zeros(0, dtype=np.float64)
        out = np.asarray(fn(params, **self.call_kwargs), dtype=np.float64).reshape(-1)
        if len(out) != len(params):
            raise ValueError(f"likelihood returned {len(out)} values for {len(params)} walkers")
        self.evaluated += len(params)
        return out

    def _bcast_params(self, params):
        torch, dist = self.torch, self.dist
        shape = torch.zeros(2, dtype=torch.int64, device=self.device)
        if self.rank == self.src:
            if params is None:
                shape[0] = self._STOP
            else:
                shape[0], shape[1] = params.shape[0], params.shape[1]
        dist.broadcast(shape, self.src, group=self.group)
        B, ndim = int(shape[0]), int(shape[1])
        if B == self._STOP:
            return None
        buf = torch.empty((B, ndim), dtype=torch.float64, device=self.device)
        if self.rank == self.src:
            buf.copy_(torch.as_tensor(params, dtype=torch.float64))
        dist.broadcast(buf, self.src, group=self.group)
        return buf.cpu().numpy()

    def _evaluate(self, params):
        torch, dist = self.torch, self.dist
        B = len(params)
        lo, hi = shard_range(B, self.rank, self.world)
        mine = self._local(params[lo:hi])
        width = -(-B // self.world)
        pad = torch.zeros(width, dtype=torch.float64, device=self.device)
        pad[:hi - lo] = torch.as_tensor(mine, dtype=torch.float64)
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(parts, pad, group=self.group)
        out = np.empty(B, dtype=np.float64)
        for r, part in enumerate(parts):
            a, b = shard_range(B, r, self.world)
            out[a:b] = part[:b - a].cpu().numpy()
        return out

    def __call__(self, params):
        params = np.asarray(params, dtype=np.float64)
        if params.ndim != 2:
            raise ValueError("params must be [walkers, ndim]")
        if self.broadcast:
            params = self._bcast_params(params)
        return self._evaluate(params)

    def serve(self):
        """Non-driving ranks: evaluate shards until the driver calls close()."""
        if not self.broadcast:
            raise RuntimeError("serve() needs broadcast=True")
        if self.rank == self.src:
            raise RuntimeError("the driving rank does not serve")
        while True:
            params = self._bcast_params(None)
            if params is None:
                return
            self._evaluate(params)

    def close(self):
        """Driving rank: release the serving ranks."""
        if self.rank == self.src and self.broadcast:
            self._bcast_params(None)


def scan_points(n, rank, world):
    """The points of an n-point scan owned by `rank` of `world`: round-robin (SURVEY.md 8(e),
    config 3), so each rank gets every part of the grid (in config 3's (M, e0) order the cost of
    a point grows with M: contiguous blocks would hand one rank all the long inspirals)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    return np.arange(rank, n, world, dtype=np.int64)


def power_summary(out):
    """Default per-point record of a scan: sum |h+|^2, sum |hx|^2 and max |h+| over f >= 0
    (out: complex [P][2][N_pos]) -- a checksum of each spectrum that travels in 24 bytes."""
    import torch
    p = (out.real ** 2 + out.imag ** 2).sum(dim=2)            # [P][2]
    mx = out[:, 0].abs().amax(dim=1, keepdim=True)             # [P][1]
    return torch.cat([p, mx], dim=1).to(torch.float64).cpu().numpy()


class ScanResult:
    """A sharded scan's outcome on one rank.

    summary [n][k]: every point's record in point order (all ranks); owner [n]: the rank that
    generated each point; seconds [world]: each rank's time for its points (host upstream,
    device work and the summary; max over ranks = the scan's time); points / out: this rank's
    point indices and their [h+, hx] (complex128 [P][2][N_pos] on this rank's device), which
    stay where they were made (the reference's scan keeps only per-point numbers,
    check_mode_by_mode.py:255-321)."""

    def __init__(self, summary, owner, seconds, points, out):
        self.summary, self.owner, self.seconds = summary, owner, seconds
        self.points, self.out = points, out


class ShardedScan:
    """A parameter scan (check_mode_by_mode.py:183-229: per point few_gen of its injection)
    sharded over the ranks, one process per GPU. Rank r generates the points scan_points(n, r,
    world) with the batched generator (GenerateEMRIWaveform.generate_batch: its rows' host
    upstream on this rank's core share, then the device work in groups of 16), reduces each
    point to a small record (`summary`: default power_summary) and all-gathers the records and
    its elapsed time. No spectrum crosses the interconnect: the only exchange is the n x k
    float64 records (RCCL over xGMI with backend "nccl", gloo on CPU).

    gen: a GenerateEMRIWaveform (or any object with generate_batch(params, out, T=, dt=, eps=,
    f_arr=, **kw) and positive_bins(T, dt, f_arr)); p0_solver(row) -> p0 (optional, e.g. the
    drivers' get_p_at_t for 0.99 Tobs) runs on this rank's rows before the generator, inside the
    timed region, as the drivers' loop does it per point; mapper (e.g. the upstream thread pool's
    map) spreads those solves over this rank's host cores."""

    def __init__(self, gen, group=None, summary=power_summary, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.gen, self.group, self.summary = gen, group, summary
        # without torch.distributed: one process, the whole scan (no exchange)
        self.single = not dist.is_initialized()
        self.rank = 0 if self.single else dist.get_rank(group)
        self.world = 1 if self.single else dist.get_world_size(group)
        nccl = not self.single and dist.get_backend(group) == "nccl"
        if device is not None:
            self.device = torch.device(device)
        elif nccl or (self.single and torch.cuda.is_available()):
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")
        self.comm_device = (torch.device("cuda", torch.cuda.current_device()) if nccl
                            else torch.device("cpu"))

    def __call__(self, params, T=1.0, dt=10.0, eps=1e-5, f_arr=None, p0_solver=None, mapper=None,
                 **kwargs):
        import time
        torch, dist = self.torch, self.dist
        params = np.array(params, dtype=np.float64).reshape(-1, 14)
        n = len(params)
        mine = scan_points(n, self.rank, self.world)
        npos = int(self.gen.positive_bins(T, dt, f_arr))
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        rows = params[mine].copy()
        if p0_solver is not None and len(rows):
            rows[:, 3] = [float(v) for v in (mapper or map)(p0_solver, list(rows))]
        out = torch.empty((len(mine), 2, npos), dtype=torch.complex128, device=self.device)
        if len(mine):
            self.gen.generate_batch(rows, out, T=T, dt=dt, eps=eps, f_arr=f_arr, **kwargs)
            rec = np.asarray(self.summary(out), dtype=np.float64).reshape(len(mine), -1)
        else:
            rec = np.zeros((0, 0))
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        elapsed = time.perf_counter() - t0
        self.rows = rows
        if self.single:
            return ScanResult(rec, np.zeros(n, dtype=np.int64), np.array([elapsed]), mine, out)
        # every rank's record width (a rank with no point reports 0)
        k = torch.tensor([rec.shape[1]], dtype=torch.int64, device=self.comm_device)
        dist.all_reduce(k, op=dist.ReduceOp.MAX, group=self.group)
        k = int(k)
        width = max(1, -(-n // self.world))   # one row even for an empty scan (its time)
        pad = torch.zeros((width, k + 1), dtype=torch.float64, device=self.comm_device)
        if len(mine):
            pad[:len(mine), :k] = torch.as_tensor(rec, dtype=torch.float64)
        pad[0, k] = elapsed   # the rank's time rides in the last column of its first row
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(parts, pad, group=self.group)
        summary = np.empty((n, k), dtype=np.float64)
        owner = np.empty(n, dtype=np.int64)
        seconds = np.empty(self.world, dtype=np.float64)
        for r, part in enumerate(parts):
            pr = part.cpu().numpy()
            idx = scan_points(n, r, self.world)
            summary[idx] = pr[:len(idx), :k]
            owner[idx] = r
            seconds[r] = pr[0, k]
        return ScanResult(summary, owner, seconds, mine, out)

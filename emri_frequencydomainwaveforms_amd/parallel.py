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

"""Walker sharding (emri_frequencydomainwaveforms_amd/parallel.py) on CPU with gloo, 2 ranks.

The GPU path uses the same code with backend "nccl" (RCCL); here the per-walker likelihood is a
host stand-in, since only the distribution logic is under test: shard bounds, parameter
broadcast, the all-gather order, and that each rank evaluates exactly its own walkers.
"""

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from emri_frequencydomainwaveforms_amd.parallel import ShardedLikelihood, shard_range  # noqa: E402


def test_shard_range_partitions():
    for n in (0, 1, 5, 8, 64, 127):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ll(params):
    return -np.sum((params - 0.5) ** 2, axis=1) * 3.0


def _worker(rank, world, port, mode, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(7)
        batches = [rng.normal(size=(b, 14)) for b in (5, 1, 8, 3)]
        if mode == "spmd":
            sl = ShardedLikelihood(_ll, broadcast=False)
            outs = [sl(p) for p in batches]
        else:
            sl = ShardedLikelihood(_ll, src=0)
            if rank == 0:
                outs = [sl(p) for p in batches]
                sl.close()
            else:
                sl.serve()
                outs = None
        q.put((rank, outs, sl.evaluated))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["spmd", "driver"])
def test_sharded_likelihood_gloo(mode):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, outs, evaluated = q.get(timeout=120)
        res[rank] = (outs, evaluated)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(7)
    batches = [rng.normal(size=(b, 14)) for b in (5, 1, 8, 3)]
    expect = [_ll(p) for p in batches]
    for rank in range(world):
        outs, evaluated = res[rank]
        if outs is not None:
            for o, e in zip(outs, expect):
                np.testing.assert_array_equal(o, e)
        # each rank evaluated exactly its shard of every batch
        mine = sum(shard_range(len(p), rank, world)[1] - shard_range(len(p), rank, world)[0]
                   for p in batches)
        assert evaluated == mine
    assert res[0][1] + res[1][1] == sum(len(p) for p in batches)

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


class _ScanGen:
    """Host stand-in for GenerateEMRIWaveform.generate_batch (the distribution logic is under
    test): row j's [h+, hx] is a deterministic function of its parameters; calls are recorded."""
    NPOS = 37

    def __init__(self):
        self.rows = []

    def positive_bins(self, T, dt, f_arr=None):
        return self.NPOS

    def generate_batch(self, params, out, T=1.0, dt=10.0, eps=1e-5, f_arr=None, **kw):
        k = torch.arange(self.NPOS, dtype=torch.float64)
        for j, p in enumerate(params):
            self.rows.append(np.array(p))
            out[j, 0] = torch.complex(p[0] * torch.cos(k * p[4]), p[3] * torch.sin(k))
            out[j, 1] = torch.complex(p[1] * k, -p[0] * torch.ones_like(k))
        return out


def _scan_expect(params):
    k = np.arange(_ScanGen.NPOS, dtype=np.float64)
    out = []
    for p in params:
        hp = p[0] * np.cos(k * p[4]) + 1j * p[3] * np.sin(k)
        hc = p[1] * k - 1j * p[0] * np.ones_like(k)
        out.append([np.sum(np.abs(hp) ** 2), np.sum(np.abs(hc) ** 2), np.abs(hp).max()])
    return np.array(out)


def _scan_worker(rank, world, port, n, q):
    import torch.distributed as dist
    from emri_frequencydomainwaveforms_amd.parallel import ShardedScan
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Ms = np.logspace(5, 7, 10)
        e0s = np.linspace(0.1, 0.6, 10)
        params = np.array([[M, 1e-5 * M, 0.0, 10.0, e0, 1.0, 1.0, 0.2, 0.2, 0.8, 0.8, 1.0, 0.0,
                            3.0] for M in Ms for e0 in e0s])[:n]
        gen = _ScanGen()
        scan = ShardedScan(gen)
        # the p0 solve (a stand-in: p0 = 10 + e0) runs on each rank's own rows
        res = scan(params, T=1.0, dt=10.0, eps=1e-2, p0_solver=lambda r: 10.0 + r[4])
        q.put((rank, res.summary, res.owner, res.seconds, res.points,
               np.array(gen.rows), res.out.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [100, 7, 1, 0])
def test_sharded_scan_gloo(n):
    """Config 3's scan over 2 gloo ranks: the shards are disjoint, round-robin and cover the
    grid; every rank gets every point's record in point order; each rank generated exactly its
    own points (after its own p0 solves); a rank with no point (n = 1) still joins the gather,
    and an empty scan (n = 0) returns empty records on every rank (advisor r05)."""
    import torch.multiprocessing as mp
    from emri_frequencydomainwaveforms_amd.parallel import scan_points
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _free_port()
    procs = [ctx.Process(target=_scan_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    Ms = np.logspace(5, 7, 10)
    e0s = np.linspace(0.1, 0.6, 10)
    params = np.array([[M, 1e-5 * M, 0.0, 10.0, e0, 1.0, 1.0, 0.2, 0.2, 0.8, 0.8, 1.0, 0.0, 3.0]
                       for M in Ms for e0 in e0s])[:n]
    params[:, 3] = 10.0 + params[:, 4]
    if n == 0:
        for r in range(world):
            summary, owner, seconds, points, rows, out = res[r]
            assert summary.shape[0] == 0 and len(owner) == 0 and len(points) == 0
            assert seconds.shape == (world,) and np.all(seconds >= 0)
        return
    expect = _scan_expect(params)
    owned = [res[r][3] for r in range(world)]
    allpts = np.concatenate(owned)
    assert len(allpts) == n and len(np.unique(allpts)) == n          # disjoint, covering
    for r in range(world):
        summary, owner, seconds, points, rows, out = res[r]
        np.testing.assert_array_equal(points, scan_points(n, r, world))
        np.testing.assert_array_equal(points, np.arange(r, n, world))  # round-robin
        np.testing.assert_allclose(summary, expect, rtol=1e-13, atol=0)
        np.testing.assert_array_equal(owner, np.arange(n) % world)
        assert seconds.shape == (world,) and np.all(seconds >= 0)
        if len(points):
            np.testing.assert_array_equal(rows, params[points])       # after the p0 solve
            assert out.shape == (len(points), 2, _ScanGen.NPOS)
        else:
            assert len(rows) == 0
    # both ranks hold the same gathered records
    np.testing.assert_array_equal(res[0][0], res[1][0])


def test_scan_points_partition():
    from emri_frequencydomainwaveforms_amd.parallel import scan_points
    for n in (0, 1, 5, 100):
        for world in (1, 2, 3, 8):
            pts = np.concatenate([scan_points(n, r, world) for r in range(world)])
            assert sorted(pts.tolist()) == list(range(n))
    with pytest.raises(ValueError):
        scan_points(4, 3, 2)

"""Per-rank host-core shares (emri_frequencydomainwaveforms_amd/hostcpu.py).

One process per GPU: each rank's upstream thread pool and native thread count come from its own
disjoint share of the node's cores, not from OMP_NUM_THREADS (torchrun sets it to 1) and not from
the whole node per rank. The gloo test launches 2 ranks as torchrun would (LOCAL_RANK,
LOCAL_WORLD_SIZE, OMP_NUM_THREADS=1) and checks the shares they pin are disjoint and sized as
the pool uses them. Reference shape: emri_pe.py:514-575 (mp.Pool next to the sampler),
ensemble.py:1283-1318 (vectorised likelihood call).
"""

import os
import socket

import numpy as np
import pytest

from emri_frequencydomainwaveforms_amd import hostcpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("ncores,world", [(128, 8), (16, 1), (16, 2), (10, 4), (3, 8), (8, 3)])
def test_rank_cores_disjoint_and_covering(ncores, world):
    aff = set(range(100, 100 + ncores))   # a faked affinity set (core ids need not start at 0)
    shares = [hostcpu.rank_cores(aff, r, world) for r in range(world)]
    assert all(len(s) >= 1 for s in shares)
    if ncores >= world:
        flat = [c for s in shares for c in s]
        assert len(flat) == len(set(flat)) == ncores          # disjoint, every core used
        sizes = [len(s) for s in shares]
        assert max(sizes) - min(sizes) <= 1
        for s in shares:                                      # contiguous runs
            assert s == list(range(s[0], s[0] + len(s)))
    else:
        assert all(len(s) == 1 for s in shares)


def test_threads_ignores_omp_and_caps(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    monkeypatch.delenv("EFD_HOST_THREADS", raising=False)
    assert hostcpu.threads(list(range(12))) == 12
    assert hostcpu.threads(list(range(64))) == hostcpu.MAX_THREADS
    monkeypatch.setenv("EFD_HOST_THREADS", "3")
    assert hostcpu.threads(list(range(64))) == 3


def test_rank_cores_bad_rank():
    with pytest.raises(ValueError):
        hostcpu.rank_cores({0, 1, 2, 3}, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    # the environment torchrun gives each rank of one node
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      OMP_NUM_THREADS="1")
    os.environ.pop("EFD_HOST_THREADS", None)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emri_frequencydomainwaveforms_amd import hostcpu as hc
        from emri_frequencydomainwaveforms_amd import waveform
        share = hc.pin()
        n = hc.threads()
        pool = waveform._pool()._max_workers
        # a faked 128-core node split the same way (the 8-GPU box's shape)
        fake = hc.rank_cores(set(range(128)), rank, world)
        got = [None] * world
        dist.all_gather_object(got, dict(share=sorted(share),
                                         affinity=sorted(os.sched_getaffinity(0)),
                                         threads=n, pool=pool, fake=fake))
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_two_ranks_pin_disjoint_shares():
    ncpu = len(os.sched_getaffinity(0))
    if ncpu < 2:
        pytest.skip("needs 2 host cores")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = res[0]
    a, b = got[0], got[1]
    assert set(a["share"]).isdisjoint(b["share"])
    assert a["affinity"] == a["share"] and b["affinity"] == b["share"]   # pinned
    assert len(a["share"]) + len(b["share"]) == ncpu
    for g in (a, b):
        # OMP_NUM_THREADS=1 from the launcher does not decide the pool or the native threads
        assert g["threads"] == g["pool"] == min(len(g["share"]), hostcpu.MAX_THREADS)
    assert set(a["fake"]).isdisjoint(b["fake"]) and len(a["fake"]) == len(b["fake"]) == 64
    assert np.array_equal(res[1][0]["share"], a["share"])   # both ranks saw the same gather


def test_per_rank_set_not_split_again(monkeypatch):
    """A launcher that already bound each rank to its own cores (a strict subset of the cgroup's
    cpuset) keeps that set whole; ranks that all report the allocation's whole set split it,
    whatever its size against the node (advisor r05: 8 ranks sharing a 16-core allocation of a
    128-core node hold node / LW cores each and must still split); EFD_HOST_SPLIT forces either
    way."""
    monkeypatch.delenv("EFD_HOST_SPLIT", raising=False)
    node = set(range(128))
    own = set(range(32, 48))                  # 16 cores of a 128-core node, 8 ranks, bound
    assert hostcpu.rank_cores(own, 3, 8, allowed=node) == sorted(own)
    assert hostcpu.rank_cores(node, 3, 8, allowed=node) == list(range(48, 64))
    alloc = set(range(16, 32))                # one 16-core allocation shared by 8 ranks
    shares = [hostcpu.rank_cores(alloc, r, 8, allowed=alloc) for r in range(8)]
    assert [len(x) for x in shares] == [2] * 8
    assert sorted(c for x in shares for c in x) == sorted(alloc)
    wide = set(range(20, 40))                 # a 20-core per-rank binding is kept, not re-split
    assert hostcpu.rank_cores(wide, 5, 8, allowed=node) == sorted(wide)
    assert hostcpu.rank_cores(alloc, 3, 8, allowed=None) == [22, 23]   # cpuset unreadable
    monkeypatch.setenv("EFD_HOST_SPLIT", "0")
    assert hostcpu.rank_cores(node, 3, 8, allowed=node) == sorted(node)
    monkeypatch.setenv("EFD_HOST_SPLIT", "1")
    assert hostcpu.rank_cores(own, 3, 8, allowed=node) == [38, 39]


def test_allowed_cores_parses_cpuset():
    a = hostcpu.allowed_cores()
    if a is not None:
        assert set(os.sched_getaffinity(0)) <= a


_PIN_CHILD = r"""
import os, sys, threading, time, json
os.environ.update(LOCAL_RANK="1", LOCAL_WORLD_SIZE="2", EFD_HOST_THREADS="5")
sys.path.insert(0, sys.argv[1])
stop = threading.Event()
t = threading.Thread(target=stop.wait, daemon=True)
t.start()
time.sleep(0.05)
from emri_frequencydomainwaveforms_amd import hostcpu
n = hostcpu.threads()        # EFD_HOST_THREADS set: the count is 5, the process still pinned
share = sorted(hostcpu.pin())
tids = [int(x) for x in os.listdir("/proc/self/task")]
aff = {tid: sorted(os.sched_getaffinity(tid)) for tid in tids}
stop.set()
print(json.dumps(dict(n=n, share=share, aff=list(aff.values()))))
"""


def test_pin_every_thread_and_override():
    """pin() restricts every thread of the process (a thread started before it included), and
    setting EFD_HOST_THREADS still pins."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if len(os.sched_getaffinity(0)) < 2:
        pytest.skip("needs 2 cores to split")
    env = dict(os.environ)
    env.pop("EFD_HOST_SPLIT", None)
    r = subprocess.run([sys.executable, "-c", _PIN_CHILD, root], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n"] == 5
    full = sorted(os.sched_getaffinity(0))
    assert out["share"] == hostcpu.rank_cores(set(full), 1, 2)
    assert len(out["aff"]) >= 2 and all(a == out["share"] for a in out["aff"])

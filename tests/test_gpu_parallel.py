"""Walker sharding over the real HIP likelihood: two processes on the one GPU (gloo carries the
parameter broadcast and the log-likelihood all-gather; RCCL is the same code with backend
"nccl" on one GPU per rank, which a one-GPU box cannot host twice).

Each rank builds the emri_pe.py-shaped setup (emri_frequencydomainwaveforms_amd.pe: injection,
Likelihood with the TransformContainer, the reference's walker start) at a short observation,
then rank 0 drives ShardedLikelihood over two red-blue half-steps while rank 1 serves. The
gathered logL of every walker must be bitwise the single-process Likelihood's, and each rank
must have evaluated exactly its contiguous shard (emri_pe.py:514-575 with Eryn vectorize=True,
ensemble.py:1283-1318).
"""

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SETUP = dict(Tobs=0.05, dt=20.0, eps=1e-2, M=3e5, mu=10.0, e0=0.3, nwalkers=16, ntemps=1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emri_frequencydomainwaveforms_amd import pe
        from emri_frequencydomainwaveforms_amd.parallel import ShardedLikelihood
        s = pe.setup(**SETUP)
        sl = ShardedLikelihood(s.like, src=0, call_kwargs=s.kwargs)
        if rank == 0:
            outs = [sl(b) for b in s.half_steps()]
            sl.close()
        else:
            sl.serve()
            outs = None
        q.put((rank, outs, sl.evaluated))
    except Exception as exc:   # surface the child's failure to the test
        q.put((rank, repr(exc), -1))
    finally:
        dist.destroy_process_group()


def test_sharded_hip_likelihood_two_ranks_bitwise():
    import torch.multiprocessing as mp
    from emri_frequencydomainwaveforms_amd import pe
    from emri_frequencydomainwaveforms_amd.parallel import shard_range
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, outs, evaluated = q.get(timeout=240)
        res[rank] = (outs, evaluated)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        assert res[rank][1] >= 0, res[rank][0]
    s = pe.setup(**SETUP)
    batches = s.half_steps()
    ref = [s.like(b, **s.kwargs) for b in batches]
    for got, exp in zip(res[0][0], ref):
        np.testing.assert_array_equal(got, exp)
    for rank in range(world):
        mine = sum(shard_range(len(b), rank, world)[1] - shard_range(len(b), rank, world)[0]
                   for b in batches)
        assert res[rank][1] == mine
    assert np.all(np.concatenate(ref) < 0.0)

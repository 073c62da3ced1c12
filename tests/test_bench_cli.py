"""bench.py's rank-count guard (CPU): --gpus must equal the launcher's WORLD_SIZE, so a
multi-GPU figure can never come from one process timing one GPU (VERDICT r4 missing #3)."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, world=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    if world is not None:
        env["WORLD_SIZE"] = str(world)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, timeout=120, env=env)


def test_gpus_without_launcher_fails():
    for mode in ([], ["--likelihood", "config4"], ["--scan", "config3"]):
        r = _run(["--gpus", "8", *mode])
        assert r.returncode == 2, r.stderr
        assert "WORLD_SIZE=1" in r.stderr and "torch.distributed.run" in r.stderr


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2"], world=4)
    assert r.returncode == 2 and "--gpus 2 but WORLD_SIZE=4" in r.stderr


def test_world_size_helper():
    sys.path.insert(0, ROOT)
    import bench
    os.environ.pop("WORLD_SIZE", None)
    assert bench.world_size(1) == 1

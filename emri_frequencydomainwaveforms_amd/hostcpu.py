"""Host-core share of this process: one process per GPU, each with its own disjoint set of cores.

The reference runs its upstream (trajectory, amplitudes, mode selection) on a process pool next
to the sampler (`emri_pe.py:545`, `mp.Pool(4)`) and hands Eryn a vectorised likelihood
(`ensemble.py:1283-1318`). Here each rank drives one GPU and runs the stand-in upstream of its
walker shard on a thread pool (`waveform._pool`) whose native calls split their knots over
`efd_host_set_threads` threads. Both counts come from this module, explicitly, so that neither
the launcher's `OMP_NUM_THREADS=1` (torchrun sets it) nor a whole node's cores per rank decide
them:

  - the process's affinity set is split into `LOCAL_WORLD_SIZE` contiguous, disjoint shares and
    rank `LOCAL_RANK` takes its own (a single process keeps the whole set). A set the launcher
    or scheduler already bound per rank -- a strict subset of the cores the process's cgroup
    allows (cpuset.cpus.effective), which torchrun never narrows -- is kept as it is. The
    number of cores is no evidence either way: 8 ranks sharing a 16-core allocation of a
    128-core node hold 16 = 128 / 8 cores each and still have to split them.
    `EFD_HOST_SPLIT=0` never splits, `EFD_HOST_SPLIT=1` always does;
  - `pin()` restricts every thread of the process to that share (os.sched_setaffinity on each
    task of /proc/self/task: the call is per thread on Linux, so threads torch or HIP started
    earlier would otherwise keep the whole node; threads started later inherit it), so ranks
    on one node do not oversubscribe each other's cores;
  - `threads()` is the share's size, capped at `MAX_THREADS`; `EFD_HOST_THREADS` overrides the
    count (the process is pinned either way).
"""

import os

MAX_THREADS = 16   # the GPU box's CPU share per GPU; more threads per walker batch stop paying


def local_rank_world(env=None):
    env = os.environ if env is None else env
    return int(env.get("LOCAL_RANK", "0")), int(env.get("LOCAL_WORLD_SIZE", "1"))


def allowed_cores():
    """The cores this process's cgroup allows (cgroup v2 cpuset.cpus.effective, else v1
    cpuset.effective_cpus), or None when neither can be read."""
    for path in ("/sys/fs/cgroup/cpuset.cpus.effective",
                 "/sys/fs/cgroup/cpuset/cpuset.effective_cpus"):
        try:
            text = open(path).read().strip()
        except OSError:
            continue
        out = set()
        try:
            for part in text.split(","):
                if not part:
                    continue
                a, _, b = part.partition("-")
                out.update(range(int(a), int(b or a) + 1))
        except ValueError:
            continue
        return out or None
    return None


def rank_cores(affinity=None, local_rank=None, local_world=None, allowed="auto"):
    """This rank's disjoint share of `affinity` (default: the process's affinity set), split
    into `local_world` contiguous chunks of equal size (the remainder goes to the first ranks).
    With fewer cores than ranks every rank keeps one core (round-robin). An affinity set that is
    a strict subset of `allowed` (default: allowed_cores(), the cgroup's cpuset) was bound per
    rank by the launcher and is returned whole; EFD_HOST_SPLIT=0 / 1 forces no split / a split."""
    cores = sorted(os.sched_getaffinity(0) if affinity is None else affinity)
    lr, lw = local_rank_world()
    lr = lr if local_rank is None else int(local_rank)
    lw = lw if local_world is None else int(local_world)
    if lw > 1 and not 0 <= lr < lw:
        raise ValueError(f"local rank {lr} outside a local world of {lw}")
    mode = os.environ.get("EFD_HOST_SPLIT", "")
    if lw <= 1 or not cores or mode == "0":
        return cores
    if mode != "1":
        allowed = allowed_cores() if allowed == "auto" else allowed
        if allowed is not None and set(cores) < set(allowed):
            return cores   # narrowed below the cgroup's cores: bound per rank, not split again
    if len(cores) < lw:
        return [cores[lr % len(cores)]]
    base, extra = divmod(len(cores), lw)
    start = lr * base + min(lr, extra)
    return cores[start:start + base + (1 if lr < extra else 0)]


_PINNED = None


def pin():
    """Restrict every thread of this process to its rank's share (once; a no-op for a single
    local process). Returns the share."""
    global _PINNED
    if _PINNED is None:
        share = rank_cores()
        _, lw = local_rank_world()
        if lw > 1 and set(share) != os.sched_getaffinity(0):
            _pin_all_threads(share)
        _PINNED = share
    return _PINNED


def _pin_all_threads(share):
    """sched_setaffinity for every thread of the process (Linux: the call takes a thread id)."""
    try:
        tids = [int(t) for t in os.listdir("/proc/self/task")]
    except OSError:
        tids = [0]
    for tid in tids:
        try:
            os.sched_setaffinity(tid, share)
        except (OSError, ProcessLookupError):
            pass   # a thread that ended meanwhile
    os.sched_setaffinity(0, share)


def threads(share=None):
    """Host threads for this rank's upstream: its share's size (at most MAX_THREADS), or
    EFD_HOST_THREADS when set. OMP_NUM_THREADS is deliberately not consulted."""
    share = pin() if share is None else share
    env = os.environ.get("EFD_HOST_THREADS")
    if env:
        return max(1, int(env))
    return max(1, min(len(share), MAX_THREADS))

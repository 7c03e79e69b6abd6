"""Host CPU budget of this process: the cores it may use (affinity mask,
capped by a cgroup CPU quota and by OMP_NUM_THREADS), shared by the ranks of
one node (LOCAL_WORLD_SIZE under torch.distributed.run). The host side of the
simulator's shot loop (simulator.py:244-315 in the reference) — NumPy's
reliability order for the rare OSD shots the device order leaves to NumPy,
the host order and the host C++ OSD — sizes its thread pools from this, so 8
ranks on one node do not each start a pool the size of the whole machine.
The library's C++ default (nthreads <= 0) computes the same process budget."""
import os


def process_cores():
    """(cores, how): the affinity mask, capped by cgroup cpu.max and OMP_NUM_THREADS."""
    try:
        n = len(os.sched_getaffinity(0))
        how = ["sched_getaffinity"]
    except AttributeError:
        n, how = os.cpu_count() or 1, ["os.cpu_count"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            c = max(1, int(float(q) / float(per)))
            if c < n:
                n, how = c, how + ["cgroup cpu.max"]
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < n:
        n, how = int(omp), how + ["OMP_NUM_THREADS"]
    return n, " capped by ".join(how)


def _own_cpuset():
    """Whether this rank's CPU set is known to be its own (not shared with the
    node's other ranks): only when the launcher says so, QLDPC_RANK_CPUSET=own
    (e.g. one `taskset` / numactl CPU list per rank). An affinity mask smaller
    than the machine proves nothing: a container cpuset, a Slurm allocation or
    a `taskset` around the launcher gives every rank the same mask."""
    return os.environ.get("QLDPC_RANK_CPUSET", "").strip().lower() == "own"


def rank_cores(cap=16):
    """Host threads one rank should use, at most `cap`, at least 1: the
    process budget (process_cores) divided among the node's ranks
    (LOCAL_WORLD_SIZE; ranks started without it share the machine with nobody
    we know of), unless the launcher declared each rank's CPU set its own
    (QLDPC_RANK_CPUSET=own), which is then already the rank's share."""
    cores, _ = process_cores()
    if _own_cpuset():
        return max(1, min(cap, cores))
    local = os.environ.get("LOCAL_WORLD_SIZE", "1")
    share = max(1, int(local)) if local.isdigit() else 1
    return max(1, min(cap, cores // share if cores >= share else 1))

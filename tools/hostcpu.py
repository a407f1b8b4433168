"""The host CPUs a run may use: the scheduler affinity mask, the cgroup CPU quota (cpu.max, v2, or
cpu.cfs_quota_us / cpu.cfs_period_us, v1) and the CPU share the GPU box's harness announces in
OMP_NUM_THREADS; `usable` is the smallest of those that are set.  os.cpu_count() reports the whole
machine (256 on the MI355X boxes), which is not what a one-GPU job owns."""
import math
import os


def _cgroup_quota():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return float(q) / float(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0 and p > 0:
            return q / p
    except (OSError, ValueError):
        pass
    return None


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def host_cores():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = _cgroup_quota()
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    limits = [aff] + ([max(1, math.floor(quota))] if quota else []) + ([omp] if omp else [])
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_cpu_quota": quota, "omp_num_threads": omp,
            "usable": min(limits), "cpu_model": cpu_model()}

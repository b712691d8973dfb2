"""Host-thread placement for one GPU's process (what a launcher's numactl / taskset would do).

The render step submits many small kernels from one or a few host threads (C2: ~50 launches per
step at ~0.2 ms of GPU work per view), so its throughput follows the host threads' cores.  On the
shared GPU boxes every process may run on all 256 CPUs of the host (two NUMA nodes) under a cgroup
quota, and the kernel scheduler moves the submitting threads onto cores that other tenants keep busy:
C2 ran at 255-460 Msplats/s from one process to the next on one box, and at 479-487 with the process
pinned to a few idle CPUs of one node (tools/c2_pin.py).  ``pin_host_threads`` picks such CPUs -- the
least busy ones (sampled from /proc/stat) of the GPU's NUMA node, in this local rank's share of the
node when several ranks share it, one hardware thread per idle core (a CPU counts as busy as its
busiest SMT sibling) -- and pins every thread of the process to them, including the HIP runtime's and
the library's resolver thread.  Nothing on the device side changes.
"""
from __future__ import annotations

import os
import time


def _cpulist(text):
    out = []
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out += list(range(int(a), int(b or a) + 1))
    return out


def _numa_of_bdf(bdf):
    try:
        return int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
    except (OSError, ValueError):
        return -1


def _gpu_numa_node_sysfs(dev_index):
    """NUMA node of visible GPU ``dev_index`` without initialising the GPU runtime: HIP_VISIBLE_DEVICES
    / ROCR_VISIBLE_DEVICES map it to a ROCr index, the KFD topology's GPU nodes (in ROCr order) give
    its PCI location.  -1 when unknown."""
    try:
        idx = dev_index
        for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
            v = os.environ.get(var)
            if v:
                idx = int(v.split(",")[idx])
        base = "/sys/class/kfd/kfd/topology/nodes"
        gpus = []
        for n in sorted(os.listdir(base), key=int):
            props = {}
            for line in open(os.path.join(base, n, "properties")):
                k, _, val = line.partition(" ")
                props[k] = val.strip()
            if int(props.get("simd_count", "0")) > 0:
                gpus.append(props)
        loc, dom = int(gpus[idx]["location_id"]), int(gpus[idx].get("domain", "0"))
        return _numa_of_bdf(f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 31:02x}.{loc & 7}")
    except (OSError, ValueError, IndexError, KeyError):
        return -1


def _gpu_numa_node(dev_index):
    """NUMA node of the visible GPU ``dev_index`` (-1 when unknown), from its PCI address: from sysfs
    first (no GPU runtime needed), else from the runtime's device properties."""
    node = _gpu_numa_node_sysfs(dev_index)
    if node >= 0:
        return node
    try:
        import torch
        pr = torch.cuda.get_device_properties(dev_index)
        return _numa_of_bdf(f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0")
    except (AttributeError, RuntimeError):
        return -1


def _busy_fraction(cpus, interval=0.05):
    """Busy fraction of each CPU over ``interval`` seconds (/proc/stat), {} when unavailable."""
    def sample():
        out = {}
        try:
            for line in open("/proc/stat"):
                if line.startswith("cpu") and line[3].isdigit():
                    f = line.split()
                    v = [int(x) for x in f[1:]]
                    idle = v[3] + (v[4] if len(v) > 4 else 0)
                    out[int(f[0][3:])] = (sum(v), idle)
        except OSError:
            pass
        return out
    a = sample()
    time.sleep(interval)
    b = sample()
    busy = {}
    for c in cpus:
        if c in a and c in b:
            tot, idle = b[c][0] - a[c][0], b[c][1] - a[c][1]
            busy[c] = 1.0 - idle / tot if tot > 0 else 0.0
    return busy


def _siblings(c):
    """The SMT siblings of CPU ``c`` (itself included), from sysfs; [c] when unknown."""
    try:
        return _cpulist(open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read())
    except (OSError, ValueError):
        return [c]


def _pick(pool, busy, n, smt):
    """The ``n`` least busy CPUs of ``pool``.  ``smt``: rank each CPU by the busier of its core's hardware
    threads (a thread whose sibling runs another tenant's work gets half a core) and take at most one
    CPU per core while there are enough idle cores, so the process's own threads do not share cores."""
    if not smt:
        return sorted(sorted(pool, key=lambda c: (busy.get(c, 1.0), c))[:n])
    sib = {c: _siblings(c) for c in pool}
    used = set()
    # the load on c's core that is not this process's: c and its siblings outside the chosen set
    foreign = lambda c: max(busy.get(x, 1.0) for x in sib[c] if x == c or x not in used)  # noqa: E731
    got = []
    for c in sorted(pool, key=lambda c: (foreign(c), busy.get(c, 1.0), c)):  # one per (nearly) idle core
        if len(got) == n or foreign(c) > 0.25:
            break
        if not used & set(sib[c]):
            got.append(c)
            used.add(c)
    while len(got) < n:  # then the least loaded of the rest (siblings of chosen CPUs count as idle)
        c = min((c for c in pool if c not in used), key=lambda c: (foreign(c), busy.get(c, 1.0), c))
        got.append(c)
        used.add(c)
    return sorted(got)


def choose_cpus(dev_index=0, local_rank=0, local_world=1, n=8):
    """The CPUs ``pin_host_threads`` would use (sorted), or [] when there is no choice to make."""
    if n <= 0 or not hasattr(os, "sched_getaffinity"):
        return []
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) <= n:
        return []
    node = _gpu_numa_node(dev_index)
    pool = allowed
    if node >= 0:
        try:
            local = [c for c in _cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read()) if c in allowed]
            pool = local if len(local) >= n else allowed
        except OSError:
            pass
    if local_world > 1:  # this rank's contiguous share of the pool (ranks of one node do not collide)
        per = max(n, len(pool) // local_world)
        start = (local_rank * per) % max(len(pool), 1)
        share = pool[start:start + per]
        pool = share if len(share) >= n else pool
    smt = os.environ.get("GSR_PIN_SMT", "1") != "0"
    # the siblings' load counts too (they may lie outside the pool)
    busy = _busy_fraction(sorted(set(pool) | {x for c in pool for x in _siblings(c)}) if smt else pool,
                          float(os.environ.get("GSR_PIN_SAMPLE_S", "0.1")))
    return _pick(pool, busy, n, smt)


def pin_host_threads(dev_index=0, local_rank=0, local_world=1, n=8):
    """Pin every thread of this process to ``choose_cpus(...)``; returns the CPUs (or [] when unpinned).
    Best called before the GPU runtime starts (its threads and its host allocations then start on those
    CPUs and their NUMA node); threads that already exist are pinned too."""
    cpus = choose_cpus(dev_index, local_rank, local_world, n)
    if not cpus:
        return []
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except OSError:
            pass
    return cpus


def unpin_host_threads(cpus):
    """Give every thread of the process the CPU set ``cpus`` (e.g. the affinity before pinning)."""
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except OSError:
            pass

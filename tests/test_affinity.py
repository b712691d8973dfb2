"""Host-thread placement (splat_affinity): the CPU choice and the pin / unpin of every thread (CPU)."""
import os
import threading

import pytest

import splat_affinity as A

pytestmark = pytest.mark.skipif(not hasattr(os, "sched_getaffinity"), reason="no sched_getaffinity")


def test_choose_cpus_is_a_subset_of_the_allowed_set():
    allowed = set(os.sched_getaffinity(0))
    if len(allowed) <= 2:
        pytest.skip("too few CPUs to choose from")
    got = A.choose_cpus(dev_index=0, n=2)
    assert len(got) == 2 and set(got) <= allowed and got == sorted(got)
    assert A.choose_cpus(n=0) == []
    assert A.choose_cpus(n=len(allowed)) == []  # nothing to choose: leave the process alone
    # several ranks on one node take disjoint shares when the node has room for them
    if len(allowed) >= 8:
        a, b = A.choose_cpus(local_rank=0, local_world=2, n=2), A.choose_cpus(local_rank=1, local_world=2, n=2)
        assert not set(a) & set(b)


def test_pin_and_unpin_every_thread():
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) <= 2:
        pytest.skip("too few CPUs to choose from")
    stop = threading.Event()
    t = threading.Thread(target=stop.wait, daemon=True)
    t.start()
    try:
        cpus = A.pin_host_threads(n=2)
        assert len(cpus) == 2
        assert sorted(os.sched_getaffinity(0)) == cpus
        assert sorted(os.sched_getaffinity(t.native_id)) == cpus  # an existing thread is pinned too
        A.unpin_host_threads(allowed)
        assert sorted(os.sched_getaffinity(0)) == allowed
        assert sorted(os.sched_getaffinity(t.native_id)) == allowed
    finally:
        A.unpin_host_threads(allowed)
        stop.set()
        t.join()


def test_pick_prefers_whole_idle_cores():
    """SMT-aware choice: a CPU whose sibling is busy ranks as busy, and one CPU per core is taken
    before any sibling pair (sysfs siblings mocked: cores (0, 4), (1, 5), (2, 6), (3, 7))."""
    sib = {c: sorted({c, c ^ 4}) for c in range(8)}
    orig = A._siblings
    A._siblings = lambda c: sib[c]
    try:
        busy = {0: 0.0, 4: 0.9, 1: 0.0, 5: 0.0, 2: 0.1, 6: 0.0, 3: 0.0, 7: 0.0}
        assert A._pick(list(range(8)), busy, 3, smt=True) == [1, 3, 6]  # core (0,4) is busy; one per core
        assert A._pick(list(range(8)), busy, 3, smt=False) == [0, 1, 3]
        assert A._pick(list(range(8)), busy, 6, smt=True) == [1, 2, 3, 5, 6, 7]  # siblings once cores run out
    finally:
        A._siblings = orig

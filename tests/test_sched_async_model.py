"""integration/0003 (asynchronous host reduce entries) against oneCCL's
schedule progress rule, modelled (CPU).

oneCCL's progress loop (src/sched/sched.cpp:440-490) starts every entry in
order and holds back the entries after an entry only when that entry is a
barrier (sched->add_barrier() marks the last entry added, sched.cpp:596-602;
wait_value_entry is constructed as one, wait_value_entry.hpp:33).  A
reduce_local_entry that completes asynchronously therefore lets the entries
after it start while it still writes inout_buf / reads in_buf -- unless it is
a barrier itself.  The patch keeps it asynchronous only then
(reduce_local_entry::start: `if (!is_barrier())` completes before returning),
and batch_reduce_entry does the same.

This test runs the loop over the entry sequences of the reference's
reduce_local_entry call sites and reports every entry that starts while a
conflicting reduce is in flight.  With the guard there are none; without it
(round 2's patch) the ring RMA allreduce (allreduce_rma.cpp:325-410: the next
write_entry sends the block just reduced) and the direct reduce-scatter
(reduce_scatter.cpp:120-135: the next recv_entry refills tmp_buf) race.  The
patch text itself is checked for the guard too.
"""
from __future__ import annotations

from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


class Entry:
    def __init__(self, kind, reads=(), writes=(), polls=0, barrier=False):
        self.kind, self.reads, self.writes = kind, set(reads), set(writes)
        self.polls = polls          # update() calls before an asynchronous entry completes
        self.barrier = barrier
        self.status = "not_started"

    def start(self, guard):
        if self.kind == "reduce" and guard and not self.barrier:
            self.status = "complete"  # reduce_local_entry: complete before returning
        elif self.polls == 0:
            self.status = "complete"
        else:
            self.status = "started"

    def update(self):
        self.polls -= 1
        if self.polls <= 0:
            self.status = "complete"


class Sched:
    def __init__(self):
        self.entries = []

    def add(self, e):
        self.entries.append(e)
        return e

    def add_barrier(self):  # sched.cpp:596-602: the last entry becomes a barrier
        if self.entries:
            self.entries[-1].barrier = True

    def run(self, guard, max_passes=10_000):
        """sched.cpp:440-490; returns the hazards seen (entry index, buffer)."""
        hazards = []
        start_idx = 0
        for _ in range(max_passes):
            if start_idx >= len(self.entries):
                return hazards
            for idx in range(start_idx, len(self.entries)):
                e = self.entries[idx]
                if e.status == "not_started":
                    for r in self.entries[:idx]:  # a reduce in flight that this entry conflicts with
                        if r.kind == "reduce" and r.status == "started":
                            clash = (e.reads & r.writes) | (e.writes & (r.reads | r.writes))
                            hazards += [(idx, b) for b in sorted(clash)]
                    e.start(guard)
                elif e.status == "started":
                    e.update()
                if idx == start_idx and e.status == "complete":
                    start_idx += 1
                elif e.barrier and (e.status != "complete" or start_idx != idx + 1):
                    break
        raise AssertionError("schedule did not finish")


def ring_rma_allreduce(P=4):
    """allreduce_rma.cpp:325-410 (reduce-scatter part and allgather part)."""
    s = Sched()
    blk = 0
    for idx in range(P - 1):
        s.add(Entry("write", reads={f"recv[{blk}]"}, polls=2))
        s.add(Entry("write", reads={"flag"}, polls=1))
        s.add(Entry("wait_value", polls=3, barrier=True))   # wait_value_entry.hpp:33
        blk = (blk + P - 1) % P
        s.add(Entry("reduce", reads={f"tmp[{blk}]"}, writes={f"recv[{blk}]"}, polls=4))
    for idx in range(P - 1):                                 # allgather
        s.add(Entry("write", reads={f"recv[{blk}]"}, polls=2))
        s.add(Entry("wait_value", polls=1, barrier=True))
        blk = (blk + P - 1) % P
    return s


def direct_reduce_scatter(P=4):
    """reduce_scatter.cpp:120-135."""
    s = Sched()
    for idx in range(1, P):
        s.add(Entry("send", reads={f"send[{idx}]"}, polls=2))
        s.add(Entry("recv", writes={"tmp"}, polls=2))
        s.add_barrier()
        s.add(Entry("reduce", reads={"tmp"}, writes={"recv"}, polls=4))
    return s


def barrier_after_reduce(P=4):
    """allreduce.cpp:122-124, 211-218, 605-607; reduce.cpp:153-155, 223-230:
    every reduce_local_entry followed by add_barrier() before the next use."""
    s = Sched()
    for idx in range(1, P):
        s.add(Entry("recv", writes={"tmp"}, polls=2))
        s.add_barrier()
        s.add(Entry("reduce", reads={"tmp"}, writes={"recv"}, polls=4))
        s.add_barrier()
        s.add(Entry("send", reads={"recv"}, polls=2))
    return s


@pytest.mark.parametrize("build", [ring_rma_allreduce, direct_reduce_scatter, barrier_after_reduce])
def test_guarded_async_reduce_has_no_hazard(build):
    assert build().run(guard=True) == []


@pytest.mark.parametrize("build", [ring_rma_allreduce, direct_reduce_scatter])
def test_unguarded_async_reduce_races(build):
    """Round 2's patch (always asynchronous): the model finds the race ADVICE
    r2 reported, so the guard is what removes it."""
    assert build().run(guard=False) != []


def test_barrier_reduce_stays_asynchronous():
    """Where a barrier follows, the reduce is still polled (the worker is
    free for other schedules meanwhile)."""
    s = barrier_after_reduce()
    s.entries[2].start(guard=True)
    assert s.entries[2].status == "started"


def test_patch_and_entry_carry_the_guard():
    p = (ROOT / "integration" / "0003-async-host-reduce-entries.patch").read_text()
    assert "+    if (!is_barrier()) {" in p and "+        ccl_comp_request_wait(comp_req);" in p
    e = (ROOT / "integration" / "src" / "sched" / "entry" / "batch_reduce_entry.hpp").read_text()
    assert "if (!is_barrier()) {" in e
    f = (ROOT / "integration" / "0004-nreduce-fused-fanin.patch").read_text()
    # 0004 adds the batch entry between two barriers, so it stays asynchronous
    i = f.index("create<batch_reduce_entry>")
    assert "add_barrier();" in f[i:i + 300]

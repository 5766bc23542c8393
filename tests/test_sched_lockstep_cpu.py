"""Lockstep scheduling across TP ranks: every rank runs its own scheduler copy on
the requests rank 0 broadcasts, so any wall-clock decision (SJF aging, prefill batching hold) could
pick different batches on different ranks and desynchronise the collectives.  In lockstep mode the
aging is counted in schedule() calls, identical on every rank."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from ome_amd.runtime.page_pool import PagePool, ReqSlotPool
from ome_amd.runtime.request import Request, SamplingParams
from ome_amd.runtime.scheduler import Scheduler


def _sched(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        s = Scheduler(PagePool(400), ReqSlotPool(33, 64), 16, max_running=32, chunked_prefill_size=64,
                      max_context=1000)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return s


def _trace(s, reqs, steps=12):
    for r in reqs:
        s.add(r)
    out = []
    for _ in range(steps):
        b = s.schedule()
        if b is None:
            out.append(None)
            continue
        out.append([(c.req.rid, c.start, c.length) for c in b.chunks])
        s.commit(b, [1] * len(b.chunks), None, 0.0, set())
    return out


def _burst(old_arrival: float):
    reqs = [Request(prompt_ids=list(range(n)), params=SamplingParams(max_new_tokens=30), rid=f"r{i}")
            for i, n in enumerate([120, 10, 70, 20, 40, 15])]
    for r in reqs:
        r.arrival_time = old_arrival
    return reqs


def test_lockstep_aging_ignores_wall_clock():
    """Leader: the head request looks 10 s old; follower: brand new.  With wall-clock aging the two
    copies admit different requests; in lockstep mode they schedule identically."""
    import time

    now = time.perf_counter()
    lead, fol = _sched(), _sched()
    lead.lockstep = fol.lockstep = True
    assert _trace(lead, _burst(now - 10.0)) == _trace(fol, _burst(now))
    # the failure mode this guards against: the same two copies WITHOUT lockstep diverge
    lead, fol = _sched(), _sched()
    assert _trace(lead, _burst(now - 10.0)) != _trace(fol, _burst(now))


def test_lockstep_aging_still_ages():
    """A long head request is admitted within OME_SJF_AGE_STEPS schedule() calls even while short
    requests keep arriving."""
    s = _sched(OME_SJF_AGE_STEPS=3)
    s.lockstep = True
    head = Request(prompt_ids=list(range(60)), params=SamplingParams(max_new_tokens=50), rid="long")
    s.add(head)
    admitted_at = None
    for step in range(10):
        s.add(Request(prompt_ids=list(range(40)), params=SamplingParams(max_new_tokens=50), rid=f"s{step}"))
        b = s.schedule()
        if b is not None:
            if any(c.req.rid == "long" for c in b.chunks):
                admitted_at = step
                break
            s.commit(b, [1] * len(b.chunks), None, 0.0, set())
    assert admitted_at is not None and admitted_at <= 4


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    # the ranks disagree on the wall-clock bound: rank 0 ages everything at once, rank 1 never
    os.environ["OME_SJF_AGE_MS"] = "0" if rank == 0 else "1000000"
    from ome_amd.runtime.engine import Engine, EngineArgs

    eng = Engine(EngineArgs(model="tiny-llama", tp_size=world, device="cpu", max_running_requests=8,
                            context_length=256, dtype="float32", chunked_prefill_size=48))
    assert eng.scheduler.lockstep
    seen = []
    orig = eng.scheduler.schedule

    def rec():
        b = orig()
        seen.append(None if b is None else [(c.req.rid, c.start, c.length) for c in b.chunks])
        return b

    eng.scheduler.schedule = rec
    if rank == 0:
        prompts = [[3 + j for j in range(n)] for n in (90, 12, 50, 20, 33, 8)]
        eng.generate(prompts, SamplingParams(max_new_tokens=6, ignore_eos=True))
        eng.stop_group()
    else:
        eng.run_forever()
    q.put((rank, [s for s in seen if s is not None]))


@pytest.mark.timeout(300)
def test_tp2_ranks_schedule_identical_batches():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] and got[0] == got[1]

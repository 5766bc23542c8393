"""Row-count-aware mixed-step chunk sizing (runtime/step_cost.py): the chooser picks the prefill
chunk that lands M = decodes + prompt tokens on the cheap side of the GEMM staircase, defers a
tiny expensive remainder at most ``max_defer`` steps, and the scheduler applies it only to mixed
steps with decodes riding along."""
from ome_amd.runtime.page_pool import PagePool, ReqSlotPool
from ome_amd.runtime.request import Request, SamplingParams
from ome_amd.runtime.scheduler import Scheduler
from ome_amd.runtime.step_cost import StepCost


def _stairs(max_rows=4096, tile=256, per_tile=100.0, base=50.0):
    """t(M) = base + per_tile * ceil(M / tile): a pure tile-quantisation staircase."""
    rows = list(range(16, max_rows + 1, 16))
    sc = StepCost.from_measurements(rows, [base + per_tile * -(-m // tile) for m in rows], max_rows,
                                    slack=256, defer_ratio=1.3, max_defer=1)
    sc.min_avail = 0   # the unit tests exercise the cut itself
    return sc


def test_table_lookup_rounds_up_to_grid():
    sc = _stairs()
    assert sc.at(0) == 0.0
    assert sc.at(1) == sc.at(16) == sc.at(256) == 150.0
    assert sc.at(257) == 250.0
    assert sc.at(8192) > sc.at(4096)   # linear extrapolation past the table


def test_choose_cuts_at_tile_boundary():
    sc = _stairs()
    # 256 decodes + 300 prompt tokens: M = 556 would open a third tile for 44 tokens; cut at 512
    assert sc.choose(256, 300, 2048) == 256
    # exactly on a boundary: take everything
    assert sc.choose(256, 768, 2048) == 768
    # 240 decodes: the boundary is at 272 prompt tokens
    assert sc.choose(240, 400, 2048) == 272
    # never more than the cap, never leaves more than `slack` behind
    p = sc.choose(256, 5000, 2048)
    assert p <= 2048 and p >= 2048 - 256


def test_defer_tiny_remainder_once():
    sc = _stairs()
    # 20 prompt tokens would open a whole new tile: defer once, then take them
    assert sc.choose(256, 20, 2048, deferred=0) == 0
    assert sc.choose(256, 20, 2048, deferred=1) == 20
    # the same 20 tokens inside the decode rows' partially filled tile cost nothing: take them
    assert sc.choose(200, 20, 2048, deferred=0) == 20


def test_from_measurements_keeps_real_spikes():
    rows = [16 * i for i in range(1, 33)]
    us = [100.0] * 32
    us[17] = 300.0   # M = 288 routed onto a bad plan
    sc = StepCost.from_measurements(rows, us, 512)
    assert sc.at(288) == 300.0 and sc.at(320) == 100.0


def _sched(cost):
    s = Scheduler(PagePool(4000), ReqSlotPool(65, 256), 16, max_running=64, chunked_prefill_size=2048,
                  max_context=4096, enable_mixed_chunk=True)
    s.cost = cost
    return s


def test_scheduler_sizes_mixed_steps():
    sc = _stairs(tile=64, per_tile=100.0)
    s = _sched(sc)
    # 40 decoding requests
    for i in range(40):
        r = Request(prompt_ids=[1] * 8, params=SamplingParams(max_new_tokens=1000, ignore_eos=True), rid=f"d{i}")
        s.add(r)
    b = s.schedule()
    s.commit(b, [2] * len(b.chunks), None, 0.0, set())
    assert s._decode_rows() == 40
    # a 100-token prompt arrives: 40 + 100 = 140 rows would open a third 64-row tile for 12
    # tokens; the step cuts the chunk so M ends on a tile boundary
    s.add(Request(prompt_ids=[3] * 100, params=SamplingParams(max_new_tokens=4), rid="p"))
    b = s.schedule()
    pf = [c for c in b.chunks if c.req.rid == "p"]
    dec = [c for c in b.chunks if c.req.rid != "p"]
    assert len(dec) == 40 and (40 + pf[0].length) % 64 == 0 and pf[0].length < 100
    first = pf[0].length
    s.commit(b, [2] * len(b.chunks), None, 0.0, set())
    # the rest follows in the next steps, each again ending on a boundary or finishing the prompt
    done = first
    for _ in range(4):
        b = s.schedule()
        pf = [c for c in b.chunks if c.req.rid == "p"]
        if pf:
            assert pf[0].start == done
            done += pf[0].length
            assert (40 + pf[0].length) % 64 == 0 or done == 100
        s.commit(b, [2] * len(b.chunks), None, 0.0, set())
        if done == 100:
            break
    assert done == 100


def test_scheduler_without_decodes_uses_full_chunk():
    s = _sched(_stairs(tile=64))
    s.add(Request(prompt_ids=[3] * 100, params=SamplingParams(max_new_tokens=4), rid="p"))
    b = s.schedule()
    assert b.num_tokens == 100


def test_prefers_prompt_boundary_within_tolerance():
    sc = _stairs()
    sc.ttft_tol = 0.05
    # best grid cut is 256 (M = 512); a prompt ends at 250: nearly the same cost, no prompt split
    assert sc.choose(256, 300, 2048, bounds=[250, 300]) == 250
    # a boundary that would open a new tile is not worth it
    assert sc.choose(256, 300, 2048, bounds=[280, 300]) == 256
    sc.ttft_tol = 0.0
    assert sc.choose(256, 300, 2048, bounds=[250, 300]) == 256


def test_small_prefills_are_not_cut():
    sc = _stairs()
    sc.min_avail = 768
    assert sc.choose(256, 300, 2048) == 300      # below min_avail: everything, no cut
    assert sc.choose(256, 20, 2048) == 20        # ... and no deferral
    assert sc.choose(256, 1300, 2048) == 1280    # large: cut at the tile boundary (M = 1536)

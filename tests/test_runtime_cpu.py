"""Runtime (scheduler / paged KV / prefix cache / engine) on CPU with the reference ops."""
import random

import pytest
import torch

from ome_amd.bench.scenarios import Scenario, validate
from ome_amd.models.config import ModelConfig, preset, rope_cos_sin
from ome_amd.ops import reference as ref
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.page_pool import PagePool, ReqSlotPool
from ome_amd.runtime.prefix_cache import PrefixCache
from ome_amd.runtime.request import Request, SamplingParams
from ome_amd.runtime.scheduler import Scheduler


@pytest.fixture(scope="module")
def eng():
    return Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=8, chunked_prefill_size=48,
                             context_length=512))


def test_engine_generates(eng):
    reqs = eng.generate([[5, 6, 7], list(range(3, 90))], SamplingParams(max_new_tokens=5, ignore_eos=True))
    assert [len(r.output_ids) for r in reqs] == [5, 5]
    assert all(r.ttft is not None and r.ttft >= 0 for r in reqs)


def test_chunked_prefill_equivalence():
    """Chunk size must not change greedy outputs (same math, different batching)."""
    prompts = [list(range(10, 10 + n)) for n in (30, 70, 5)]
    outs = []
    for chunk in (16, 512):
        e = Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=8, chunked_prefill_size=chunk,
                              context_length=512, disable_radix_cache=True))
        outs.append([r.output_ids for r in e.generate(prompts, SamplingParams(max_new_tokens=6, ignore_eos=True))])
    assert outs[0] == outs[1]


def test_prefix_cache_hits_and_determinism(eng):
    p = list(range(200, 260))
    a = eng.generate([p], SamplingParams(max_new_tokens=4, ignore_eos=True))[0]
    b = eng.generate([p], SamplingParams(max_new_tokens=4, ignore_eos=True))[0]
    assert b.num_prefix_hit == 48 and a.output_ids == b.output_ids


def test_decode_matches_full_recompute():
    e = Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=4, context_length=256,
                          disable_radix_cache=True))
    r = e.generate([[9, 8, 7, 6]], SamplingParams(max_new_tokens=6, ignore_eos=True))[0]
    r2 = e.generate([r.prompt_ids + r.output_ids[:-1]], SamplingParams(max_new_tokens=1, ignore_eos=True))[0]
    assert r2.output_ids[0] == r.output_ids[-1]


def test_preemption_under_kv_pressure():
    pages, slots = PagePool(12), ReqSlotPool(9, 64)
    s = Scheduler(pages, slots, 16, max_running=8, chunked_prefill_size=1000, max_context=1000)
    reqs = [Request(prompt_ids=list(range(40)), params=SamplingParams(max_new_tokens=200)) for _ in range(3)]
    for r in reqs:
        s.add(r)
    b = s.schedule()
    assert b.mode == "prefill" and len(b.chunks) == 3  # 3 x 3 pages = 9 of 11
    s.commit(b, [1, 1, 1], None, 0.0, set())
    steps = 0
    while s.num_running and steps < 100:
        b = s.schedule()
        if b is None:
            break
        s.commit(b, [1] * len(b.chunks), None, 0.0, set())
        steps += 1
    assert s.num_preemptions >= 1
    assert pages.num_free + sum(len(r.pages) for r in s.running) == 11


def test_decode_batch_drops_requests_preempted_while_scheduling():
    """The newest request needs a page, the only victim is an older one already picked for this
    decode step: the step must not carry the preempted (page-less) request."""
    pages, slots = PagePool(5), ReqSlotPool(9, 64)
    s = Scheduler(pages, slots, 16, max_running=8, chunked_prefill_size=1000, max_context=1000)
    a = Request(prompt_ids=list(range(20)), params=SamplingParams(max_new_tokens=50))
    b = Request(prompt_ids=list(range(32)), params=SamplingParams(max_new_tokens=50))
    s.add(a)
    s.add(b)
    bt = s.schedule()
    assert len(bt.chunks) == 2 and pages.num_free == 0
    s.commit(bt, [1, 1], None, 0.0, set())
    bt = s.schedule()
    assert bt.mode == "decode" and [c.req for c in bt.chunks] == [b]
    assert a.state.name == "WAITING" and s.num_preemptions == 1
    assert all(len(c.req.pages) * 16 >= c.req.seq_len for c in bt.chunks)


def test_sjf_admission_with_aging(monkeypatch):
    """A burst is admitted shortest-prompt first within the chunk budget; a request older than the
    aging bound (or preempted) goes first regardless of length."""
    import time as _time

    pages, slots = PagePool(200), ReqSlotPool(17, 64)
    s = Scheduler(pages, slots, 16, max_running=16, chunked_prefill_size=100, max_context=1000)
    assert s.policy == "sjf"
    lens = [90, 10, 60, 20, 30]
    reqs = [Request(prompt_ids=list(range(n)), params=SamplingParams(max_new_tokens=4)) for n in lens]
    for r in reqs:
        s.add(r)
    b = s.schedule()
    # budget 100: 10 + 20 + 30 whole, then the first 40 tokens of the 60-token prompt
    assert [len(c.req.prompt_ids) for c in b.chunks] == [10, 20, 30, 60] and b.chunks[-1].length == 40
    # aging: the 90-token head has waited past the bound -> admitted before the 60-token one
    s2 = Scheduler(PagePool(200), ReqSlotPool(17, 64), 16, max_running=16, chunked_prefill_size=100,
                   max_context=1000)
    old = Request(prompt_ids=list(range(90)), params=SamplingParams(max_new_tokens=4))
    old.arrival_time = _time.perf_counter() - 10.0
    young = Request(prompt_ids=list(range(60)), params=SamplingParams(max_new_tokens=4))
    s2.add(old)
    s2.add(young)
    assert [len(c.req.prompt_ids) for c in s2.schedule().chunks][0] == 90
    # fifo policy keeps arrival order
    monkeypatch.setenv("OME_SCHED_POLICY", "fifo")
    s3 = Scheduler(PagePool(200), ReqSlotPool(17, 64), 16, max_running=16, chunked_prefill_size=100,
                   max_context=1000)
    for n in (50, 10):
        s3.add(Request(prompt_ids=list(range(n)), params=SamplingParams(max_new_tokens=4)))
    assert [len(c.req.prompt_ids) for c in s3.schedule().chunks] == [50, 10]


def test_loadgen_calibrated_prompt_length():
    from ome_amd.bench.loadgen import PromptFactory

    pf = PromptFactory(None, 0)
    pf.calibrate([(50, 50 * 4.6 + 12), (400, 400 * 4.6 + 12)])   # byte-level server tokenizer
    text = pf.make(480, random.Random(1))
    assert abs(len(text.split()) * 4.6 + 12 - 480) < 6
    a, b = pf.make(100, random.Random(1)), pf.make(100, random.Random(2))
    assert a != b


def test_stop_conditions():
    pages, slots = PagePool(100), ReqSlotPool(9, 64)
    s = Scheduler(pages, slots, 16, max_running=8, chunked_prefill_size=1000, max_context=1000)
    r = Request(prompt_ids=[1, 2, 3], params=SamplingParams(max_new_tokens=10))
    s.add(r)
    b = s.schedule()
    done = s.commit(b, [2], None, 0.0, eos_ids={2})
    assert done == [r] and r.finish_reason == "stop" and pages.num_free == 99


def test_prefix_cache_unit():
    pool = PagePool(20)
    pc = PrefixCache(pool, 4)
    toks = list(range(12))
    pages = pool.alloc(3)
    kept = pc.insert(toks, pages)
    assert kept == set(pages)
    assert pc.match(toks[:11]) == pages[:2]
    pc.release(pages[:2])
    assert pc.evict(5) == 3 and pc.num_pages == 0


def test_prefix_cache_eviction_lru_and_scales():
    """Eviction pops least-recently-used unpinned pages (deepest first among equals), never a
    pinned one, and stays cheap with a pool full of cached prefixes (the e2e sweep found
    per-allocation full sorts stalling the engine once ~120k pages were cached)."""
    import time as _t

    pool = PagePool(200_001)
    pc = PrefixCache(pool, 4)
    seqs = []
    for r in range(25_000):            # 25k cached 2-page prefixes = 50k cached pages
        toks = [r * 8 + j for j in range(8)]
        pages = pool.alloc(2)
        pc.insert(toks, pages)
        seqs.append((toks, pages))
    hot = pc.match(seqs[0][0])         # pin the oldest prefix: it must survive
    t0 = _t.perf_counter()
    freed = sum(pc.evict(4) for _ in range(2000))
    assert _t.perf_counter() - t0 < 1.0
    assert freed == 8000 and all(p in pc.meta for p in hot)
    # the 4000 oldest unpinned prefixes went first; within a prefix the deeper page first
    assert seqs[1][1][1] not in pc.meta and seqs[1][1][0] not in pc.meta
    assert seqs[4001][1][0] in pc.meta
    pc.release(hot)                    # unpinned, but recently used: not the next victim
    assert pc.evict(1) == 1 and seqs[4001][1][1] not in pc.meta and all(p in pc.meta for p in hot)


def test_prefix_cache_image_digest_salt():
    """Same token ids (placeholder-id collision forced), different pixels: no KV page sharing
    from the first image position on; text pages before the image stay shared."""
    from ome_amd.multimodal.inputs import MMInput
    from ome_amd.runtime.scheduler import _mm_salt

    pool = PagePool(40)
    pc = PrefixCache(pool, 4)
    toks = list(range(8)) + [777] * 8 + [1, 2, 3, 4]
    a = MMInput(torch.zeros(4, 6), [(1, 2, 2)], [(8, 8)])
    b = MMInput(torch.ones(4, 6), [(1, 2, 2)], [(8, 8)])
    pages = pool.alloc(5)
    pc.insert(toks, pages, *_mm_salt(type("R", (), {"mm": a})()))
    got_b = pc.match(toks, *_mm_salt(type("R", (), {"mm": b})()))
    assert got_b == pages[:2]                   # only the two text pages before the image
    pc.release(got_b)
    got_a = pc.match(toks, *a.cache_key())
    assert got_a == pages                       # same image: full reuse
    pc.release(got_a)
    assert pc.match(toks) == pages[:2]          # a text-only request never sees image pages


def test_scenarios():
    rng = random.Random(0)
    for s in ["N(480,240)/(300,150)", "D(100,100)", "U(10,20)/(5,6)", "E(128)", "I(512,512)"]:
        i, o = Scenario.parse(s).sample(rng)
        assert i >= 1
    assert validate("D(100,100)") and not validate("E(64)", "text-to-text")
    assert not validate("D(100,100)junk")
    with pytest.raises(ValueError):
        Scenario.parse("X(1)")


def test_rope_llama3_scaling_matches_hf_formula():
    cfg = preset("llama-3.1-8b")
    cs = rope_cos_sin(cfg, 16)
    assert cs.shape == (16, 128)
    assert torch.allclose(cs[0, :64], torch.ones(64))


def test_model_config_from_reference_fixtures():
    import json
    import os

    fx = "/root/reference/pkg/hfutil/modelconfig/testdata"
    if not os.path.isdir(fx):
        pytest.skip("reference fixtures not mounted")
    c = ModelConfig.from_hf(json.load(open(f"{fx}/llama3.json")))
    assert (c.hidden_size, c.num_layers, c.num_kv_heads) == (8192, 80, 8)
    d = ModelConfig.from_hf(json.load(open(f"{fx}/deepseek_v3.json")))
    assert d.is_moe and d.is_mla and d.num_experts == 256 and d.num_experts_per_tok == 8


def test_reference_attention_consistency():
    """paged_prefill with q_len==1 rows equals paged_decode."""
    torch.manual_seed(0)
    Hq, Hkv, D, P = 8, 2, 128, 16
    kc = torch.randn(10, Hkv, P, D, dtype=torch.bfloat16)
    vc = torch.randn(10, Hkv, D, P, dtype=torch.bfloat16)
    bt = torch.tensor([[1, 2, 3], [4, 5, 6]], dtype=torch.int32)
    sl = torch.tensor([40, 17], dtype=torch.int32)
    q = torch.randn(2, Hq, D, dtype=torch.bfloat16)
    a = ref.paged_decode(q, kc, vc, bt, sl, 0.1)
    b = ref.paged_prefill(q, kc, vc, bt, torch.tensor([0, 1, 2]), sl, 0.1)
    assert torch.allclose(a.float(), b.float(), atol=1e-2)


def test_prefix_cache_keys_are_content_digests():
    """Chain keys are 128-bit BLAKE2b digests of the page contents: prompts that differ in any
    token of a page never share that page or anything after it."""
    pc = PrefixCache(PagePool(32), 4)
    a = list(range(100, 112))
    pages = pc.pool.alloc(3)
    pc.insert(a, pages)
    assert all(isinstance(h, bytes) and len(h) == 16 for h in pc.by_hash)
    b = a[:5] + [a[5] + 1] + a[6:]
    assert pc.match(b) == pages[:1]
    assert pc.match(a) == pages

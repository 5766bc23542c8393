"""End-to-end runtime on the GPU: HIP-graph decode must agree with eager prefill numerics."""
import pytest
import torch

from ome_amd.models.common import AttnMeta
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return Engine(EngineArgs(model="tiny-llama", device="cuda", max_running_requests=16, chunked_prefill_size=64,
                             context_length=1024))


def test_generate_and_graphs(eng):
    assert eng.runner.use_graph and eng.runner.graphs
    prompts = [[7 + i for i in range(n)] for n in (1, 5, 16, 17, 63, 200)]
    reqs = eng.generate(prompts, SamplingParams(max_new_tokens=12, ignore_eos=True))
    for r in reqs:
        assert len(r.output_ids) == 12 and r.finish_reason == "length"


def _hidden_prefill(eng, ids):
    """Final hidden of every position via a fresh eager prefill of the whole sequence."""
    run = eng.runner
    slot = run.slots.alloc()
    pages = run.pages.alloc(-(-len(ids) // run.P))
    run.slots.set_pages(slot, 0, pages)
    run.slots.flush()
    T = len(ids)
    dv = run.device
    t = lambda a: torch.tensor(a, dtype=torch.int32, device=dv)  # noqa: E731
    from ome_amd import ops

    meta = AttnMeta("prefill", t(list(range(T))), t([pages[p // run.P] * run.P + p % run.P for p in range(T)]),
                    run.slots.table.index_select(0, t([slot])), cu_q=t([0, T]), kv_lens=t([T]),
                    items=t(ops.prefill_work_items([T], [T])).view(-1, 2))
    h = run.model.forward(t(ids), meta, run.kv)
    run.pages.free(pages)
    run.slots.free(slot)
    return h


def test_decode_matches_prefill(eng):
    r = eng.generate([[11, 12, 13, 14, 15, 16, 17]], SamplingParams(max_new_tokens=20, ignore_eos=True))[0]
    seq = r.prompt_ids + r.output_ids
    h = _hidden_prefill(eng, seq[:-1])
    logits = eng.runner.model.compute_logits(h[-20:]).float()
    # greedy tokens produced by graph decode must be the argmax (or within bf16 noise of it)
    top = logits.argmax(-1).cpu().tolist()
    agree = sum(int(a == b) for a, b in zip(top, r.output_ids))
    assert agree >= 18, (top, r.output_ids)


def test_prefix_cache_reuse(eng):
    p = list(range(100, 180))
    a = eng.generate([p], SamplingParams(max_new_tokens=6, ignore_eos=True))[0]
    b = eng.generate([p], SamplingParams(max_new_tokens=6, ignore_eos=True))[0]
    assert b.num_prefix_hit >= 64
    assert a.output_ids == b.output_ids


def test_sampling_seeded(eng):
    sp = SamplingParams(max_new_tokens=8, temperature=0.9, top_p=0.9, top_k=50, seed=123, ignore_eos=True)
    a = eng.generate([[1, 2, 3]], sp)[0]
    b = eng.generate([[1, 2, 3]], SamplingParams(**{**sp.__dict__}))[0]
    assert a.output_ids == b.output_ids

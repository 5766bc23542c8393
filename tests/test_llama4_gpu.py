"""Llama 4 class model (chunked attention on RoPE layers, NoPE temperature tuning, sigmoid-scaled
top-1 experts + shared expert) through the gfx950 kernels with HIP-graph decode: graph decode must
agree with an eager prefill recompute, across the 64-token chunk boundary."""
import pytest

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_engine_gpu import _hidden_prefill

pytestmark = pytest.mark.gpu


def test_llama4_engine_graph_decode_matches_prefill():
    eng = Engine(EngineArgs(model="tiny-llama4", device="cuda", max_running_requests=8, context_length=512))
    m = eng.runner.model
    assert type(m).__name__ == "Llama4ForCausalLM" and m.windows[0] == -64 and m.windows[3] == -1
    assert eng.runner.use_graph
    prompts = [[11 + (i * 13 + j) % 900 for j in range(5 + 70 * i)] for i in range(3)]  # cross a chunk edge
    reqs = eng.generate(prompts, SamplingParams(max_new_tokens=16, ignore_eos=True))
    for r in reqs:
        assert len(r.output_ids) == 16
        seq = r.prompt_ids + r.output_ids
        h = _hidden_prefill(eng, seq[:-1])
        top = m.compute_logits(h[-16:]).float().argmax(-1).cpu().tolist()
        assert sum(int(a == b) for a, b in zip(top, r.output_ids)) >= 14, (top, r.output_ids)

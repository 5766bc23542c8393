"""GPT-OSS class model through the gfx950 kernels (head_dim 64, attention sinks, sliding windows,
biased grouped-GEMM experts with the clamped SwiGLU) with HIP-graph decode."""
import pytest

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_engine_gpu import _hidden_prefill

pytestmark = pytest.mark.gpu


def test_gpt_oss_engine_graph_decode_matches_prefill():
    eng = Engine(EngineArgs(model="tiny-gpt-oss", device="cuda", max_running_requests=8, context_length=512))
    m = eng.runner.model
    assert type(m).__name__ == "GptOssForCausalLM" and m.D == 64
    prompts = [[11 + (i * 13 + j) % 900 for j in range(5 + 40 * i)] for i in range(3)]  # > window for the last
    reqs = eng.generate(prompts, SamplingParams(max_new_tokens=16, ignore_eos=True))
    for r in reqs:
        assert len(r.output_ids) == 16
        seq = r.prompt_ids + r.output_ids
        h = _hidden_prefill(eng, seq[:-1])
        top = m.compute_logits(h[-16:]).float().argmax(-1).cpu().tolist()
        assert sum(int(a == b) for a, b in zip(top, r.output_ids)) >= 14, (top, r.output_ids)

"""DeciLM / Nemotron-NAS in bf16 on gfx950: per-layer KV-head paged caches, no-op and linear
blocks, graph decode -- against the fp32 transcription of ``tests/test_decilm_cpu.py``."""
import pytest
import torch

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_decilm_cpu import _checkpoint, _ref_logits
from tests.test_engine_gpu import _hidden_prefill

pytestmark = pytest.mark.gpu


def test_decilm_on_gpu(tmp_path):
    w = _checkpoint(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=8, context_length=512))
    m = eng.runner.model
    assert eng.runner.use_graph
    ids = [(7 * i + 3) % 290 + 5 for i in range(40)]
    got = m.compute_logits(_hidden_prefill(eng, ids)).float().cpu()
    want = _ref_logits(w, ids)
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    reqs = eng.generate([ids, ids[:9]], SamplingParams(max_new_tokens=10, ignore_eos=True))
    for r in reqs:
        seq = r.prompt_ids + r.output_ids
        top = m.compute_logits(_hidden_prefill(eng, seq[:-1])[-10:]).float().argmax(-1).cpu().tolist()
        assert sum(int(a == b) for a, b in zip(top, r.output_ids)) >= 8, (top, r.output_ids)

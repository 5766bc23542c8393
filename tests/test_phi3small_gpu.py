"""Phi-3-small on gfx950 (bf16): the engine's greedy continuation and prefill logits track the
fp32 CPU restatement of tests/test_phi3small_cpu.py (block-sparse layers included)."""
import pytest
import torch

from ome_amd.runtime.engine import Engine, EngineArgs
from tests.test_phi3small_cpu import IDS, _checkpoint, _prefill_logits, _ref_logits

pytestmark = pytest.mark.gpu


def test_phi3small_bf16_on_gpu(tmp_path):
    w = _checkpoint(tmp_path)
    want = _ref_logits(w, IDS)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", dtype="bfloat16", max_running_requests=2,
                            context_length=256, cuda_graph=False))
    got = _prefill_logits(eng, IDS, [45]).cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.995, cos.min()
    assert (got.argmax(-1) == want.argmax(-1)).float().mean().item() > 0.9

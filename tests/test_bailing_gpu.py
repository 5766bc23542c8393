"""Bailing MoE (Ling) and XVERSE MoE on gfx950: the mapped checkpoints of ``test_bailing_cpu`` /
``test_xverse_cpu`` in bf16 (grouped
MFMA MoE GEMMs, fused shared expert, normalised head) with HIP-graph decode, every greedy token a
near-argmax of the fp32 transformers reference on the same prefix."""
import pytest
import torch

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_bailing_cpu import _models
from tests.test_xverse_cpu import _models as _xverse_models

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("family", ["bailing", "xverse"])
def test_bailing_on_gpu(tmp_path, family):
    hf = (_models if family == "bailing" else _xverse_models)(tmp_path)
    prompts = [[(7 * i + 3 + 5 * s) % 500 + 3 for i in range(12 + 20 * s)] for s in range(3)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=256))
    for p, r in zip(prompts, eng.generate(prompts, SamplingParams(max_new_tokens=8, ignore_eos=True))):
        with torch.no_grad():
            lp = torch.log_softmax(hf(torch.tensor([p + r.output_ids])).logits[0].float(), -1)
        lp = lp[len(p) - 1:len(p) - 1 + len(r.output_ids)]
        gap = [(lp[t].max() - lp[t, tok]).item() for t, tok in enumerate(r.output_ids)]
        assert r.output_ids[0] == int(lp[0].argmax()) and max(gap) < 0.05, gap

"""MiniCPM3 on gfx950: the (288, 256) MLA kernel instance with a partial head group (5 heads)
serving a tiny random checkpoint in bf16, against transformers fp32 greedy decoding."""
import pytest
import torch

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_minicpm3_cpu import _hf_model

pytestmark = pytest.mark.gpu


def test_minicpm3_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    prompts = [[(7 * i + 3 + 11 * s) % 500 + 3 for i in range(20 + 30 * s)] for s in range(3)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=512))
    reqs = eng.generate(prompts, SamplingParams(max_new_tokens=8, ignore_eos=True))
    for p, r in zip(prompts, reqs):
        with torch.no_grad():
            ref = hf.generate(torch.tensor([p]), max_new_tokens=8, do_sample=False)[0, len(p):].tolist()
        assert sum(int(a == b) for a, b in zip(r.output_ids, ref)) >= 6, (r.output_ids, ref)

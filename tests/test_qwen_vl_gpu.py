"""Qwen-VL vision tower + Resampler on gfx950 (bf16, varlen MFMA attention) against the fp32
restatement of tests/test_qwen_vl_cpu.py, and an image prompt through the engine."""
import pytest
import torch

from ome_amd.models.qwen_vl import preprocess_qwen_vl
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_qwen_vl_cpu import START, END, _checkpoint, _image, _visual_ref

pytestmark = pytest.mark.gpu


def test_qwen_vl_bf16_on_gpu(tmp_path):
    _, vis = _checkpoint(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", dtype="bfloat16", max_running_requests=2,
                            context_length=256, cuda_graph=False))
    m = eng.runner.model
    px = preprocess_qwen_vl(_image(), 56)
    want = _visual_ref(vis, px)
    got = m.encode_images(px).float().cpu()
    assert torch.nn.functional.cosine_similarity(got, want, dim=-1).min().item() > 0.995
    req = eng.make_mm_request([1, 9, START, END, 12, 7], [_image()], SamplingParams(max_new_tokens=4, ignore_eos=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    assert len(req.output_ids) == 4

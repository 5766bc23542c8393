"""Qwen2.5-VL on gfx950: the windowed vision tower (varlen MFMA attention over windows and images,
RMSNorm / SwiGLU kernels) in bf16 vs transformers fp32, and an image request served end to end."""
import numpy as np
import torch

import pytest

from ome_amd.multimodal.inputs import expand_image_tokens, preprocess_image
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_qwen2_5_vl_cpu import IMG, VE, VS, _hf_model, _image

pytestmark = pytest.mark.gpu


def test_qwen2_5_vl_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    img = _image(170, 230)
    pv, grid = preprocess_image(img)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=1024))
    m = eng.runner.model
    with torch.no_grad():
        want = hf.model.visual(torch.from_numpy(pv), grid_thw=torch.tensor([grid])).pooler_output.float()
    got = m.encode_images(torch.from_numpy(pv), [grid]).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.995, cos.min().item()
    prompt = [5, 9, 17, VS, IMG, VE, 33, 41, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=8, ignore_eos=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex, _ = expand_image_tokens(prompt, IMG, [grid], 2)
    t = torch.tensor([ex])
    with torch.no_grad():
        ref = hf.generate(t, pixel_values=torch.from_numpy(pv), image_grid_thw=torch.tensor([grid]),
                          mm_token_type_ids=(t == IMG).int(), max_new_tokens=8, do_sample=False)[0, len(ex):]
    agree = sum(int(a == b) for a, b in zip(req.output_ids, ref.tolist()))
    assert agree >= 6, (req.output_ids, ref.tolist())
    assert np.isfinite(np.array(req.output_ids)).all()

"""Qwen3-VL dense / MoE on gfx950: vision tower + deepstack features in bf16 against transformers
fp32, and an image request served end to end (interleaved M-RoPE rows, deepstack injection,
HIP-graph decode)."""
import pytest
import torch

from ome_amd.multimodal.inputs import expand_image_tokens, preprocess_image
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_qwen3_vl_cpu import IMG, VE, VS, _hf_model, _image

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("moe", [False, True])
def test_qwen3_vl_on_gpu(tmp_path, moe):
    hf = _hf_model(tmp_path, moe)
    img = _image(120, 90)
    pv, grid = preprocess_image(img, patch=16, min_pixels=65536, max_pixels=16777216, mean=(0.5,) * 3,
                                std=(0.5,) * 3)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=1024))
    m = eng.runner.model
    with torch.no_grad():
        out = hf.model.visual(torch.from_numpy(pv), grid_thw=torch.tensor([grid]))
    main, deep = m.encode_images(torch.from_numpy(pv), [grid])
    for a, b in [(main, out.pooler_output)] + list(zip(deep, out.deepstack_features)):
        cos = torch.nn.functional.cosine_similarity(a.float().cpu(), b.float(), dim=-1)
        assert cos.min().item() > 0.99, cos.min().item()
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
    assert sum(int(a == b) for a, b in zip(req.output_ids, ref.tolist())) >= 6, (req.output_ids, ref.tolist())

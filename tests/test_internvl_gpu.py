"""InternVL on gfx950: InternViT (varlen MFMA attention, LayerNorm kernels, layer scale) + pixel
shuffle + projector in bf16 against transformers fp32, and a two-image request (5 tiles)
served through the engine, in the original InternVLChatModel layout."""
import pytest
import torch

from ome_amd.models.internvl import preprocess_internvl
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_internvl_cpu import END, IMG, START, _hf_model, _image, _to_original_layout

pytestmark = pytest.mark.gpu


def test_internvl_on_gpu(tmp_path):
    src = tmp_path / "hf"
    src.mkdir()
    hf = _hf_model(src)
    _to_original_layout(src, tmp_path / "orig")
    imgs = [_image(0, 80, 60), _image(1, 100, 330)]
    px = torch.cat([preprocess_internvl(im, 112, 6) for im in imgs])
    eng = Engine(EngineArgs(model_path=str(tmp_path / "orig"), device="cuda", max_running_requests=4,
                            context_length=1024))
    m = eng.runner.model
    with torch.no_grad():
        want = torch.cat(list(hf.get_image_features(pixel_values=px, return_dict=True).pooler_output)).float()
    got = m.encode_images(px).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    req = eng.make_mm_request([1, 9, START, IMG, END, 33, 41, START, IMG, END, 12, 7], imgs,
                              SamplingParams(max_new_tokens=8, ignore_eos=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ex]), pixel_values=px, max_new_tokens=8, do_sample=False)[0, len(ex):]
    assert sum(int(a == b) for a, b in zip(req.output_ids, ref.tolist())) >= 6, (req.output_ids, ref.tolist())

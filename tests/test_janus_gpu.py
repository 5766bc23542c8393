"""Janus-Pro image understanding on gfx950: SigLIP tower (varlen MFMA attention) + aligner in
bf16 against transformers fp32, and a two-image request served through the engine."""
import pytest
import torch

from ome_amd.models.janus import preprocess_janus
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_janus_cpu import BOI, EOI, IMG, _hf_model, _image

pytestmark = pytest.mark.gpu


def test_janus_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    imgs = [_image(0), _image(1, 50, 90)]
    px = torch.cat([preprocess_janus(im, 64) for im in imgs])
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=512))
    m = eng.runner.model
    m.boi, m.eoi = BOI, EOI
    with torch.no_grad():
        want = torch.cat(list(hf.model.get_image_features(pixel_values=px).pooler_output)).float()
    got = m.encode_images(px).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    req = eng.make_mm_request([1, 9, BOI, IMG, EOI, 33, 41, BOI, IMG, EOI, 12, 7], imgs,
                              SamplingParams(max_new_tokens=8, ignore_eos=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ex]), pixel_values=px, max_new_tokens=8, do_sample=False,
                          generation_mode="text")[0, len(ex):]
    assert sum(int(a == b) for a, b in zip(req.output_ids, ref.tolist())) >= 6, (req.output_ids, ref.tolist())

"""LLaVA-NeXT on gfx950: CLIP tower + projector + anyres packing (unpad, newline) in bf16 against
transformers fp32, and an anyres request served through the engine."""
import pytest
import torch

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_llava_next_cpu import IMG, _hf_model, _hf_pixels, _image

pytestmark = pytest.mark.gpu


def test_llava_next_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    imgs = [_image(1, 40, 150)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=2048))
    m = eng.runner.model
    pv, sizes = _hf_pixels(imgs)
    req = eng.make_mm_request([1, 9, 17, IMG, 33, 41, 7], imgs, SamplingParams(max_new_tokens=8, ignore_eos=True))
    with torch.no_grad():
        want = hf.model.get_image_features(pixel_values=pv, image_sizes=sizes)
        want = torch.cat(list(getattr(want, "pooler_output", want))).float()
    got = m.encode_images(req.mm.pixel_values, req.mm.grid_thw).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    # tiny random weights give nearly flat distributions: every bf16 greedy choice must be a
    # near-argmax of the fp32 reference conditioned on the same prefix
    seq = torch.tensor([ex + req.output_ids])
    with torch.no_grad():
        logits = hf(seq, pixel_values=pv, image_sizes=sizes).logits[0].float()
    lp = torch.log_softmax(logits[len(ex) - 1:len(ex) - 1 + len(req.output_ids)], -1)
    gap = [(lp[t].max() - lp[t, tok]).item() for t, tok in enumerate(req.output_ids)]
    assert req.output_ids[0] == int(lp[0].argmax()) and max(gap) < 0.05, gap

"""Mistral 3 / Pixtral on gfx950: tower (2D RoPE, varlen MFMA attention, RMSNorm / SwiGLU kernels)
+ patch merger + projector in bf16 against transformers fp32, and a two-image request served
through the engine."""
import pytest
import torch

from ome_amd.models.mistral3 import preprocess_pixtral
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_mistral3_cpu import IMG, _hf_model, _hf_pixels, _image

pytestmark = pytest.mark.gpu


def test_mistral3_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    imgs = [_image(0, 80, 60), _image(1, 50, 110)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=512))
    m = eng.runner.model
    pix = [_hf_pixels(im) for im in imgs]
    Hm, Wm = max(p[1][0] for p in pix), max(p[1][1] for p in pix)
    pv = torch.zeros(2, 3, Hm, Wm)
    for i, (p, (H, W)) in enumerate(pix):
        pv[i, :, :H, :W] = p[:, :H, :W]
    sizes = torch.tensor([p[1] for p in pix])
    with torch.no_grad():
        want = torch.cat(list(hf.get_image_features(pixel_values=pv, image_sizes=sizes,
                                                    return_dict=True).pooler_output)).float()
    pre = [preprocess_pixtral(im, 112, 28, 14) for im in imgs]
    got = m.encode_images(torch.cat([r for r, _, _ in pre]), [(1, h, w) for _, h, w in pre]).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    req = eng.make_mm_request([1, 9, 17, IMG, 33, 41, IMG, 22, 7], imgs, SamplingParams(max_new_tokens=8,
                                                                                       ignore_eos=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    # teacher-forced: HF log-probs along the engine's own tokens (a near-tied step of the random
    # model may pick either token; every pick must be within bf16 noise of HF's argmax)
    seq = torch.tensor([ex + req.output_ids])
    with torch.no_grad():
        logits = hf(seq, pixel_values=pv, image_sizes=sizes).logits[0].float()
    lp = torch.log_softmax(logits[len(ex) - 1:len(ex) - 1 + len(req.output_ids)], -1)
    gap = [(lp[t].max() - lp[t, tok]).item() for t, tok in enumerate(req.output_ids)]
    assert req.output_ids[0] == int(lp[0].argmax()) and max(gap) < 0.1, gap

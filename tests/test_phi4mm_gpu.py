"""Phi-4-multimodal on gfx950: dynamic-HD SigLIP features (varlen MFMA attention over the valid
patches of each crop) in bf16 against transformers fp32, and a two-image request through the
engine (Phi-3 decoder path, partial rotary) with every greedy token a near-argmax of the fp32
reference on the same prefix."""
import pytest
import torch

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_phi4mm_cpu import IMG, _hf_inputs, _hf_model, _image

pytestmark = pytest.mark.gpu


def test_phi4mm_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    imgs = [_image(0, 80, 60), _image(1, 60, 110)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=1024))
    m = eng.runner.model
    m.crop = 56
    pre, pv, am, sizes = _hf_inputs(imgs)
    req = eng.make_mm_request([1, 9, IMG, 33, 41, IMG, 12, 7], [(p, g) for p, g in pre],
                              SamplingParams(max_new_tokens=8, ignore_eos=True))
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    ids = torch.tensor([ex])
    with torch.no_grad():
        emb = hf.model.embed_tokens(ids)
        want = hf.model.embed_tokens_extend(ids, emb, image_pixel_values=pv, image_sizes=sizes,
                                            image_attention_mask=am)[0][ids[0] == IMG].float()
    got = m.encode_images(req.mm.pixel_values, req.mm.grid_thw).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    eng.add_request(req)
    while not req.finished:
        eng.step()
    seq = torch.tensor([ex + req.output_ids])
    with torch.no_grad():
        logits = hf(seq, image_pixel_values=pv, image_sizes=sizes, image_attention_mask=am).logits[0].float()
    lp = torch.log_softmax(logits[len(ex) - 1:len(ex) - 1 + len(req.output_ids)], -1)
    gap = [(lp[t].max() - lp[t, tok]).item() for t, tok in enumerate(req.output_ids)]
    assert req.output_ids[0] == int(lp[0].argmax()) and max(gap) < 0.05, gap

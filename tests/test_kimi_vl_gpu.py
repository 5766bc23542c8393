"""Kimi-VL on gfx950: MoonViT tower (resampled positions, 2D rotary, varlen MFMA attention,
LayerNorm / GELU-tanh kernels) in bf16 against transformers' Kimi-K2.5 fp32, and a two-image
request through the engine (MLA decode over the latent cache, sigmoid grouped MoE) with every
greedy token a near-argmax of the fp32 reference on the same prefix."""
import pytest
import torch

from ome_amd.models.kimi_vl import preprocess_kimi_vl
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_kimi_vl_cpu import BOI, EOI, IMG, _hf_model, _image

pytestmark = pytest.mark.gpu


def test_kimi_vl_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    imgs = [_image(0, 80, 60), _image(1, 60, 110)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=1024))
    m = eng.runner.model
    pre = [preprocess_kimi_vl(im) for im in imgs]
    pv = torch.cat([torch.from_numpy(p) for p, _ in pre]).reshape(-1, 3, 14, 14)
    grid = torch.tensor([g for _, g in pre])
    with torch.no_grad():
        want = torch.cat(list(hf.model.get_image_features(pixel_values=pv, image_grid_thw=grid).pooler_output)).float()
    got = m.encode_images(pv.reshape(pv.shape[0], -1), [tuple(g) for g in grid.tolist()]).float().cpu()
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
    seq = torch.tensor([ex + req.output_ids])
    with torch.no_grad():
        logits = hf(seq, pixel_values=pv, image_grid_thw=grid).logits[0].float()
    lp = torch.log_softmax(logits[len(ex) - 1:len(ex) - 1 + len(req.output_ids)], -1)
    gap = [(lp[t].max() - lp[t, tok]).item() for t, tok in enumerate(req.output_ids)]
    assert req.output_ids[0] == int(lp[0].argmax()) and max(gap) < 0.05, gap

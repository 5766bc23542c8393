"""GLM-4.5V on gfx950: vision tower (grid-sampled positions, varlen MFMA attention, SwiGLU kernels)
in bf16 against transformers fp32, and a two-image request through the engine (M-RoPE over the
partial rotary half, sigmoid grouped MoE routing) with every greedy token a near-argmax of the
fp32 reference on the same prefix."""
import pytest
import torch

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_glm4v_cpu import BOI, EOI, IMG, _hf_model, _hf_pixels, _image

pytestmark = pytest.mark.gpu


def test_glm4v_on_gpu(tmp_path):
    hf = _hf_model(tmp_path)
    imgs = [_image(0, 80, 60), _image(1, 60, 110)]
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=1024))
    m = eng.runner.model
    pv, grid = _hf_pixels(imgs)
    with torch.no_grad():
        want = torch.cat(list(hf.model.get_image_features(pixel_values=pv, image_grid_thw=grid).pooler_output)).float()
    got = m.encode_images(pv, [tuple(g.tolist()) for g in grid]).float().cpu()
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
        logits = hf(seq, pixel_values=pv, image_grid_thw=grid, mm_token_type_ids=(seq == IMG).int()).logits[0].float()
    lp = torch.log_softmax(logits[len(ex) - 1:len(ex) - 1 + len(req.output_ids)], -1)
    gap = [(lp[t].max() - lp[t, tok]).item() for t, tok in enumerate(req.output_ids)]
    # bf16 engine vs fp32 HF: the sigmoid grouped router of the random MoE can flip an expert on a
    # near-tied score, so allow ONE step of larger drift after the first token (every other step
    # within 0.05 nats).  Its size depends on which expert flips: 1.51 nats with the fast varlen
    # vision-attention body, whose outputs differ from the generic body's by ~1 bf16 ulp
    # (profiles/r05_varlen_attn.md), 0 with the generic body (OME_VARLEN_FAST=0)
    assert req.output_ids[0] == int(lp[0].argmax()) and sorted(gap)[-2] < 0.05 and max(gap) < 2.5, gap

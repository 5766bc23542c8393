"""NVILA on gfx950 (bf16): the Dynamic-S2 SigLIP tower + chessboard 3x3-fold projector against
the fp32 restatement of tests/test_nvila_cpu.py, and an image request served through the engine
(every greedy choice a near-argmax of transformers' Qwen2 in fp32 on the same prefix)."""
import pytest
import torch

from ome_amd.models.nvila import preprocess_nvila
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_nvila_cpu import IMG, SCALES, _checkpoint, _features_ref, _image

pytestmark = pytest.mark.gpu


def test_nvila_on_gpu(tmp_path):
    llm, vt, proj = _checkpoint(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=2048))
    m = eng.runner.model
    img = _image()
    px, (rows, cols) = preprocess_nvila(img, SCALES, 84, 12)
    want = _features_ref(vt, proj, px, rows, cols)
    got = m.encode_images(px, [(rows, cols)]).float().cpu()
    cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
    assert cos.min().item() > 0.99, cos.min().item()
    req = eng.make_mm_request([1, 9, IMG, 12, 7, 40], [img], SamplingParams(max_new_tokens=6, ignore_eos=True))
    eng.add_request(req)
    while not req.finished:
        eng.step()
    s, n = req.mm.spans[0]
    ids = torch.tensor(req.prompt_ids + req.output_ids)
    with torch.no_grad():
        emb = llm.get_input_embeddings()(ids)
        emb[s:s + n] = want
        logits = llm(inputs_embeds=emb[None]).logits[0].float()
    L = len(req.prompt_ids)
    lp = torch.log_softmax(logits[L - 1:L - 1 + len(req.output_ids)], -1)
    gap = [(lp[t].max() - lp[t, tok]).item() for t, tok in enumerate(req.output_ids)]
    assert req.output_ids[0] == int(lp[0].argmax()) and max(gap) < 0.05, gap

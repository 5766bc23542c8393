"""CLIP embeddings on gfx950 (causal varlen attention for the text encoder, CLIP tower for images)
in bf16 against transformers fp32."""
import pytest
import torch

from ome_amd.models.llava import preprocess_clip
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams
from tests.test_clip_cpu import EOS, _hf, _image

pytestmark = pytest.mark.gpu


def test_clip_on_gpu(tmp_path):
    hf = _hf(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=77))
    prompts = [[1, 5, 9, 17, EOS], [1] + list(range(40, 100)) + [EOS]]
    reqs = [eng.make_request(p, SamplingParams(max_new_tokens=0)) for p in prompts]
    reqs.append(eng.make_mm_request([], [_image(0)], SamplingParams(max_new_tokens=0)))
    for r in reqs:
        r.is_embedding = True
        eng.add_request(r)
    while not all(r.finished for r in reqs):
        eng.step()
    with torch.no_grad():
        want = [torch.nn.functional.normalize(hf.get_text_features(input_ids=torch.tensor([p]), return_dict=True)
                                              .pooler_output[0], dim=-1) for p in prompts]
        want.append(torch.nn.functional.normalize(hf.get_image_features(
            pixel_values=preprocess_clip(_image(0), 56), return_dict=True).pooler_output[0], dim=-1))
    for r, w in zip(reqs, want):
        assert torch.nn.functional.cosine_similarity(torch.tensor(r.embedding), w, dim=0).item() > 0.995

"""CLIP embeddings (``models/clip.py``) against transformers (tiny random CLIPModel, fp32): text
features (causal encoder over packed prompts, first-EOS pooling, projection) and image features
(class token, post-LayerNorm, projection), L2-normalised, through the engine's embedding path and
the ``/v1/embeddings`` endpoint with an image item."""
import base64
import io

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.models.llava import preprocess_clip  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

EOS = 299


def _hf(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = dict(vocab_size=300, hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=2,
              max_position_embeddings=77, eos_token_id=EOS, bos_token_id=1, pad_token_id=0, projection_dim=64)
    vc = dict(hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=2, image_size=56,
              patch_size=14, projection_dim=64)
    m = T.CLIPModel(T.CLIPConfig(text_config=tc, vision_config=vc, projection_dim=64))
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
            elif "logit_scale" not in n:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    m.save_pretrained(tmp_path, safe_serialization=True)
    return m


def _image(seed=0):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (70, 50, 3), dtype=np.uint8))


def test_clip_text_and_image_embeddings(tmp_path):
    hf = _hf(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=77))
    assert type(eng.runner.model).__name__ == "CLIPModel" and eng.cfg.is_embedding
    prompts = [[1, 5, 9, 17, EOS], [1, 40, 41, 42, 43, 44, 45, EOS, 0], [1, EOS]]
    reqs = [eng.make_request(p, SamplingParams(max_new_tokens=0)) for p in prompts]
    img_req = eng.make_mm_request([], [_image(0)], SamplingParams(max_new_tokens=0))
    for r in reqs + [img_req]:
        r.is_embedding = True
        eng.add_request(r)
    while not all(r.finished for r in reqs + [img_req]):
        eng.step()
    with torch.no_grad():
        want = torch.stack([torch.nn.functional.normalize(
            hf.get_text_features(input_ids=torch.tensor([p]), return_dict=True).pooler_output[0], dim=-1)
            for p in prompts])
        want_img = torch.nn.functional.normalize(hf.get_image_features(
            pixel_values=preprocess_clip(_image(0), 56), return_dict=True).pooler_output[0], dim=-1)
    got = torch.tensor([r.embedding for r in reqs])
    assert torch.allclose(got, want, atol=1e-4), (got - want).abs().max()
    assert torch.allclose(torch.tensor(img_req.embedding), want_img, atol=1e-4)


def test_clip_embeddings_endpoint_with_image(tmp_path):
    from fastapi.testclient import TestClient

    from ome_amd.runtime.server import create_app

    hf = _hf(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=77))
    eng.start()
    try:
        buf = io.BytesIO()
        _image(3).save(buf, format="PNG")
        url = "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()
        r = TestClient(create_app(eng)).post("/v1/embeddings", json={"input": [{"image": url}, [1, 5, EOS]]}).json()
        assert len(r["data"]) == 2 and len(r["data"][0]["embedding"]) == 64
        with torch.no_grad():
            want = torch.nn.functional.normalize(hf.get_image_features(
                pixel_values=preprocess_clip(_image(3), 56), return_dict=True).pooler_output[0], dim=-1)
        assert torch.allclose(torch.tensor(r["data"][0]["embedding"]), want, atol=1e-4)
    finally:
        eng.shutdown()

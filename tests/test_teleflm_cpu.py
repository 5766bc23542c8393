"""Tele-FLM (``TeleFLMModel``) on CPU against transformers' Llama: with muP on, Tele-FLM's logits
equal a Llama whose embedding table is pre-scaled by ``input_mult``, times ``output_mult /
mup_scale_factor`` -- the identity this test checks (fp32, CPU reference ops).  No Tele-FLM class
is importable here, so parity with the remote code itself is unpinned."""
import json

import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models import build_model, model_class  # noqa: E402
from ome_amd.models.common import AttnMeta, PagedKVCache  # noqa: E402
from ome_amd.models.config import PRESETS, ModelConfig  # noqa: E402


def _forward(m, ids):
    T = len(ids)
    kv = PagedKVCache(m.cfg.num_layers, 8, m.tp.hkv, m.D, 16, m.dtype, "cpu")
    bt = torch.tensor([[1, 2, 3, 4]], dtype=torch.int32)
    meta = AttnMeta("prefill", torch.arange(T, dtype=torch.int32), torch.arange(16, 16 + T, dtype=torch.int32), bt,
                    cu_q=torch.tensor([0, T], dtype=torch.int32), kv_lens=torch.tensor([T], dtype=torch.int32),
                    items=torch.tensor([[0, 0]], dtype=torch.int32))
    return m.compute_logits(m.forward(torch.tensor(ids, dtype=torch.int32), meta, kv))


def test_teleflm_matches_scaled_llama(tmp_path):
    hf = dict(PRESETS["tiny-teleflm"])
    torch.manual_seed(0)
    lc = transformers.LlamaConfig(vocab_size=hf["vocab_size"], hidden_size=hf["hidden_size"],
                                  intermediate_size=hf["intermediate_size"], num_hidden_layers=hf["num_hidden_layers"],
                                  num_attention_heads=hf["num_attention_heads"],
                                  num_key_value_heads=hf["num_key_value_heads"], rms_norm_eps=hf["rms_norm_eps"],
                                  rope_theta=hf["rope_theta"], max_position_embeddings=hf["max_position_embeddings"],
                                  tie_word_embeddings=False)
    ref = transformers.LlamaForCausalLM(lc).float().eval()
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if p.dim() == 2:
                p.normal_(0.0, 0.05)
    sd = {k: v.detach().clone().contiguous() for k, v in ref.state_dict().items() if "rotary" not in k}
    save_file(sd, tmp_path / "model.safetensors")
    (tmp_path / "config.json").write_text(json.dumps(hf))
    cfg = ModelConfig.from_path(tmp_path)
    assert model_class(cfg).__name__ == "TeleFLMForCausalLM" and not cfg.is_embedding
    m = build_model(cfg, "cpu", torch.float32, model_path=str(tmp_path))
    ids = [5, 17, 300, 2, 999, 41, 7]
    ours = _forward(m, ids)
    with torch.no_grad():
        ref.model.embed_tokens.weight.mul_(hf["input_mult"])
        want = ref(torch.tensor([ids])).logits[0] * (hf["output_mult"] / hf["mup_scale_factor"])
    assert torch.allclose(ours, want, atol=2e-4, rtol=1e-3), (ours - want).abs().max()


def test_teleflm_catalog_size():
    assert 50e9 < ModelConfig.from_hf(PRESETS["tele-flm"]).num_params() < 55e9   # tele-flm-rt.yaml 50B-55B

"""Llama 4 (text) against Hugging Face transformers: a tiny random ``Llama4ForCausalLM`` is saved as
safetensors, loaded by ome_amd, and the prefill logits of every position must match HF's eager
forward (fp32, CPU reference ops).  The prompt is longer than ``attention_chunk_size`` and
``floor_scale`` so chunked attention on the RoPE layers, the NoPE layer's temperature tuning, the
interleaved-pair RoPE re-layout, the L2 q/k norm, sigmoid-scaled expert inputs, the shared expert
and interleaved dense / MoE layers are all exercised; greedy decode must equal HF ``generate``."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd.models.config import preset  # noqa: E402
from ome_amd.models.llama4 import pair_to_halves  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402
from tests.test_gemma_cpu import _our_logits  # noqa: E402


def _hf_model(tmp_path, k: int = 1):
    torch.manual_seed(0)
    cfg = transformers.Llama4TextConfig(
        vocab_size=512, hidden_size=128, intermediate_size=64, intermediate_size_mlp=192, num_hidden_layers=4,
        num_attention_heads=4, num_key_value_heads=2, head_dim=32, num_local_experts=4, num_experts_per_tok=k,
        interleave_moe_layer_step=2, attention_chunk_size=16, max_position_embeddings=512, floor_scale=8,
        attn_scale=0.1, pad_token_id=0, bos_token_id=1, eos_token_id=2,
        rope_parameters={"rope_type": "llama3", "rope_theta": 500000.0, "factor": 8.0, "low_freq_factor": 1.0,
                         "high_freq_factor": 4.0, "original_max_position_embeddings": 64})
    m = transformers.Llama4ForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.2)
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    return m


def test_pair_to_halves_is_neox_layout():
    D = 8
    w = torch.arange(2 * D).float().view(2 * D, 1)
    got = pair_to_halves(w, 2, D).view(-1).tolist()
    assert got == [0, 2, 4, 6, 1, 3, 5, 7, 8, 10, 12, 14, 9, 11, 13, 15]


def test_llama4_preset_shapes():
    c = preset("llama-4-scout-17b-16e")
    assert c.architecture == "Llama4ForConditionalGeneration" and c.num_experts == 16 and c.num_experts_per_tok == 1
    assert c.hidden_size == 5120 and c.num_layers == 48 and c.extra["attention_chunk_size"] == 8192


@pytest.mark.parametrize("k", [1, 2])
def test_llama4_prefill_logits_match_hf(tmp_path, k):
    hf = _hf_model(tmp_path, k)
    ids = [(7 * i + 3) % 500 + 3 for i in range(40)]  # > chunk (16) and > floor_scale (8)
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "Llama4ForCausalLM"
    assert m.moe_layers == {1, 3} and m.use_rope == [True, True, True, False]
    assert m.windows == [-16, -16, -16, -1]
    got = _our_logits(eng, ids)
    err = (got - want).abs().max().item()
    assert err < 2e-3 * max(1.0, want.abs().max().item()), err
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=6, do_sample=False)[0, len(ids):].tolist()
    r = eng.generate([ids], SamplingParams(max_new_tokens=6, ignore_eos=True))[0]
    assert r.output_ids == ref

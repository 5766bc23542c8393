"""MiniCPM3 (``models/minicpm3.py``: MLA with a 256 + 32 latent, LongRoPE, muP scalings folded into
the weights) against transformers: a tiny random ``MiniCPM3ForCausalLM`` (fp32, CPU reference
ops), prefill logits of every position and greedy generation through the engine, with default
and LongRoPE rope parameters."""
import pytest
import torch

transformers = pytest.importorskip("transformers")
if not hasattr(transformers, "MiniCPM3Config"):
    pytest.skip("transformers without MiniCPM3", allow_module_level=True)

from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402
from tests.test_nemotron_h_cpu import _prefill_logits  # noqa: E402


def _hf_model(tmp_path, longrope=False):
    torch.manual_seed(0)
    rp = {"rope_type": "default", "rope_theta": 10000.0}
    if longrope:
        g = torch.Generator().manual_seed(1)
        rp = {"rope_type": "longrope", "rope_theta": 10000.0, "original_max_position_embeddings": 4096, "factor": 1.0,
              "short_factor": (1 + torch.rand(16, generator=g)).tolist(),
              "long_factor": (2 + torch.rand(16, generator=g)).tolist()}
    cfg = transformers.MiniCPM3Config(
        vocab_size=512, hidden_size=160, intermediate_size=256, num_hidden_layers=2, num_attention_heads=5,
        num_key_value_heads=5, kv_lora_rank=256, q_lora_rank=64, qk_nope_head_dim=16, qk_rope_head_dim=32,
        v_head_dim=16, max_position_embeddings=8192, scale_emb=12, scale_depth=1.4, dim_model_base=32,
        tie_word_embeddings=True, rope_parameters=rp, pad_token_id=0, bos_token_id=1, eos_token_id=2)
    m = transformers.MiniCPM3ForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1)
            else:
                p.normal_(0.0, 0.05)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


@pytest.mark.parametrize("longrope", [False, True])
def test_minicpm3_matches_hf(tmp_path, longrope):
    hf = _hf_model(tmp_path, longrope)
    ids = [(7 * i + 3) % 500 + 3 for i in range(40)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "MiniCPM3ForCausalLM" and m.lat == 256 and m.rope == 32
    got = _prefill_logits(eng, ids, [40])
    assert (got - want).abs().max().item() < 2e-3 * max(1.0, want.abs().max().item())
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=8, do_sample=False)[0, len(ids):].tolist()
    assert eng.generate([ids], SamplingParams(max_new_tokens=8, ignore_eos=True))[0].output_ids == ref

"""GPT-OSS against Hugging Face transformers: a tiny random GptOssForCausalLM (sinks, alternating
sliding windows, YaRN with truncate=False, biased router / experts, clamped SwiGLU with
interleaved gate/up) must give the same prefill logits and greedy tokens through ome_amd's CPU
reference path; and the MXFP4 expert dequantisation must equal transformers' own converter."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd.models.gpt_oss import dequant_mxfp4  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402
from tests.test_gemma_cpu import _our_logits  # noqa: E402


def _hf_model(tmp_path):
    torch.manual_seed(0)
    cfg = transformers.GptOssConfig(vocab_size=512, hidden_size=128, intermediate_size=64, num_hidden_layers=4,
                                    num_attention_heads=8, num_key_value_heads=2, head_dim=64, num_local_experts=8,
                                    num_experts_per_tok=2, sliding_window=16, max_position_embeddings=1024,
                                    rope_parameters={"rope_type": "yarn", "factor": 8.0, "beta_fast": 32.0,
                                                     "beta_slow": 1.0, "truncate": False,
                                                     "original_max_position_embeddings": 128,
                                                     "rope_theta": 150000.0},
                                    pad_token_id=0, eos_token_id=2)
    m = transformers.GptOssForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1)
            elif "sinks" in n:
                p.normal_(0.0, 1.0)
            else:
                p.normal_(0.0, 0.06)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    return m


def test_gpt_oss_matches_hf(tmp_path):
    hf = _hf_model(tmp_path)
    ids = [(11 * i + 5) % 500 + 3 for i in range(40)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "GptOssForCausalLM" and m.windows[:2] == [16, -1]
    got = _our_logits(eng, ids)
    err = (got - want).abs().max().item()
    assert err < 2e-3 * max(1.0, want.abs().max().item()), err
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=6, do_sample=False)[0, len(ids):].tolist()
    assert eng.generate([ids], SamplingParams(max_new_tokens=6, ignore_eos=True))[0].output_ids == ref


def test_mxfp4_dequant_matches_transformers():
    from transformers.integrations.mxfp4 import convert_moe_packed_tensors

    g = torch.Generator().manual_seed(0)
    blocks = torch.randint(0, 256, (3, 64, 4, 16), generator=g, dtype=torch.uint8)
    scales = torch.randint(118, 136, (3, 64, 4), generator=g, dtype=torch.uint8)
    ref = convert_moe_packed_tensors(blocks, scales, dtype=torch.float32)   # [E, in, out]
    ours = dequant_mxfp4(blocks, scales).transpose(1, 2)                   # [E, out, in] -> [E, in, out]
    assert torch.equal(ours, ref)

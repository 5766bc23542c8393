"""Bailing MoE (Ling; ``models/bailing.py``): a Bailing-named checkpoint derived from a tiny random
transformers Qwen2-MoE (fused ``query_key_value``, ``attention.dense``, ``word_embeddings``,
``shared_experts``; the Qwen2-MoE shared-expert gate is held at sigmoid(0) = 0.5 and compensated
in the Bailing shared down projection; ``norm_head`` applied to the Qwen2-MoE head) must give the
same logits and greedy tokens.  Bailing's own semantics are parity-unpinned (no transformers
implementation); this pins the name mapping and the shared-expert / norm-head handling."""
import json

import pytest
import torch
from safetensors.torch import save_file

transformers = pytest.importorskip("transformers")

from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402
from tests.test_nemotron_h_cpu import _prefill_logits  # noqa: E402


def _models(tmp_path):
    T = transformers
    torch.manual_seed(0)
    cfg = T.Qwen2MoeConfig(vocab_size=512, hidden_size=256, intermediate_size=256, num_hidden_layers=2,
                           num_attention_heads=4, num_key_value_heads=2, num_experts=8, num_experts_per_tok=2,
                           moe_intermediate_size=64, shared_expert_intermediate_size=128, norm_topk_prob=True,
                           max_position_embeddings=1024, tie_word_embeddings=False, rope_theta=600000.0)
    m = T.Qwen2MoeForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1)
            elif n.endswith("shared_expert_gate.weight"):
                p.zero_()
            else:
                p.normal_(0.0, 0.08)
        raw_head = m.lm_head.weight.detach().clone()
        m.lm_head.weight.copy_(torch.nn.functional.normalize(raw_head, dim=0, eps=1e-7))
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    sd, out = m.state_dict(), {}
    for k, v in sd.items():
        if k == "model.embed_tokens.weight":
            out["model.word_embeddings.weight"] = v
        elif k == "lm_head.weight":
            out[k] = raw_head
        elif ".self_attn.q_proj." in k:
            pre, kind = k.split(".self_attn.q_proj.")
            out[f"{pre}.attention.query_key_value.{kind}"] = torch.cat(
                [v, sd[f"{pre}.self_attn.k_proj.{kind}"], sd[f"{pre}.self_attn.v_proj.{kind}"]])
        elif ".self_attn.k_proj." in k or ".self_attn.v_proj." in k or k.endswith("shared_expert_gate.weight"):
            continue
        elif ".self_attn.o_proj." in k:
            out[k.replace(".self_attn.o_proj.", ".attention.dense.")] = v
        elif ".mlp.shared_expert." in k:
            out[k.replace(".mlp.shared_expert.", ".mlp.shared_experts.")] = v * (0.5 if "down_proj" in k else 1.0)
        else:
            out[k] = v
    save_file({k: v.contiguous() for k, v in out.items()}, str(tmp_path / "model.safetensors"))
    bcfg = {"architectures": ["BailingMoeForCausalLM"], "model_type": "bailing_moe", "vocab_size": 512,
            "hidden_size": 256, "intermediate_size": 256, "num_hidden_layers": 2, "num_attention_heads": 4,
            "num_key_value_heads": 2, "num_experts": 8, "num_shared_experts": 2, "num_experts_per_tok": 2,
            "moe_intermediate_size": 64, "norm_topk_prob": True, "use_qkv_bias": True, "use_bias": False,
            "norm_head": True, "rope_theta": 600000.0, "max_position_embeddings": 1024, "rms_norm_eps": 1e-6,
            "hidden_act": "silu", "first_k_dense_replace": 0, "tie_word_embeddings": False}
    (tmp_path / "config.json").write_text(json.dumps(bcfg))
    m.generation_config.eos_token_id = None
    return m


def test_bailing_matches_equivalent_qwen2_moe(tmp_path):
    hf = _models(tmp_path)
    ids = [(7 * i + 3) % 500 + 3 for i in range(30)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    assert type(eng.runner.model).__name__ == "BailingMoeForCausalLM"
    got = _prefill_logits(eng, ids, [30])
    assert (got - want).abs().max().item() < 2e-3 * max(1.0, want.abs().max().item())
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=8, do_sample=False)[0, len(ids):].tolist()
    assert eng.generate([ids], SamplingParams(max_new_tokens=8, ignore_eos=True))[0].output_ids == ref

"""XVERSE MoE (``models/xverse.py``): an XVERSE-named checkpoint derived from a tiny random
transformers Qwen2-MoE (``mlp.router``, ``mlp.shared_experts``, ``moe_top_k``, no attention biases,
top-k weights not renormalised; the Qwen2-MoE shared-expert gate held at sigmoid(0) = 0.5 and
compensated in the shared down projection) must give the same logits and greedy tokens.  XVERSE's
own semantics are parity-unpinned (no transformers implementation)."""
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
                           num_attention_heads=4, num_key_value_heads=4, num_experts=8, num_experts_per_tok=3,
                           moe_intermediate_size=64, shared_expert_intermediate_size=128, norm_topk_prob=False,
                           max_position_embeddings=1024, tie_word_embeddings=False, rope_theta=500000.0)
    m = T.Qwen2MoeForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1)
            elif n.endswith("shared_expert_gate.weight") or n.endswith(".bias"):
                p.zero_()
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    out = {}
    for k, v in m.state_dict().items():
        if k.endswith(".bias") or k.endswith("shared_expert_gate.weight"):
            continue
        if ".mlp.gate.weight" in k:
            k = k.replace(".mlp.gate.weight", ".mlp.router.weight")
        elif ".mlp.shared_expert." in k:
            v = v * (0.5 if "down_proj" in k else 1.0)
            k = k.replace(".mlp.shared_expert.", ".mlp.shared_experts.")
        out[k] = v
    save_file({k: v.contiguous() for k, v in out.items()}, str(tmp_path / "model.safetensors"))
    xcfg = {"architectures": ["XverseMoeForCausalLM"], "model_type": "xverse", "vocab_size": 512, "hidden_size": 256,
            "intermediate_size": 64, "num_hidden_layers": 2, "num_attention_heads": 4, "num_key_value_heads": 4,
            "num_experts": 8, "moe_top_k": 3, "num_shared_experts": 2, "rope_theta": 500000.0,
            "max_position_embeddings": 1024, "rms_norm_eps": 1e-6, "hidden_act": "silu", "tie_word_embeddings": False}
    (tmp_path / "config.json").write_text(json.dumps(xcfg))
    m.generation_config.eos_token_id = None
    return m


def test_xverse_matches_equivalent_qwen2_moe(tmp_path):
    hf = _models(tmp_path)
    ids = [(7 * i + 3) % 500 + 3 for i in range(30)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "XverseMoeForCausalLM" and m.k == 3 and not m.renorm
    got = _prefill_logits(eng, ids, [30])
    assert (got - want).abs().max().item() < 2e-3 * max(1.0, want.abs().max().item())
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=8, do_sample=False)[0, len(ids):].tolist()
    assert eng.generate([ids], SamplingParams(max_new_tokens=8, ignore_eos=True))[0].output_ids == ref

"""Qwen3-Next (Gated DeltaNet + gated attention + MoE with a gated shared expert) against Hugging
Face transformers: a tiny random ``Qwen3NextForCausalLM`` is saved as safetensors, loaded by
ome_amd, and (fp32, CPU reference ops)

* the prefill logits of every position match HF's forward (HF runs the chunked delta rule, ours
  the recurrent form -- same function);
* the same logits come out when the prompt is fed in two chunks (conv + delta-rule state carried
  in the per-slot state);
* greedy decoding equals HF ``generate``, also with chunked prefill inside the engine;
* the gated-delta reference op agrees with a direct transcription of HF's recurrent update."""
import pytest
import torch

transformers = pytest.importorskip("transformers")
if not hasattr(transformers, "Qwen3NextConfig"):
    pytest.skip("transformers without Qwen3-Next", allow_module_level=True)

from ome_amd import ops  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402
from tests.test_nemotron_h_cpu import _prefill_logits  # noqa: E402


def _hf_model(tmp_path):
    torch.manual_seed(0)
    cfg = transformers.Qwen3NextConfig(
        vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=4, num_attention_heads=4,
        num_key_value_heads=2, head_dim=64, linear_num_key_heads=2, linear_num_value_heads=4, linear_key_head_dim=32,
        linear_value_head_dim=16, linear_conv_kernel_dim=4, num_experts=8, num_experts_per_tok=2,
        moe_intermediate_size=64, shared_expert_intermediate_size=96, max_position_embeddings=512,
        pad_token_id=0, bos_token_id=1, eos_token_id=2)
    m = transformers.Qwen3NextForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("norm.weight") and "linear_attn" not in n:
                p.normal_(0.0, 0.1)            # (1 + w) norms
            elif n.endswith("linear_attn.norm.weight"):
                p.normal_(1.0, 0.1)
            elif n.endswith("A_log"):
                p.uniform_(-1.0, 1.0)
            elif n.endswith("dt_bias"):
                p.normal_(0.0, 0.5)
            elif "conv1d" in n:
                p.normal_(0.0, 0.3)
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


def test_qwen3_next_logits_and_generate_match_hf(tmp_path):
    hf = _hf_model(tmp_path)
    ids = [(7 * i + 3) % 500 + 3 for i in range(40)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "Qwen3NextForCausalLM" and m.kv_layers == [3] and m.lin_layers == [0, 1, 2]
    assert eng.scheduler.prefix_cache is None and m.cfg.rot_dim == 16
    tol = 2e-3 * max(1.0, want.abs().max().item())
    got = _prefill_logits(eng, ids, [40])
    assert (got - want).abs().max().item() < tol
    got2 = _prefill_logits(eng, ids, [13, 27])  # state carried across chunks
    assert (got2 - want).abs().max().item() < tol
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=8, do_sample=False)[0, len(ids):].tolist()
    assert eng.generate([ids], SamplingParams(max_new_tokens=8, ignore_eos=True))[0].output_ids == ref
    eng2 = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                             context_length=256, chunked_prefill_size=16))
    reqs = eng2.generate([ids, ids[:9]], SamplingParams(max_new_tokens=8, ignore_eos=True))
    assert reqs[0].output_ids == ref
    with torch.no_grad():
        ref9 = hf.generate(torch.tensor([ids[:9]]), max_new_tokens=8, do_sample=False)[0, 9:].tolist()
    assert reqs[1].output_ids == ref9


def test_gdn_reference_matches_recurrence():
    torch.manual_seed(1)
    T, Hk, Hv, dk, dv = 6, 2, 4, 8, 4
    q, k, v = torch.randn(T, Hk * dk), torch.randn(T, Hk * dk), torch.randn(T, Hv * dv)
    a, b = torch.randn(T, Hv), torch.randn(T, Hv)
    A_log, dtb = torch.rand(Hv), torch.randn(Hv)
    st = torch.zeros(2, Hv, dv, dk)
    cu, slot, reset = (torch.tensor(x, dtype=torch.int32) for x in ([0, T], [1], [1]))
    y = ops.gdn_scan(q, k, v, a, b, A_log, dtb, st, cu, slot, reset, Hv, Hk)
    S = torch.zeros(Hv, dk, dv)
    for r in range(T):
        qr = torch.nn.functional.normalize(q[r].view(Hk, dk), dim=-1).repeat_interleave(2, 0) * dk ** -0.5
        kr = torch.nn.functional.normalize(k[r].view(Hk, dk), dim=-1).repeat_interleave(2, 0)
        g = -A_log.exp() * torch.nn.functional.softplus(a[r] + dtb)
        S = S * g.exp()[:, None, None]
        kv = torch.einsum("hkv,hk->hv", S, kr)
        S = S + torch.einsum("hk,hv->hkv", kr, (v[r].view(Hv, dv) - kv) * torch.sigmoid(b[r])[:, None])
        want = torch.einsum("hkv,hk->hv", S, qr)
        assert torch.allclose(y[r].view(Hv, dv), want, atol=1e-4)
    assert torch.allclose(st[1], S.transpose(1, 2), atol=1e-5) and st[0].abs().max() == 0

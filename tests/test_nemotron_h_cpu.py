"""NemotronH (hybrid Mamba-2 / attention / ReLU^2-MLP) against Hugging Face transformers: a tiny random
``NemotronHForCausalLM`` is saved as safetensors, loaded by ome_amd, and (fp32, CPU reference ops)

* the prefill logits of every position match HF's forward;
* the same logits come out when the prompt is fed in two chunks (conv / SSM state carried across
  chunks through the per-slot state);
* greedy decoding equals HF ``generate`` (recurrent single-row state updates), also with
  chunked prefill inside the engine;
* the SSM reference ops agree with a direct transcription of HF's recurrent update."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd import ops  # noqa: E402
from ome_amd.models.common import AttnMeta  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402


def _hf_model(tmp_path, pattern="M-M*-M", **kw):
    torch.manual_seed(0)
    cfg = transformers.NemotronHConfig(
        vocab_size=512, hidden_size=128, num_attention_heads=4, num_key_value_heads=2, head_dim=32,
        intermediate_size=256, mamba_num_heads=8, mamba_head_dim=16, ssm_state_size=32, n_groups=2, conv_kernel=4,
        hybrid_override_pattern=pattern, max_position_embeddings=512, chunk_size=16, pad_token_id=0,
        bos_token_id=1, eos_token_id=2, **kw)
    m = transformers.NemotronHForCausalLM(cfg)
    with torch.no_grad():
        for n, b in m.named_buffers():
            if n.endswith("e_score_correction_bias"):
                b.normal_(0.0, 0.05)
        for n, p in m.named_parameters():
            if n.endswith("norm.weight") or n.endswith("norm_f.weight"):
                p.normal_(1.0, 0.1)
            elif n.endswith("A_log"):
                p.uniform_(-1.0, 1.0)
            elif n.endswith("dt_bias"):
                p.normal_(-1.0, 0.5)
            elif n.endswith(".D"):
                p.normal_(1.0, 0.2)
            elif "conv1d" in n:
                p.normal_(0.0, 0.3)
            else:
                p.normal_(0.0, 0.08)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    m.generation_config.eos_token_id = None
    return m


def _prefill_logits(eng, ids, chunks):
    """Prefill ``ids`` through the runner in the given chunk sizes; logits of every position."""
    run = eng.runner
    slot = run.slots.alloc()
    pages = run.pages.alloc(-(-len(ids) // run.P))
    run.slots.set_pages(slot, 0, pages)
    run.slots.flush()
    t = lambda a: torch.tensor(a, dtype=torch.int32)  # noqa: E731
    outs, s = [], 0
    for n in chunks:
        rng = list(range(s, s + n))
        meta = AttnMeta("prefill", t(rng), t([pages[p // run.P] * run.P + p % run.P for p in rng]),
                        run.slots.table.index_select(0, t([slot])), cu_q=t([0, n]), kv_lens=t([s + n]),
                        items=t(ops.prefill_work_items([n], [s + n])).view(-1, 2))
        meta.extra["ssm"] = (t([0, n]), t([slot]), t([int(s == 0)]))
        h = run.model.forward(t(ids[s:s + n]), meta, run.kv)
        outs.append(run.model.compute_logits(h).float())
        s += n
    run.pages.free(pages)
    run.slots.free(slot)
    return torch.cat(outs, 0)


def test_nemotron_h_logits_and_generate_match_hf(tmp_path):
    hf = _hf_model(tmp_path)
    ids = [(7 * i + 3) % 500 + 3 for i in range(40)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "NemotronHForCausalLM" and m.kv_layers == [3] and m.mamba_layers == [0, 2, 5]
    assert eng.scheduler.prefix_cache is None
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


@pytest.mark.parametrize("latent", [None, 64])
def test_nemotron_h_moe_matches_hf(tmp_path, latent):
    """``E`` blocks: sigmoid grouped routing with correction bias, ReLU^2 experts (+ latent
    projection), shared expert."""
    hf = _hf_model(tmp_path, "ME*E", n_routed_experts=8, num_experts_per_tok=2, moe_intermediate_size=64,
                   moe_shared_expert_intermediate_size=96, n_group=2, topk_group=1, routed_scaling_factor=2.5,
                   norm_topk_prob=True, moe_latent_size=latent)
    ids = [(5 * i + 11) % 500 + 3 for i in range(30)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert m.types == ["linear_attention", "moe", "full_attention", "moe"] and m.E == 8
    got = _prefill_logits(eng, ids, [30])
    assert (got - want).abs().max().item() < 2e-3 * max(1.0, want.abs().max().item())
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=6, do_sample=False)[0, len(ids):].tolist()
    assert eng.generate([ids], SamplingParams(max_new_tokens=6, ignore_eos=True))[0].output_ids == ref


def test_ssm_scan_reference_matches_recurrence():
    torch.manual_seed(1)
    T, H, P, N, G = 5, 4, 8, 16, 2
    x, dt = torch.randn(T, H * P), torch.randn(T, H)
    B, C = torch.randn(T, G * N), torch.randn(T, G * N)
    A, D, db = -torch.rand(H) - 0.1, torch.randn(H), torch.randn(H)
    st = torch.zeros(2, H, P, N)
    cu, slot, reset = (torch.tensor(v, dtype=torch.int32) for v in ([0, T], [1], [1]))
    y = ops.ssm_scan(x, dt, B, C, A, D, db, 0.0, st, cu, slot, reset, H, P, N, G)
    h = torch.zeros(H, P, N)
    for r in range(T):
        d = torch.nn.functional.softplus(dt[r] + db)
        b = B[r].view(G, N).repeat_interleave(H // G, 0)
        c = C[r].view(G, N).repeat_interleave(H // G, 0)
        h = h * torch.exp(d * A)[:, None, None] + d[:, None, None] * x[r].view(H, P)[..., None] * b[:, None]
        want = (h * c[:, None]).sum(-1) + D[:, None] * x[r].view(H, P)
        assert torch.allclose(y[r].view(H, P), want, atol=1e-5)
    assert torch.allclose(st[1], h, atol=1e-5) and st[0].abs().max() == 0

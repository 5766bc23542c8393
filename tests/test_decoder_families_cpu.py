"""Spec-driven decoder families (``ome_amd/models/decoder.py``) against Hugging Face transformers.

A tiny random HF model of each family is saved as safetensors, loaded by ome_amd through its
checkpoint-name table and run on the CPU reference ops: prefill logits at every position must
match HF's eager forward, and greedy decoding (prefill + paged decode steps) must agree with
``generate``.  Variants cover every DecoderSpec axis: LayerNorm with / without bias / affine,
the five residual forms, plain and gated MLPs (ReLU, GELU, ReLU^2), learned positions (OPT),
interleaved rotary pairs (GPT-J, GLM, Cohere), a rotary half that is not a multiple of the
kernel's 8-dim lanes plus a zero-padded head dim (StableLM 80 -> 128), per-head and shared
q/k LayerNorms, full-width q/k RMSNorm (OLMo-2), clip_qkv (OLMo), the fused QKV layouts
(concat, per-head, Falcon-40B groups, multi-query), OPT-350m's post-LN with projections and
ALiBi positions (Bloom with 5 heads: the non-power-of-two slope tail; MPT with clip_qkv)."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

from test_gemma_cpu import _our_logits  # noqa: E402

V = 512


def _cfg(kind: str):
    T = transformers
    common = dict(vocab_size=V, bos_token_id=1, eos_token_id=2, pad_token_id=0)
    if kind == "opt":
        return T.OPTForCausalLM, T.OPTConfig(hidden_size=128, num_hidden_layers=3, ffn_dim=256, num_attention_heads=2,
                                             max_position_embeddings=512, word_embed_proj_dim=128, **common)
    if kind == "opt_postln":  # OPT-350m shape: post-LN, project_in / project_out
        return T.OPTForCausalLM, T.OPTConfig(hidden_size=128, num_hidden_layers=3, ffn_dim=256, num_attention_heads=2,
                                             max_position_embeddings=512, word_embed_proj_dim=64,
                                             do_layer_norm_before=False, **common)
    if kind == "gptj":
        return T.GPTJForCausalLM, T.GPTJConfig(n_positions=512, n_embd=128, n_layer=3, n_head=2, rotary_dim=32,
                                               **common)
    if kind.startswith("falcon"):
        kw = dict(hidden_size=256, num_hidden_layers=3, num_attention_heads=4, max_position_embeddings=512, **common)
        if kind == "falcon_40b":
            kw.update(new_decoder_architecture=True, num_kv_heads=2)
        elif kind == "falcon_rw":
            kw.update(multi_query=False, parallel_attn=False, bias=True)
        return T.FalconForCausalLM, T.FalconConfig(**kw)
    if kind.startswith("stablelm"):
        return T.StableLmForCausalLM, T.StableLmConfig(
            hidden_size=160, intermediate_size=256, num_hidden_layers=3, num_attention_heads=2,
            num_key_value_heads=2, partial_rotary_factor=0.25, qk_layernorm=True, use_qkv_bias=True,
            use_parallel_residual=(kind == "stablelm_parallel"), max_position_embeddings=512, **common)
    if kind == "persimmon":
        return T.PersimmonForCausalLM, T.PersimmonConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3,
                                                         num_attention_heads=2, partial_rotary_factor=0.5,
                                                         qk_layernorm=True, max_position_embeddings=512, **common)
    if kind == "cohere":
        return T.CohereForCausalLM, T.CohereConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3,
                                                   num_attention_heads=2, num_key_value_heads=1, use_qk_norm=True,
                                                   logit_scale=0.5, max_position_embeddings=512, **common)
    if kind in ("glm", "glm4"):
        C, M = (T.GlmConfig, T.GlmForCausalLM) if kind == "glm" else (T.Glm4Config, T.Glm4ForCausalLM)
        return M, C(hidden_size=128, intermediate_size=256, num_hidden_layers=3, num_attention_heads=2,
                    num_key_value_heads=1, head_dim=64, partial_rotary_factor=0.5, attention_bias=True,
                    max_position_embeddings=512, **common)
    if kind == "olmo2":
        return T.Olmo2ForCausalLM, T.Olmo2Config(hidden_size=128, intermediate_size=256, num_hidden_layers=3,
                                                 num_attention_heads=2, num_key_value_heads=2,
                                                 max_position_embeddings=512, **common)
    if kind == "olmo":
        return T.OlmoForCausalLM, T.OlmoConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3,
                                               num_attention_heads=2, num_key_value_heads=2, clip_qkv=0.3,
                                               max_position_embeddings=512, **common)
    if kind == "bloom":  # 5 heads: exercises the non-power-of-two ALiBi slope tail
        return T.BloomForCausalLM, T.BloomConfig(hidden_size=320, n_layer=3, n_head=5, **common)
    if kind == "mpt":
        return T.MptForCausalLM, T.MptConfig(d_model=192, n_heads=3, n_layers=3, max_seq_len=512,
                                             attn_config={"alibi": True, "alibi_bias_max": 8, "clip_qkv": 0.5},
                                             **common)
    if kind.startswith("phi3"):  # head_dim 96: zero-padded to 128
        kw = dict(hidden_size=192, intermediate_size=256, num_hidden_layers=3, num_attention_heads=2,
                  num_key_value_heads=2, max_position_embeddings=512, sliding_window=24, **common)
        if kind == "phi3_longrope":
            kw.update(max_position_embeddings=1024, original_max_position_embeddings=32, rope_scaling={
                "type": "longrope", "short_factor": [1.0 + 0.05 * i for i in range(48)],
                "long_factor": [1.5 + 0.1 * i for i in range(48)]})
        return T.Phi3ForCausalLM, T.Phi3Config(**kw)
    if kind == "granite":
        return T.GraniteForCausalLM, T.GraniteConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3,
                                                     num_attention_heads=2, num_key_value_heads=1,
                                                     embedding_multiplier=6.0, residual_multiplier=0.3,
                                                     attention_multiplier=0.05, logits_scaling=4.0,
                                                     max_position_embeddings=512, **common)
    if kind == "smollm3":
        return T.SmolLM3ForCausalLM, T.SmolLM3Config(hidden_size=128, intermediate_size=256, num_hidden_layers=4,
                                                     num_attention_heads=2, num_key_value_heads=1,
                                                     no_rope_layers=[1, 0, 1, 0], max_position_embeddings=512,
                                                     **common)
    if kind == "olmoe":
        return T.OlmoeForCausalLM, T.OlmoeConfig(hidden_size=128, intermediate_size=64, num_hidden_layers=2,
                                                 num_attention_heads=2, num_key_value_heads=2, num_experts=8,
                                                 num_experts_per_tok=3, norm_topk_prob=False,
                                                 max_position_embeddings=512, **common)
    if kind == "granitemoe":
        return T.GraniteMoeForCausalLM, T.GraniteMoeConfig(hidden_size=128, intermediate_size=64, num_hidden_layers=2,
                                                           num_attention_heads=2, num_key_value_heads=1,
                                                           num_local_experts=6, num_experts_per_tok=2,
                                                           embedding_multiplier=4.0, residual_multiplier=0.4,
                                                           attention_multiplier=0.06, logits_scaling=3.0,
                                                           max_position_embeddings=512, **common)
    if kind == "dbrx":
        return T.DbrxForCausalLM, T.DbrxConfig(d_model=128, n_heads=2, n_layers=2, max_seq_len=512,
                                               attn_config={"kv_n_heads": 1, "clip_qkv": 1.5, "rope_theta": 10000.0},
                                               ffn_config={"ffn_hidden_size": 64, "moe_num_experts": 4, "moe_top_k": 2},
                                               **common)
    if kind == "ernie_moe":
        return T.Ernie4_5_MoeForCausalLM, T.Ernie4_5_MoeConfig(
            hidden_size=128, intermediate_size=192, num_hidden_layers=3, num_attention_heads=2, num_key_value_heads=1,
            moe_intermediate_size=64, moe_num_experts=8, moe_k=2, moe_num_shared_experts=1, moe_layer_start_index=1,
            moe_layer_end_index=2, max_position_embeddings=512, **common)
    if kind == "minimax_m2":
        return T.MiniMaxM2ForCausalLM, T.MiniMaxM2Config(hidden_size=128, intermediate_size=64, num_hidden_layers=2,
                                                         num_attention_heads=2, num_key_value_heads=1, head_dim=64,
                                                         num_local_experts=8, num_experts_per_tok=2,
                                                         max_position_embeddings=512, **common)
    if kind == "arcee":
        return T.ArceeForCausalLM, T.ArceeConfig(hidden_size=128, intermediate_size=256, num_hidden_layers=3,
                                                 num_attention_heads=2, num_key_value_heads=1, hidden_act="relu2",
                                                 max_position_embeddings=512, **common)
    raise KeyError(kind)


def _hf_model(kind: str, tmp_path):
    torch.manual_seed(0)
    cls, cfg = _cfg(kind)
    m = cls(cfg)
    with torch.no_grad():
        for n, b in m.named_buffers():
            if n.endswith("e_score_correction_bias"):  # exercise the selection-only router bias
                b.copy_(torch.randn_like(b.float()) * 0.05)
        for n, p in m.named_parameters():
            if n.endswith("e_score_correction_bias"):
                p.copy_(torch.randn_like(p) * 0.05)
            elif kind == "dbrx" and "router" in n:  # well-separated routing: bf16 must not flip experts
                p.normal_(0.0, 1.0)
            elif ("norm" in n or "ln" in n.split(".")[-2]) and n.endswith("weight"):
                p.normal_(1.0, 0.2)
            elif p.dim() == 2:
                p.normal_(0.0, 0.08)
            else:
                p.normal_(0.0, 0.05)
    m = m.float().eval()
    m.config._attn_implementation = "eager"
    m.save_pretrained(tmp_path, safe_serialization=True)
    return m


KINDS = ["opt", "opt_postln", "gptj", "falcon_7b", "falcon_40b", "falcon_rw", "stablelm", "stablelm_parallel",
         "persimmon", "cohere", "glm", "glm4", "olmo2", "olmo", "arcee", "bloom", "mpt", "phi3", "phi3_longrope",
         "granite", "smollm3", "olmoe", "granitemoe", "dbrx", "ernie_moe", "minimax_m2"]


@pytest.mark.parametrize("kind", KINDS)
def test_decoder_family_matches_hf(tmp_path, kind):
    hf = _hf_model(kind, tmp_path)
    ids = [(7 * i + 3) % 500 + 3 for i in range(40)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ in ("DecoderForCausalLM", "DecoderMoEForCausalLM")
    if kind.startswith("stablelm"):
        assert m.D == 128 and m.Dt == 80 and m.rot_true == 20 and m.rot_k == 32 and m.perm is not None
    got = _our_logits(eng, ids)
    err = (got - want).abs().max().item()
    assert err < 2e-3 * max(1.0, want.abs().max().item()), err
    with torch.no_grad():
        want_ids = hf.generate(torch.tensor([ids]), max_new_tokens=6, do_sample=False)[0, len(ids):].tolist()
    r = eng.generate([ids], SamplingParams(max_new_tokens=6, ignore_eos=True))[0]
    assert r.output_ids == want_ids


def test_rope_layout_is_a_permutation():
    from ome_amd.models.decoder import rope_layout

    for dt, dp, rot, style in [(80, 128, 20, "neox"), (64, 64, 32, "interleaved"), (128, 128, 64, "interleaved"),
                               (256, 256, 64, "interleaved"), (80, 128, 40, "interleaved")]:
        perm, rk = rope_layout(dt, dp, rot, style)
        assert sorted(perm.tolist()) == list(range(dp)) and rk % 16 == 0 and rk <= dp
    assert rope_layout(128, 128, 128, "neox") == (None, 128)

"""Spec-driven dense decoder: the long tail of the reference runtime catalog's architectures on
the same HIP kernels as the Llama path.

The reference serves ~80 HF architectures through SGLang/vLLM images
(``config/runtimes/srt/**``, ``modelArchitecture:`` of each ClusterServingRuntime).  Most dense
decoders differ from Llama only in a handful of orthogonal choices, so instead of one class per
family this module describes each family by a :class:`DecoderSpec` and runs all of them through
one forward built from the existing kernels (RMSNorm / LayerNorm with fused residual, fused
RoPE + paged-KV write, MFMA paged attention, SwiGLU / plain activations, hipBLASLt GEMMs):

* norm: RMSNorm, LayerNorm with bias, LayerNorm without bias (Cohere), LayerNorm without affine
  (OLMo-1);
* residual: sequential pre-norm, parallel with one shared norm (GPT-J, Cohere, Falcon-7B,
  StableLM-2 parallel), parallel with two norms (Falcon-40B ``ln_attn`` / ``ln_mlp``),
  sandwich (GLM-4 post-block norms), post-block norms only (OLMo-2), post-LN (OPT-350m);
* MLP: gated (SwiGLU / GeGLU) or plain ``fc -> act -> down`` with optional biases (ReLU, GELU,
  ReLU^2);
* positions: RoPE (NeoX halves or GPT-J / GLM / Cohere interleaved pairs, any partial width),
  or OPT's learned absolute embeddings;
* attention extras: per-head LayerNorm q/k norms (Persimmon, StableLM, Cohere), full-width
  RMSNorm q/k norms (OLMo-2), ``clip_qkv`` (OLMo-1);
* fused checkpoint layouts: ``[Q;K;V]`` concat, NeoX ``[heads, 3, D]``, Falcon-40B
  ``[kv_groups, q_per_group + 2, D]``, ``gate_up_proj``;
* head dims outside the kernel tiles {64, 128, 256} (StableLM-3B / Persimmon-like 80) are
  zero-padded per head at load time, and any RoPE geometry the kernel cannot rotate directly
  (interleaved pairs, a rotary half that is not a multiple of 8 lanes) is mapped onto it by a
  *rope layout*: a per-head permutation of the Q/K weight rows plus a widened cos/sin table whose
  extra frequencies are the identity (cos 1, sin 0).  Q.K is invariant under a permutation
  applied to both, so the kernel's NeoX rotate_half produces exactly the family's rotation.

Families (HF ``architectures[0]``): OPTForCausalLM, GPTJForCausalLM, FalconForCausalLM,
StableLmForCausalLM, PersimmonForCausalLM, CohereForCausalLM, GlmForCausalLM, Glm4ForCausalLM,
Olmo2ForCausalLM, OlmoForCausalLM, ArceeForCausalLM, BloomForCausalLM, MptForCausalLM (ALiBi
positions: per-head slopes added inside the MFMA attention kernels).  Each is checked against transformers on
CPU (``tests/test_decoder_families_cpu.py``) and on gfx950 (``tests/test_decoder_families_gpu.py``).
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig, rope_cos_sin
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

# kernel activation codes (csrc/kernels/elementwise.hip): plain ``ops.act`` and gated ``ops.act_and_mul``
ACT_PLAIN = {"silu": 0, "swish": 0, "gelu_pytorch_tanh": 1, "gelu_new": 1, "gelu_fast": 1, "gelu": 3,
             "relu2": 4, "relu": 5}
ACT_GATED = {"silu": 0, "swish": 0, "gelu_pytorch_tanh": 1, "gelu_new": 1, "gelu_fast": 1,
             "gegelu": 3}   # gegelu: Phi-3-small (ops.act_and_mul act 3, gate / up de-interleaved at load)

_LLAMA_NAMES = [
    (r"(?:model\.)?embed_tokens\.weight", "embed"),
    (r"(?:model\.)?norm\.(weight|bias)", r"norm.\1"),
    (r"lm_head\.(weight|bias)", r"lm_head.\1"),
    (r"(?:model\.)?layers\.(\d+)\.self_attn\.(q|k|v|o)_proj\.(weight|bias)", r"L.\1.\2.\3"),
    (r"(?:model\.)?layers\.(\d+)\.mlp\.gate_up_proj\.weight", r"L.\1.gate_up.weight"),
    (r"(?:model\.)?layers\.(\d+)\.mlp\.(gate|up|down)_proj\.(weight|bias)", r"L.\1.\2.\3"),
    (r"(?:model\.)?layers\.(\d+)\.input_layernorm\.(weight|bias)", r"L.\1.ln1.\2"),
    (r"(?:model\.)?layers\.(\d+)\.post_attention_layernorm\.(weight|bias)", r"L.\1.ln2.\2"),
    (r"(?:model\.)?layers\.(\d+)\.self_attn\.(q|k)_norm\.(weight|bias)", r"L.\1.\2_norm.\3"),
]


@dataclass
class DecoderSpec:
    norm: str = "rms"            # rms | ln (LayerNorm, bias) | ln_nobias | ln_noaffine
    residual: str = "seq"        # seq | parallel_shared | parallel | sandwich | post | post_ln
    mlp: str = "gated"           # gated ([gate; up]) | plain (fc -> act -> down)
    rope: str = "neox"           # neox | interleaved | none
    qkv_layout: str = "split"    # split | concat | heads3 | groups
    qk_norm: str = ""            # "" | rms_head (kernel) | ln_head (per-head LayerNorm) | rms_full
    qk_norm_per_head_w: bool = False  # q/k norm weights are [heads, D] (StableLM, Cohere)
    pos_offset: int = -1         # learned absolute position embeddings (OPT: 2); -1 = none
    lm_head_bias: bool = False
    alibi: str = ""              # "" | bloom (Bloom / Falcon slopes) | mpt (MPT slopes, alibi_bias_max)
    embed_norm: bool = False     # LayerNorm right after the token embedding (Bloom)
    embed_scale: float = 1.0     # Granite embedding_multiplier, MiniCPM scale_emb
    residual_scale: float = 1.0  # block outputs scaled before the residual add (Granite, MiniCPM)
    attn_scale: float | None = None  # softmax scale override (Granite attention_multiplier)
    logit_mult: float | None = None  # logits multiplier (Cohere logit_scale, 1/logits_scaling, MiniCPM)
    head: str = ""               # "" | score (Linear, LlamaForSequenceClassification) | reward_mlp (Qwen2 RM) | v_head
    lm_head_norm: bool = False   # Baichuan-2 NormHead: lm_head rows L2-normalised
    names: list = field(default_factory=lambda: list(_LLAMA_NAMES))
    prefixes: tuple = ()


def _spec_for(cfg: ModelConfig) -> DecoderSpec:
    arch, hf = cfg.architecture, cfg.extra or {}
    if arch == "OPTForCausalLM":
        return DecoderSpec(norm="ln", residual="seq" if hf.get("do_layer_norm_before", True) else "post_ln",
                           mlp="plain", rope="none", pos_offset=2, prefixes=("model.decoder.", "decoder."), names=[
                               (r"embed_tokens\.weight", "embed"), (r"embed_positions\.weight", "pos_embed"),
                               (r"final_layer_norm\.(weight|bias)", r"norm.\1"),
                               (r"project_in\.weight", "proj_in.weight"), (r"project_out\.weight", "proj_out.weight"),
                               (r"lm_head\.weight", "lm_head.weight"),
                               (r"layers\.(\d+)\.self_attn\.(q|k|v)_proj\.(weight|bias)", r"L.\1.\2.\3"),
                               (r"layers\.(\d+)\.self_attn\.out_proj\.(weight|bias)", r"L.\1.o.\2"),
                               (r"layers\.(\d+)\.self_attn_layer_norm\.(weight|bias)", r"L.\1.ln1.\2"),
                               (r"layers\.(\d+)\.final_layer_norm\.(weight|bias)", r"L.\1.ln2.\2"),
                               (r"layers\.(\d+)\.fc1\.(weight|bias)", r"L.\1.fc.\2"),
                               (r"layers\.(\d+)\.fc2\.(weight|bias)", r"L.\1.down.\2")])
    if arch == "GPTJForCausalLM":
        return DecoderSpec(norm="ln", residual="parallel_shared", mlp="plain", rope="interleaved",
                           lm_head_bias=True, prefixes=("transformer.",), names=[
                               (r"wte\.weight", "embed"), (r"ln_f\.(weight|bias)", r"norm.\1"),
                               (r"lm_head\.(weight|bias)", r"lm_head.\1"),
                               (r"h\.(\d+)\.ln_1\.(weight|bias)", r"L.\1.ln1.\2"),
                               (r"h\.(\d+)\.attn\.(q|k|v)_proj\.weight", r"L.\1.\2.weight"),
                               (r"h\.(\d+)\.attn\.out_proj\.weight", r"L.\1.o.weight"),
                               (r"h\.(\d+)\.mlp\.fc_in\.(weight|bias)", r"L.\1.fc.\2"),
                               (r"h\.(\d+)\.mlp\.fc_out\.(weight|bias)", r"L.\1.down.\2")])
    if arch in ("FalconForCausalLM", "RWForCausalLM"):
        new = bool(hf.get("new_decoder_architecture"))
        parallel = bool(hf.get("parallel_attn", True))
        nln = hf.get("num_ln_in_parallel_attn") or (2 if new else 1)
        residual = ("parallel" if nln == 2 else "parallel_shared") if (new or parallel) else "seq"
        layout = "groups" if new else ("concat" if hf.get("multi_query", True) else "heads3")
        if hf.get("alibi"):
            raise NotImplementedError("Falcon with ALiBi positions")
        return DecoderSpec(norm="ln", residual=residual, mlp="plain", qkv_layout=layout, prefixes=("transformer.",), names=[
                               (r"word_embeddings\.weight", "embed"), (r"ln_f\.(weight|bias)", r"norm.\1"),
                               (r"lm_head\.weight", "lm_head.weight"),
                               (r"h\.(\d+)\.self_attention\.query_key_value\.(weight|bias)", r"L.\1.qkv.\2"),
                               (r"h\.(\d+)\.self_attention\.dense\.(weight|bias)", r"L.\1.o.\2"),
                               (r"h\.(\d+)\.mlp\.dense_h_to_4h\.(weight|bias)", r"L.\1.fc.\2"),
                               (r"h\.(\d+)\.mlp\.dense_4h_to_h\.(weight|bias)", r"L.\1.down.\2"),
                               (r"h\.(\d+)\.(?:input_layernorm|ln_attn)\.(weight|bias)", r"L.\1.ln1.\2"),
                               (r"h\.(\d+)\.(?:post_attention_layernorm|ln_mlp)\.(weight|bias)", r"L.\1.ln2.\2")])
    if arch == "StableLmForCausalLM":
        names = list(_LLAMA_NAMES) + [
            (r"(?:model\.)?layers\.(\d+)\.self_attn\.(q|k)_layernorm\.norms\.(\d+)\.weight", r"L.\1.\2_norm.h\3")]
        return DecoderSpec(norm="ln", residual="parallel_shared" if hf.get("use_parallel_residual") else "seq",
                           qk_norm="ln_head" if hf.get("qk_layernorm") else "", qk_norm_per_head_w=True,
                           names=names)
    if arch == "PersimmonForCausalLM":
        return DecoderSpec(norm="ln", mlp="plain", qkv_layout="heads3",
                           qk_norm="ln_head" if hf.get("qk_layernorm", True) else "", prefixes=("model.",), names=[
                               (r"embed_tokens\.weight", "embed"), (r"final_layernorm\.(weight|bias)", r"norm.\1"),
                               (r"lm_head\.weight", "lm_head.weight"),
                               (r"layers\.(\d+)\.self_attn\.query_key_value\.(weight|bias)", r"L.\1.qkv.\2"),
                               (r"layers\.(\d+)\.self_attn\.dense\.(weight|bias)", r"L.\1.o.\2"),
                               (r"layers\.(\d+)\.self_attn\.(q|k)_layernorm\.(weight|bias)", r"L.\1.\2_norm.\3"),
                               (r"layers\.(\d+)\.mlp\.dense_h_to_4h\.(weight|bias)", r"L.\1.fc.\2"),
                               (r"layers\.(\d+)\.mlp\.dense_4h_to_h\.(weight|bias)", r"L.\1.down.\2"),
                               (r"layers\.(\d+)\.input_layernorm\.(weight|bias)", r"L.\1.ln1.\2"),
                               (r"layers\.(\d+)\.post_attention_layernorm\.(weight|bias)", r"L.\1.ln2.\2")])
    if arch == "CohereForCausalLM":
        return DecoderSpec(norm="ln_nobias", residual="parallel_shared", rope="interleaved",
                           qk_norm="ln_head" if hf.get("use_qk_norm") else "", qk_norm_per_head_w=True)
    if arch in ("GlmForCausalLM", "Glm4ForCausalLM"):
        names = list(_LLAMA_NAMES) + [
            (r"(?:model\.)?layers\.(\d+)\.post_self_attn_layernorm\.weight", r"L.\1.post_attn.weight"),
            (r"(?:model\.)?layers\.(\d+)\.post_mlp_layernorm\.weight", r"L.\1.post_mlp.weight")]
        return DecoderSpec(rope="interleaved", residual="sandwich" if arch == "Glm4ForCausalLM" else "seq",
                           names=names)
    if arch == "Olmo2ForCausalLM":
        names = [n for n in _LLAMA_NAMES if "layernorm" not in n[0]] + [
            (r"(?:model\.)?layers\.(\d+)\.post_attention_layernorm\.weight", r"L.\1.post_attn.weight"),
            (r"(?:model\.)?layers\.(\d+)\.post_feedforward_layernorm\.weight", r"L.\1.post_mlp.weight")]
        return DecoderSpec(residual="post", qk_norm="rms_full", names=names)
    if arch == "BloomForCausalLM":
        return DecoderSpec(norm="ln", mlp="plain", rope="none", qkv_layout="heads3", alibi="bloom", embed_norm=True,
                           prefixes=("transformer.",), names=[
                               (r"word_embeddings\.weight", "embed"),
                               (r"word_embeddings_layernorm\.(weight|bias)", r"emb_ln.\1"),
                               (r"ln_f\.(weight|bias)", r"norm.\1"), (r"lm_head\.weight", "lm_head.weight"),
                               (r"h\.(\d+)\.input_layernorm\.(weight|bias)", r"L.\1.ln1.\2"),
                               (r"h\.(\d+)\.self_attention\.query_key_value\.(weight|bias)", r"L.\1.qkv.\2"),
                               (r"h\.(\d+)\.self_attention\.dense\.(weight|bias)", r"L.\1.o.\2"),
                               (r"h\.(\d+)\.post_attention_layernorm\.(weight|bias)", r"L.\1.ln2.\2"),
                               (r"h\.(\d+)\.mlp\.dense_h_to_4h\.(weight|bias)", r"L.\1.fc.\2"),
                               (r"h\.(\d+)\.mlp\.dense_4h_to_h\.(weight|bias)", r"L.\1.down.\2")])
    if arch in ("MptForCausalLM", "MPTForCausalLM"):  # HF port and the mosaicml remote class: same names
        return DecoderSpec(norm="ln_nobias", mlp="plain", rope="none", qkv_layout="concat",
                           alibi="mpt" if (hf.get("attn_config") or {}).get("alibi", True) else "",
                           prefixes=("transformer.",), names=[
                               (r"wte\.weight", "embed"), (r"norm_f\.weight", "norm.weight"),
                               (r"lm_head\.weight", "lm_head.weight"),
                               (r"blocks\.(\d+)\.norm_1\.weight", r"L.\1.ln1.weight"),
                               (r"blocks\.(\d+)\.norm_2\.weight", r"L.\1.ln2.weight"),
                               (r"blocks\.(\d+)\.attn\.Wqkv\.weight", r"L.\1.qkv.weight"),
                               (r"blocks\.(\d+)\.attn\.out_proj\.weight", r"L.\1.o.weight"),
                               (r"blocks\.(\d+)\.ffn\.up_proj\.weight", r"L.\1.fc.weight"),
                               (r"blocks\.(\d+)\.ffn\.down_proj\.weight", r"L.\1.down.weight")])
    if arch in ("Phi3ForCausalLM", "Phi3VForCausalLM"):   # Phi3V: the decoder of models/phi3v.py
        names = list(_LLAMA_NAMES) + [(r"(?:model\.)?layers\.(\d+)\.self_attn\.qkv_proj\.weight", r"L.\1.qkv.weight")]
        return DecoderSpec(qkv_layout="concat", names=names)
    if arch == "GraniteForCausalLM":
        return DecoderSpec(embed_scale=float(hf.get("embedding_multiplier", 1.0)),
                           residual_scale=float(hf.get("residual_multiplier", 1.0)),
                           attn_scale=hf.get("attention_multiplier"),
                           logit_mult=1.0 / float(hf.get("logits_scaling", 1.0)))
    if arch == "SmolLM3ForCausalLM":
        return DecoderSpec()  # NoPE layers from ``no_rope_layers`` (DecoderForCausalLM.__init__)
    if arch in ("InternLM2ForCausalLM", "InternLM2ForRewardModel"):
        return DecoderSpec(qkv_layout="groups", head="v_head" if arch.endswith("RewardModel") else "",
                           prefixes=("model.",), names=[
                               (r"tok_embeddings\.weight", "embed"), (r"norm\.weight", "norm.weight"),
                               (r"output\.weight", "lm_head.weight"), (r"v_head\.weight", "head.0.weight"),
                               (r"layers\.(\d+)\.attention\.wqkv\.(weight|bias)", r"L.\1.qkv.\2"),
                               (r"layers\.(\d+)\.attention\.wo\.(weight|bias)", r"L.\1.o.\2"),
                               (r"layers\.(\d+)\.feed_forward\.w1\.weight", r"L.\1.gate.weight"),
                               (r"layers\.(\d+)\.feed_forward\.w3\.weight", r"L.\1.up.weight"),
                               (r"layers\.(\d+)\.feed_forward\.w2\.weight", r"L.\1.down.weight"),
                               (r"layers\.(\d+)\.attention_norm\.weight", r"L.\1.ln1.weight"),
                               (r"layers\.(\d+)\.ffn_norm\.weight", r"L.\1.ln2.weight")])
    if arch in ("Qwen2ForRewardModel", "LlamaForSequenceClassification", "Qwen2ForSequenceClassification",
                "MistralForSequenceClassification"):
        names = list(_LLAMA_NAMES) + [(r"score\.(\d+)\.(weight|bias)", r"head.\1.\2"),
                                      (r"score\.(weight|bias)", r"head.0.\1")]
        return DecoderSpec(head="reward_mlp" if arch == "Qwen2ForRewardModel" else "score", names=names)
    if arch == "Phi3SmallForCausalLM":   # models/phi3small.py: grouped biased QKV, LayerNorm, muP scalings
        hd = cfg.attn_head_dim or cfg.head_dim   # the checkpoint's head dim (before kernel padding)
        mup = bool(hf.get("mup_use_scaling", True))
        return DecoderSpec(norm="ln", qkv_layout="groups",
                           embed_scale=float(hf.get("mup_embedding_multiplier") or 1.0),
                           attn_scale=float(hf.get("mup_attn_multiplier", 1.0)) / hd if mup else None,
                           logit_mult=1.0 / float(hf.get("mup_width_multiplier") or 1.0),
                           prefixes=("model.",), names=[
                               (r"embed_tokens\.weight", "embed"), (r"final_layernorm\.(weight|bias)", r"norm.\1"),
                               (r"lm_head\.weight", "lm_head.weight"),
                               (r"layers\.(\d+)\.self_attn\.query_key_value\.(weight|bias)", r"L.\1.qkv.\2"),
                               (r"layers\.(\d+)\.self_attn\.dense\.(weight|bias)", r"L.\1.o.\2"),
                               (r"layers\.(\d+)\.mlp\.gate_up_il\.(weight|bias)", r"L.\1.gate_up.\2"),
                               (r"layers\.(\d+)\.mlp\.down_proj\.(weight|bias)", r"L.\1.down.\2"),
                               (r"layers\.(\d+)\.input_layernorm\.(weight|bias)", r"L.\1.ln1.\2"),
                               (r"layers\.(\d+)\.post_attention_layernorm\.(weight|bias)", r"L.\1.ln2.\2")])
    if arch == "MiMoForCausalLM":  # Qwen2 layout; the multi-token-prediction layers (mtp_layers.*) are unused
        return DecoderSpec()
    if arch == "QWenLMHeadModel":  # Qwen (v1): fused biased c_attn, SwiGLU as c_proj(w1(x) * silu(w2(x)))
        return DecoderSpec(qkv_layout="concat", prefixes=("transformer.",), names=[
            (r"wte\.weight", "embed"), (r"ln_f\.weight", "norm.weight"), (r"lm_head\.weight", "lm_head.weight"),
            (r"h\.(\d+)\.ln_1\.weight", r"L.\1.ln1.weight"), (r"h\.(\d+)\.ln_2\.weight", r"L.\1.ln2.weight"),
            (r"h\.(\d+)\.attn\.c_attn\.(weight|bias)", r"L.\1.qkv.\2"),
            (r"h\.(\d+)\.attn\.c_proj\.weight", r"L.\1.o.weight"),
            (r"h\.(\d+)\.mlp\.w1\.weight", r"L.\1.up.weight"), (r"h\.(\d+)\.mlp\.w2\.weight", r"L.\1.gate.weight"),
            (r"h\.(\d+)\.mlp\.c_proj\.weight", r"L.\1.down.weight")])
    if arch == "BaichuanForCausalLM":  # fused W_pack; 13B: ALiBi; Baichuan-2: NormHead
        names = list(_LLAMA_NAMES) + [(r"(?:model\.)?layers\.(\d+)\.self_attn\.W_pack\.weight", r"L.\1.qkv.weight")]
        big = cfg.hidden_size == 5120 and cfg.num_layers == 40
        return DecoderSpec(qkv_layout="concat", names=names, rope="none" if big else "neox", alibi="bloom" if big else "",
                           lm_head_norm=cfg.vocab_size == 125696)
    if arch == "ExaoneForCausalLM":
        return DecoderSpec(prefixes=("transformer.",), names=[
            (r"wte\.weight", "embed"), (r"ln_f\.weight", "norm.weight"), (r"lm_head\.weight", "lm_head.weight"),
            (r"h\.(\d+)\.ln_1\.weight", r"L.\1.ln1.weight"), (r"h\.(\d+)\.ln_2\.weight", r"L.\1.ln2.weight"),
            (r"h\.(\d+)\.attn\.attention\.(q|k|v)_proj\.weight", r"L.\1.\2.weight"),
            (r"h\.(\d+)\.attn\.attention\.out_proj\.weight", r"L.\1.o.weight"),
            (r"h\.(\d+)\.mlp\.c_fc_0\.weight", r"L.\1.gate.weight"), (r"h\.(\d+)\.mlp\.c_fc_1\.weight", r"L.\1.up.weight"),
            (r"h\.(\d+)\.mlp\.c_proj\.weight", r"L.\1.down.weight")])
    if arch == "OrionForCausalLM":  # Llama with LayerNorm (weight + bias)
        return DecoderSpec(norm="ln")
    if arch == "MiniCPMForCausalLM":
        return DecoderSpec(embed_scale=float(hf.get("scale_emb", 1.0)),
                           residual_scale=float(hf.get("scale_depth", 1.0)) / math.sqrt(cfg.num_layers),
                           logit_mult=float(hf.get("dim_model_base", cfg.hidden_size)) / cfg.hidden_size)
    if arch in ("ChatGLMModel", "ChatGLMForConditionalGeneration"):  # ChatGLM2/3, GLM-4 (THUDM remote code)
        return DecoderSpec(rope="interleaved", qkv_layout="concat", prefixes=("transformer.",), names=[
            (r"embedding\.word_embeddings\.weight", "embed"), (r"encoder\.final_layernorm\.weight", "norm.weight"),
            (r"output_layer\.weight", "lm_head.weight"),
            (r"encoder\.layers\.(\d+)\.input_layernorm\.weight", r"L.\1.ln1.weight"),
            (r"encoder\.layers\.(\d+)\.post_attention_layernorm\.weight", r"L.\1.ln2.weight"),
            (r"encoder\.layers\.(\d+)\.self_attention\.query_key_value\.(weight|bias)", r"L.\1.qkv.\2"),
            (r"encoder\.layers\.(\d+)\.self_attention\.dense\.weight", r"L.\1.o.weight"),
            (r"encoder\.layers\.(\d+)\.mlp\.dense_h_to_4h\.weight", r"L.\1.gate_up.weight"),
            (r"encoder\.layers\.(\d+)\.mlp\.dense_4h_to_h\.weight", r"L.\1.down.weight")])
    if arch in ("OlmoeForCausalLM", "MiniMaxM2ForCausalLM"):  # full-width q/k RMSNorm + experts (decoder_moe.py)
        return DecoderSpec(qk_norm="rms_full")
    if arch == "GraniteMoeForCausalLM":
        return DecoderSpec(embed_scale=float(hf.get("embedding_multiplier", 1.0)),
                           residual_scale=float(hf.get("residual_multiplier", 1.0)),
                           attn_scale=hf.get("attention_multiplier"),
                           logit_mult=1.0 / float(hf.get("logits_scaling", 1.0)))
    if arch == "Ernie4_5_MoeForCausalLM":
        return DecoderSpec(rope="interleaved")
    if arch == "DbrxForCausalLM":
        return DecoderSpec(norm="ln_nobias", qkv_layout="concat", prefixes=("transformer.",), names=[
            (r"wte\.weight", "embed"), (r"norm_f\.weight", "norm.weight"), (r"lm_head\.weight", "lm_head.weight"),
            (r"blocks\.(\d+)\.norm_attn_norm\.norm_1\.weight", r"L.\1.ln1.weight"),
            (r"blocks\.(\d+)\.norm_attn_norm\.norm_2\.weight", r"L.\1.ln2.weight"),
            (r"blocks\.(\d+)\.norm_attn_norm\.attn\.Wqkv\.weight", r"L.\1.qkv.weight"),
            (r"blocks\.(\d+)\.norm_attn_norm\.attn\.out_proj\.weight", r"L.\1.o.weight")])
    if arch == "OlmoForCausalLM":
        return DecoderSpec(norm="ln_noaffine")
    if arch == "ArceeForCausalLM":
        names = [n for n in _LLAMA_NAMES if "gate|up|down" not in n[0]] + [
            (r"(?:model\.)?layers\.(\d+)\.mlp\.up_proj\.(weight|bias)", r"L.\1.fc.\2"),
            (r"(?:model\.)?layers\.(\d+)\.mlp\.down_proj\.(weight|bias)", r"L.\1.down.\2")]
        return DecoderSpec(mlp="plain", names=names)
    raise NotImplementedError(f"no decoder spec for {arch}")


from ome_amd.models.config import PADDED_HEAD_ARCHS as DECODER_ARCHS  # noqa: E402,F401


def alibi_slopes(n: int, kind: str, bias_max: float = 8.0) -> torch.Tensor:
    """ALiBi slopes per head: Bloom/Falcon (``build_alibi_tensor``: geometric in the closest power
    of two, odd powers of the next one for the rest) or MPT (``1 / 2^(i * bias_max / n2)``,
    interleaved when ``n`` is not a power of two)."""
    if kind == "mpt":
        n2 = 2 ** math.ceil(math.log2(n))
        sl = 1.0 / torch.pow(2.0, torch.arange(1, n2 + 1, dtype=torch.float64) * (bias_max / n2))
        if n2 != n:
            sl = torch.cat([sl[1::2], sl[::2]])[:n]
        return sl.float()
    c = 2 ** math.floor(math.log2(n))
    base = 2.0 ** (-(2.0 ** -(math.log2(c) - 3)))
    sl = base ** torch.arange(1, 1 + c, dtype=torch.float64)
    if c != n:
        eb = 2.0 ** (-(2.0 ** -(math.log2(2 * c) - 3)))
        sl = torch.cat([sl, eb ** torch.arange(1, 1 + 2 * min(c, n - c), 2, dtype=torch.float64)])
    return sl.float()


def rope_layout(d_true: int, d_pad: int, rot: int, style: str) -> tuple[torch.Tensor | None, int]:
    """Map a family's RoPE geometry onto the kernel's NeoX rotate_half over ``rot_k`` dims.

    Returns ``(perm, rot_k)``: ``perm[j]`` is the original head dim placed at kernel dim ``j``
    (``>= d_true`` = a zero pad dim), or ``None`` when the identity works.  Pair ``i`` of the
    family (dims (i, i + rot/2) for NeoX, (2i, 2i+1) interleaved) lands on kernel dims
    (i, H + i) with H = rot/2 rounded up to a multiple of 8; kernel pairs i >= rot/2 rotate
    pass-through dims with the identity (see :func:`widen_table`)."""
    h = rot // 2
    if rot == 0 or (style == "neox" and h % 8 == 0 and d_true == d_pad):
        return None, rot
    H = -(-h // 8) * 8
    if 2 * H > d_pad:
        raise ValueError(f"rotary width {rot} cannot be laid out in head dim {d_pad}")
    if style == "interleaved":
        first, second = [2 * i for i in range(h)], [2 * i + 1 for i in range(h)]
    else:
        first, second = list(range(h)), [h + i for i in range(h)]
    used = set(first) | set(second)
    rest = [d for d in range(d_pad) if d not in used]  # pass-through dims, then pads
    perm = first + rest[: H - h] + second + rest[H - h: 2 * (H - h)] + rest[2 * (H - h):]
    return torch.tensor(perm, dtype=torch.long), 2 * H


def widen_table(cs: torch.Tensor, rot: int, rot_k: int) -> torch.Tensor:
    """[max_pos, rot] cos|sin table -> [max_pos, rot_k] with identity rotations appended."""
    if rot_k == rot:
        return cs
    h, H = rot // 2, rot_k // 2
    out = torch.zeros(cs.shape[0], rot_k, dtype=cs.dtype, device=cs.device)
    out[:, :H] = 1.0
    out[:, :h] = cs[:, :h]
    out[:, H:H + h] = cs[:, h:]
    return out


class DecoderForCausalLM(LlamaForCausalLM):
    """One forward for every :class:`DecoderSpec` family (weights as plain tensors, as in the
    Llama path; TP is Megatron-style with row-parallel biases added on rank 0 only)."""

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        self.spec = sp = _spec_for(cfg)
        hf = cfg.extra or {}
        self.Dt = cfg.attn_head_dim or self.D
        self.scale = 1.0 / math.sqrt(self.Dt)
        self.rot_true = int(round(cfg.partial_rotary_factor * self.D)) if sp.rope != "none" else 0
        self.perm, self.rot_k = rope_layout(self.Dt, self.D, self.rot_true, sp.rope)
        if self.rot_k != self.rot_true:
            self.cos_sin = widen_table(self.cos_sin, self.rot_true, self.rot_k)
        # kernel positions of the checkpoint's head dims (pad dims excluded) and, per position,
        # the checkpoint dim it holds -- per-head q/k LayerNorm weights are gathered by it
        if self.perm is not None:
            pos = torch.nonzero(self.perm < self.Dt).flatten()
            self._true_dims, self._true_src = pos.to(self.device), self.perm[pos]
        elif self.Dt != self.D:
            self._true_dims, self._true_src = torch.arange(self.Dt, device=self.device), torch.arange(self.Dt)
        else:
            self._true_dims = self._true_src = None
        plain = ACT_PLAIN if sp.mlp == "plain" else ACT_GATED
        act = cfg.hidden_act
        if act not in plain:
            raise NotImplementedError(f"hidden_act {act!r} for a {sp.mlp} MLP")
        self.act = plain[act]
        self.clip_qkv = hf.get("clip_qkv")
        self.logit_scale = float(sp.logit_mult if sp.logit_mult is not None else (hf.get("logit_scale") or 1.0))
        if sp.attn_scale is not None:
            self.scale = float(sp.attn_scale)
        # per-layer RoPE on/off (SmolLM3 ``no_rope_layers``: 1 = rotate, 0 = NoPE)
        nrl = hf.get("no_rope_layers")
        self.rope_on = [bool(nrl[i]) if nrl else True for i in range(cfg.num_layers)]
        self.head_w: list[torch.Tensor] = []  # classification / reward head (weight, bias, ...)
        if sp.qk_norm == "rms_full" and self.tp.tp > cfg.num_kv_heads:
            raise NotImplementedError("full-width q/k RMSNorm with replicated KV heads")
        L = cfg.num_layers
        none = lambda: [None] * L  # noqa: E731
        self.ln1b, self.ln2b, self.b_o, self.w_fc, self.b_fc, self.b_d = none(), none(), none(), none(), none(), none()
        self.post_attn, self.post_mlp = none(), none()
        self.qnb, self.knb = none(), none()
        self.norm_b = self.lm_head_b = self.pos_embed = self.proj_in = self.proj_out = None
        self.emb_ln = self.emb_ln_b = None
        self.num_labels = int(hf.get("num_labels") or len(hf.get("id2label") or {}) or 1)
        self.alibi = None
        if sp.alibi:
            sl = alibi_slopes(cfg.num_heads, sp.alibi, float((hf.get("attn_config") or {}).get("alibi_bias_max", 8)))
            self.alibi = sl[self.tp.rank * self.tp.hq:(self.tp.rank + 1) * self.tp.hq].contiguous().to(self.device)

    # ------------------------------------------------------------------ norms
    def _norm(self, x, w, b):
        if self.spec.norm == "rms":
            return ops.rmsnorm(x, w, self.eps)
        return ops.layernorm(x, w if w is not None else self._ones, b, self.eps)

    def _add_norm(self, x, res, w, b):
        """In place: res <- x + res; x <- norm(res)."""
        if self.spec.norm == "rms":
            ops.fused_add_rmsnorm(x, res, w, self.eps)
        else:
            ops.fused_add_layernorm(x, res, w if w is not None else self._ones, b, self.eps)

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "DecoderForCausalLM":
        cfg, tp, D, sp = self.cfg, self.tp, self.D, self.spec
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 7919 * pstate.get().tp_rank)
        H, r0 = cfg.hidden_size, tp.rank == 0
        rows = (tp.hq + 2 * tp.hkv) * D
        zeros = lambda *s: torch.zeros(*s, dtype=self.dtype, device=self.device)  # noqa: E731
        ln = sp.norm in ("ln", "ln_nobias", "ln_noaffine")
        bias = cfg.attention_bias
        for i in self.layers:
            self.w_qkv[i] = self._alloc(rows, H, std=std, gen=gen)
            self.b_qkv[i] = self._alloc(rows, std=std, gen=gen) if bias else None
            self.w_o[i] = self._alloc(H, tp.hq * D, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
            self.b_o[i] = (self._alloc(H, std=std, gen=gen) if r0 else zeros(H)) if bias else None
            if self.Dt != D:  # zero the pad dims, as a padded checkpoint has them
                keep = torch.zeros(D, dtype=torch.bool, device=self.device)
                keep[self._true_dims] = True
                self.w_qkv[i].view(-1, D, H)[:, ~keep] = 0
                if self.b_qkv[i] is not None:
                    self.b_qkv[i].view(-1, D)[:, ~keep] = 0
                self.w_o[i].view(H, -1, D)[:, :, self.Dt:] = 0
            if sp.residual != "post":
                self.ln1[i] = self._alloc(H, std=None, gen=gen)
                self.ln2[i] = self._alloc(H, std=None, gen=gen)
                if ln and sp.norm == "ln":
                    self.ln1b[i], self.ln2b[i] = zeros(H), zeros(H)
            if sp.residual in ("sandwich", "post"):
                self.post_attn[i], self.post_mlp[i] = self._alloc(H, std=None, gen=gen), self._alloc(H, std=None, gen=gen)
            if i in getattr(self, "moe_layers", ()):  # experts allocated by DecoderMoEForCausalLM
                pass
            elif sp.mlp == "gated":
                self.w_gu[i] = self._alloc(2 * tp.inter, H, std=std, gen=gen)
            else:
                self.w_fc[i] = self._alloc(tp.inter, H, std=std, gen=gen)
                self.b_fc[i] = self._alloc(tp.inter, std=std, gen=gen) if bias else None
            if i not in getattr(self, "moe_layers", ()):
                self.w_d[i] = self._alloc(H, tp.inter, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
                self.b_d[i] = (self._alloc(H, std=std, gen=gen) if r0 else zeros(H)) if (bias and sp.mlp == "plain") \
                    else None
            if sp.qk_norm == "rms_head":
                self.qn[i], self.kn[i] = self._alloc(D, std=None, gen=gen), self._alloc(D, std=None, gen=gen)
            elif sp.qk_norm == "ln_head":
                self.qn[i] = self._alloc(tp.hq, self.Dt, std=None, gen=gen)
                self.kn[i] = self._alloc(tp.hkv, self.Dt, std=None, gen=gen)
            elif sp.qk_norm == "rms_full":
                self.qn[i], self.kn[i] = self._alloc(tp.hq * D, std=None, gen=gen), self._alloc(tp.hkv * D, std=None, gen=gen)
        self.embed = self._alloc(tp.vocab, H, std=1.0, gen=gen)
        if sp.embed_norm:
            self.emb_ln, self.emb_ln_b = self._alloc(H, std=None, gen=gen), zeros(H)
        if sp.pos_offset >= 0:
            self.pos_embed = self._alloc(cfg.max_position_embeddings + sp.pos_offset, H, std=std, gen=gen)
        self.norm = self._alloc(H, std=None, gen=gen)
        if sp.norm == "ln":
            self.norm_b = zeros(H)
        self.lm_head = self.embed if cfg.tie_word_embeddings else self._alloc(tp.vocab, H, std=std, gen=gen)
        if sp.lm_head_bias:
            self.lm_head_b = self._alloc(tp.vocab, std=std, gen=gen)
        if sp.head == "reward_mlp":
            self.head_w = [zeros(H), self._alloc(H, H, std=std, gen=gen), zeros(self.num_labels),
                           self._alloc(self.num_labels, H, std=std, gen=gen)]
        elif sp.head:
            self.head_w = [self._alloc(self.num_labels, H, std=std, gen=gen)]
        self._finish()
        return self

    def _rename(self, name: str):
        for p in self.spec.prefixes:
            if name.startswith(p):
                name = name[len(p):]
                break
        for pat, tmpl in self.spec.names:
            m = re.fullmatch(pat, name)
            if m:
                return m.expand(tmpl)
        return None

    def load_hf_weights(self, weights) -> "DecoderForCausalLM":
        cfg, tp = self.cfg, self.tp
        per: dict[int, dict[str, torch.Tensor]] = {}
        glob: dict[str, torch.Tensor] = {}
        for name, w in weights:
            key = self._rename(name)
            if key is None:
                continue
            if key.startswith("L."):
                _, i, rest = key.split(".", 2)
                if int(i) in self._layer_set:
                    per.setdefault(int(i), {})[rest] = w
            else:
                glob[key] = w
        put = lambda t: t.to(device=self.device, dtype=self.dtype).contiguous()  # noqa: E731
        if "embed" not in glob:
            raise ValueError("checkpoint has no token embedding")
        self.embed = put(self._vocab_shard(glob["embed"]))
        self.lm_head = put(self._vocab_shard(glob["lm_head.weight"])) if "lm_head.weight" in glob else self.embed
        if "lm_head.bias" in glob:
            self.lm_head_b = put(self._vocab_shard(glob["lm_head.bias"][:, None])[:, 0])
        self.norm = put(glob["norm.weight"]) if "norm.weight" in glob else None
        self.norm_b = put(glob["norm.bias"]) if "norm.bias" in glob else None
        if "pos_embed" in glob:
            self.pos_embed = put(glob["pos_embed"])
        sp = self.spec
        if sp.head:
            hk = sorted(k for k in glob if k.startswith("head."))
            self.head_w = [put(glob[k]) for k in hk]  # head.0.bias, head.0.weight, head.2.bias, head.2.weight
        if sp.lm_head_norm:
            self.lm_head = put(torch.nn.functional.normalize(glob["lm_head.weight"].float(), dim=-1)[
                self.tp.vocab_start:self.tp.vocab_end]) if "lm_head.weight" in glob else self.lm_head
            if self.lm_head.shape[0] < self.tp.vocab:
                self.lm_head = torch.cat([self.lm_head, self.lm_head.new_zeros(self.tp.vocab - self.lm_head.shape[0],
                                                                               self.lm_head.shape[1])], 0)
        if "emb_ln.weight" in glob:
            self.emb_ln, self.emb_ln_b = put(glob["emb_ln.weight"]), put(glob["emb_ln.bias"])
        if "proj_in.weight" in glob:
            self.proj_in, self.proj_out = put(glob["proj_in.weight"]), put(glob["proj_out.weight"])
        for i in self.layers:
            if i not in per:
                raise ValueError(f"checkpoint incomplete: layer {i} missing")
            self._load_layer(i, per.pop(i), put)
        self._finish()
        return self

    def _split_qkv(self, p: dict, kind: str):
        """Full (unsharded) q, k, v [rows, ...] of one layer from separate or fused tensors."""
        cfg, Dt = self.cfg, self.Dt
        nh, nkv = cfg.num_heads, cfg.num_kv_heads
        if f"q.{kind}" in p:
            return p[f"q.{kind}"], p[f"k.{kind}"], p[f"v.{kind}"]
        w = p.get(f"qkv.{kind}")
        if w is None:
            return None, None, None
        lay = self.spec.qkv_layout
        tail = w.shape[1:]
        if lay == "concat":
            return w.split([nh * Dt, nkv * Dt, nkv * Dt], 0)
        if lay == "heads3":
            t = w.reshape(nh, 3, Dt, *tail)
            return (t[:, 0].reshape(nh * Dt, *tail), t[:, 1].reshape(nh * Dt, *tail), t[:, 2].reshape(nh * Dt, *tail))
        if lay == "groups":  # Falcon-40B: [kv_groups, q_per_group + 2, Dt]
            g = nh // nkv
            t = w.reshape(nkv, g + 2, Dt, *tail)
            return (t[:, :g].reshape(nh * Dt, *tail), t[:, g].reshape(nkv * Dt, *tail),
                    t[:, g + 1].reshape(nkv * Dt, *tail))
        raise ValueError(lay)

    def _heads(self, t: torch.Tensor, n: int, rope: bool) -> torch.Tensor:
        """[n*Dt, ...] -> [n*D, ...]: zero-pad each head to the kernel tile and, for Q/K,
        apply the rope-layout permutation."""
        D, Dt = self.D, self.Dt
        if D == Dt and (self.perm is None or not rope):
            return t
        t = t.reshape(n, Dt, *t.shape[1:])
        if D != Dt:
            t = torch.cat([t, t.new_zeros(n, D - Dt, *t.shape[2:])], 1)
        if rope and self.perm is not None:
            t = t.index_select(1, self.perm.to(t.device))
        return t.reshape(n * D, *t.shape[2:])

    def _load_layer(self, i: int, p: dict, put) -> None:
        cfg, tp, D, Dt, sp = self.cfg, self.tp, self.D, self.Dt, self.spec
        nh, nkv, H = cfg.num_heads, cfg.num_kv_heads, cfg.hidden_size
        r0 = tp.rank == 0
        parts_w, parts_b = [], []
        for kind, parts in (("weight", parts_w), ("bias", parts_b)):
            q, k, v = self._split_qkv(p, kind)
            if q is None:
                continue
            q, k, v = self._heads(q, nh, True), self._heads(k, nkv, True), self._heads(v, nkv, False)
            parts += [q.narrow(0, tp.rank * tp.hq * D, tp.hq * D), k.narrow(0, tp.kv_start * D, tp.hkv * D),
                      v.narrow(0, tp.kv_start * D, tp.hkv * D)]
        self.w_qkv[i] = put(torch.cat(parts_w, 0))
        self.b_qkv[i] = put(torch.cat(parts_b, 0)) if parts_b else None
        wo = p["o.weight"]  # [H, nh*Dt] -> pad per head in the input dim, this rank's heads
        if D != Dt:
            wo = torch.cat([wo.reshape(H, nh, Dt), wo.new_zeros(H, nh, D - Dt)], 2).reshape(H, nh * D)
        self.w_o[i] = put(wo.narrow(1, tp.rank * tp.hq * D, tp.hq * D))
        if "o.bias" in p:
            self.b_o[i] = put(p["o.bias"]) if r0 else torch.zeros(H, dtype=self.dtype, device=self.device)
        self._load_mlp(i, p, put)
        for nm, wl, bl in (("ln1", self.ln1, self.ln1b), ("ln2", self.ln2, self.ln2b)):
            if f"{nm}.weight" in p:
                wl[i] = put(p[f"{nm}.weight"])
            if f"{nm}.bias" in p:
                bl[i] = put(p[f"{nm}.bias"])
        if "post_attn.weight" in p:
            self.post_attn[i], self.post_mlp[i] = put(p["post_attn.weight"]), put(p["post_mlp.weight"])
        self._load_qk_norm(i, p, put)

    def _load_mlp(self, i: int, p: dict, put) -> None:
        tp, sp, H = self.tp, self.spec, self.cfg.hidden_size
        r0 = tp.rank == 0

        def inter_rows(t):
            n = min(tp.inter, t.shape[0] - tp.rank * tp.inter)
            return t.narrow(0, tp.rank * tp.inter, n)

        if sp.mlp == "gated":
            if "gate_up.weight" in p:
                g, u = p["gate_up.weight"].chunk(2, 0)
            else:
                g, u = p["gate.weight"], p["up.weight"]
            self.w_gu[i] = put(torch.cat([inter_rows(g), inter_rows(u)], 0))
        else:
            self.w_fc[i] = put(inter_rows(p["fc.weight"]))
            if "fc.bias" in p:
                self.b_fc[i] = put(inter_rows(p["fc.bias"]))
        wd = p["down.weight"]
        self.w_d[i] = put(wd.narrow(1, tp.rank * tp.inter, min(tp.inter, wd.shape[1] - tp.rank * tp.inter)))
        if "down.bias" in p:
            self.b_d[i] = put(p["down.bias"]) if r0 else torch.zeros(H, dtype=self.dtype, device=self.device)

    def _load_qk_norm(self, i: int, p: dict, put) -> None:
        cfg, tp, D, Dt, sp = self.cfg, self.tp, self.D, self.Dt, self.spec
        if not sp.qk_norm:
            return
        for c, lst, blst, n, start, cnt in (("q", self.qn, self.qnb, cfg.num_heads, tp.rank * tp.hq, tp.hq),
                                            ("k", self.kn, self.knb, cfg.num_kv_heads, tp.kv_start, tp.hkv)):
            if sp.qk_norm == "rms_full":  # one weight over all heads' dims [n*Dt]
                w = self._heads(p[f"{c}_norm.weight"].reshape(n * Dt, 1), n, True)[:, 0]
                lst[i] = put(w.narrow(0, start * D, cnt * D))
                continue
            if sp.qk_norm_per_head_w:
                if f"{c}_norm.weight" in p:  # Cohere: [n, Dt]
                    w = p[f"{c}_norm.weight"].reshape(n, Dt)
                else:  # StableLM: one LayerNorm module per head
                    w = torch.stack([p[f"{c}_norm.h{h}"] for h in range(n)], 0)
                lst[i] = put(self._to_kernel_dims(w.narrow(0, start, cnt)))
            else:  # Persimmon: one LayerNorm (weight, bias) shared by every head
                lst[i] = put(self._to_kernel_dims(p[f"{c}_norm.weight"].reshape(1, Dt).expand(cnt, Dt)))
                if f"{c}_norm.bias" in p:
                    blst[i] = put(self._to_kernel_dims(p[f"{c}_norm.bias"].reshape(1, Dt).expand(cnt, Dt)))

    def _to_kernel_dims(self, w: torch.Tensor) -> torch.Tensor:
        """[heads, Dt] per-dim parameters in checkpoint order -> the order of the true dims in
        the kernel layout (what :meth:`_qk_prenorm` gathers)."""
        return w if self._true_src is None else w.index_select(1, self._true_src.to(w.device))

    def _finish(self) -> None:
        H = self.cfg.hidden_size
        self._ones = torch.ones(H, dtype=self.dtype, device=self.device)
        if self.norm is None:
            self.norm = None if self.spec.norm == "ln_noaffine" else self._ones
        self._post_load()

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in (self.emb_ln, self.emb_ln_b)
                                         if t is not None)
        for lst in (self.ln1b, self.ln2b, self.b_o, self.w_fc, self.b_fc, self.b_d, self.post_attn, self.post_mlp,
                    self.qnb, self.knb, [self.norm_b, self.lm_head_b, self.pos_embed, self.proj_in, self.proj_out]):
            n += sum(t.numel() * t.element_size() for t in lst if isinstance(t, torch.Tensor))
        return n

    # ------------------------------------------------------------------ forward
    def _qk_prenorm(self, i: int, qkv: torch.Tensor) -> None:
        """q/k norms the fused RoPE kernel does not do itself, in place on the QKV rows."""
        tp, D, mode = self.tp, self.D, self.spec.qk_norm
        T = qkv.shape[0]
        q = qkv[:, : tp.hq * D]
        k = qkv[:, tp.hq * D:(tp.hq + tp.hkv) * D]
        if mode == "rms_full":
            for t, w, n in ((q, self.qn[i], self.cfg.num_heads), (k, self.kn[i], self.cfg.num_kv_heads)):
                ss = t.float().square().sum(-1, keepdim=True)
                if tp.tp > 1:
                    ss = pstate.tp_all_reduce(ss)
                t.copy_((t.float() * torch.rsqrt(ss / (n * self.Dt) + self.eps) * w.float()).to(t.dtype))
            return
        # per-head LayerNorm over the true head dims (pad dims stay zero)
        for t, w, b, n in ((q, self.qn[i], self.qnb[i], tp.hq), (k, self.kn[i], self.knb[i], tp.hkv)):
            v = t.view(T, n, D)
            x = v.float() if self._true_dims is None else v.index_select(2, self._true_dims).float()
            mu = x.mean(-1, keepdim=True)
            var = (x - mu).square().mean(-1, keepdim=True)
            y = (x - mu) * torch.rsqrt(var + self.eps) * w.float()
            if b is not None:
                y = y + b.float()
            if self._true_dims is None:
                v.copy_(y.to(t.dtype))
            else:
                v.index_copy_(2, self._true_dims, y.to(t.dtype))

    def _attn_block(self, i: int, x: torch.Tensor, meta: AttnMeta, kv: PagedKVCache) -> torch.Tensor:
        """Attention sub-block up to the row-parallel output projection (not yet reduced)."""
        tp, D, sp = self.tp, self.D, self.spec
        T = x.shape[0]
        qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
        if self.clip_qkv:
            qkv.clamp_(-self.clip_qkv, self.clip_qkv)
        if sp.qk_norm in ("ln_head", "rms_full"):
            self._qk_prenorm(i, qkv)
        q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
        k_cache, v_cache = kv.layer(i)
        ks, vs = kv.scales(i)
        kern_norm = sp.qk_norm == "rms_head"
        ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, self.rot_k, q, k_cache, v_cache, meta.slots,
                           tp.hq, tp.hkv, D, self.rot_k > 0 and self.rope_on[i], self.qn[i] if kern_norm else None,
                           self.kn[i] if kern_norm else None, self.eps, ks, vs)
        attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
        return linear(attn.view(T, tp.hq * D), self.w_o[i], self.b_o[i])

    def _mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        if self.spec.mlp == "gated":
            return linear(ops.act_and_mul(linear(x, self.w_gu[i]), self.act), self.w_d[i], self.b_d[i])
        h = linear(x, self.w_fc[i], self.b_fc[i])
        ops.act(h, self.act)
        return linear(h, self.w_d[i], self.b_d[i])

    def _embed(self, ids: torch.Tensor, meta: AttnMeta, input_embeds: torch.Tensor | None) -> torch.Tensor:
        if input_embeds is not None:
            return input_embeds
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if self.proj_in is not None:
            h = linear(h, self.proj_in)
        if self.pos_embed is not None:
            h = h + ops.embedding(meta.positions + self.spec.pos_offset, self.pos_embed)
        if self.emb_ln is not None:
            h = ops.layernorm(h, self.emb_ln, self.emb_ln_b, self.eps)
        if self.spec.embed_scale != 1.0:
            h = h * self.spec.embed_scale
        return h

    def attention(self, q, k_cache, v_cache, meta: AttnMeta, ks: float = 1.0, vs: float = 1.0) -> torch.Tensor:
        if self.alibi is None:
            return super().attention(q, k_cache, v_cache, meta, ks, vs)
        al = self.alibi
        if meta.is_decode:
            return ops.paged_decode(q, k_cache, v_cache, meta.block_tables, meta.seq_lens, self.scale,
                                    meta.decode_ws, self.window, order=meta.order, k_scale=ks, v_scale=vs, alibi=al)
        if meta.mode == "mixed":
            n = meta.num_prefill
            out = torch.empty_like(q)
            ops.paged_prefill(q[:n], k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                              self.scale, self.window, out=out[:n], k_scale=ks, v_scale=vs, alibi=al)
            ops.paged_decode(q[n:], k_cache, v_cache, meta.dec_block_tables, meta.seq_lens, self.scale,
                             meta.decode_ws, self.window, out=out[n:], order=meta.order, k_scale=ks, v_scale=vs,
                             alibi=al)
            return out
        return ops.paged_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                                 self.scale, self.window, k_scale=ks, v_scale=vs, alibi=al)

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        st, mode = pstate.get(), self.spec.residual
        T, H = ids.shape[0], self.cfg.hidden_size
        rs = self.spec.residual_scale

        def ar(t):  # TP all-reduce of a block output (+ Granite / MiniCPM residual scaling)
            t = pstate.tp_all_reduce(t)
            return t if rs == 1.0 else t.mul_(rs)

        if st.pp_size > 1 and not st.is_first_pp:
            x, residual = pstate.pp_recv(((T, H), self.dtype, ids.device), ((T, H), self.dtype, ids.device))
        else:
            h = self._embed(ids, meta, input_embeds)
            first = self.layers[0]
            if mode == "post":
                x, residual = torch.zeros_like(h), h
            elif mode == "post_ln":
                x, residual = h, None
            else:
                x, residual = self._norm(h, self.ln1[first], self.ln1b[first]), h
        for i in self.layers:
            if mode == "post_ln":  # OPT-350m: h = LN(h + attn(h)); h = LN(h + mlp(h))
                a = ar(self._attn_block(i, x, meta, kv))
                self._add_norm(a, x, self.ln1[i], self.ln1b[i])
                m = ar(self._mlp(i, a))
                self._add_norm(m, a, self.ln2[i], self.ln2b[i])
                x = m
                continue
            if mode == "post":  # OLMo-2: h += norm(attn(h)); h += norm(mlp(h))
                residual.add_(x)
                a = ops.rmsnorm(ar(self._attn_block(i, residual, meta, kv)), self.post_attn[i], self.eps)
                residual.add_(a)
                x = ops.rmsnorm(ar(self._mlp(i, residual)), self.post_mlp[i], self.eps)
                continue
            if i > 0:
                self._add_norm(x, residual, self.ln1[i], self.ln1b[i])
            if mode == "parallel_shared":
                x = ar(self._attn_block(i, x, meta, kv) + self._mlp(i, x))
            elif mode == "parallel":
                x2 = self._norm(residual, self.ln2[i], self.ln2b[i])
                x = ar(self._attn_block(i, x, meta, kv) + self._mlp(i, x2))
            else:  # seq / sandwich
                o = ar(self._attn_block(i, x, meta, kv))
                if mode == "sandwich":
                    o = ops.rmsnorm(o, self.post_attn[i], self.eps)
                self._add_norm(o, residual, self.ln2[i], self.ln2b[i])
                x = ar(self._mlp(i, o))
                if mode == "sandwich":
                    x = ops.rmsnorm(x, self.post_mlp[i], self.eps)
        if st.pp_size > 1 and not st.is_last_pp:
            pstate.pp_send(x, residual if residual is not None else x)
            return None
        if mode == "post_ln":
            return x if self.proj_out is None else linear(x, self.proj_out)
        if mode == "post":
            residual.add_(x)
            return ops.rmsnorm(residual, self.norm, self.eps)
        self._add_norm(x, residual, self.norm, self.norm_b)
        return x if self.proj_out is None else linear(x, self.proj_out)

    def pool(self, hidden: torch.Tensor, cu: torch.Tensor) -> torch.Tensor:
        """Embedding / reward / classification output per sequence (rows ``cu[s]:cu[s+1]``):
        last-token pooling, then the model's head (scores, un-normalised) or L2 normalisation."""
        if not self.spec.head:
            return ops.pool(hidden, cu, 0, True)
        last = hidden.index_select(0, (cu[1:] - 1).long())
        w = self.head_w
        if self.spec.head == "reward_mlp":  # score = Linear(ReLU(Linear(h)))
            return linear(torch.relu(linear(last, w[1], w[0])), w[3], w[2]).float()
        return linear(last, w[-1], w[0] if len(w) > 1 else None).float()

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        logits = linear(hidden, self.lm_head, self.lm_head_b)
        if self.tp.tp > 1:
            logits = pstate.tp_all_gather(logits, dim=-1)
        logits = logits[:, : self.cfg.vocab_size]
        if self.logit_scale != 1.0:
            logits = logits * self.logit_scale
        return logits

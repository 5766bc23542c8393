"""Model architecture config for the first-party runtime (parsed from HF ``config.json``).

Covers the dense decoder families of the reference runtime catalog (Llama 2/3/3.1/3.2,
Mistral, Qwen2/2.5, Qwen3, and their embedding variants) and the MoE families
(Mixtral, Qwen2/3-MoE, DeepSeek-V2/V3-style); see ``config/runtimes`` of the reference
(``config/runtimes/srt/meta/llama-3-8b-instruct-rt.yaml``) for the architectures it serves.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any

import torch


# dense families of ``models/decoder.py`` (zero-padded head dims are handled there)
PADDED_HEAD_ARCHS = {"Phi3SmallForCausalLM", "OPTForCausalLM", "GPTJForCausalLM", "FalconForCausalLM", "RWForCausalLM",
                     "StableLmForCausalLM", "PersimmonForCausalLM", "CohereForCausalLM", "GlmForCausalLM",
                     "Glm4ForCausalLM", "Olmo2ForCausalLM", "OlmoForCausalLM", "ArceeForCausalLM",
                     "BloomForCausalLM", "MptForCausalLM", "MPTForCausalLM", "Phi3ForCausalLM", "GraniteForCausalLM",
                     "SmolLM3ForCausalLM", "InternLM2ForCausalLM", "InternLM2ForRewardModel", "Qwen2ForRewardModel",
                     "LlamaForSequenceClassification", "Qwen2ForSequenceClassification",
                     "MistralForSequenceClassification", "MiMoForCausalLM", "QWenLMHeadModel", "BaichuanForCausalLM",
                     "ExaoneForCausalLM", "OrionForCausalLM", "MiniCPMForCausalLM", "ChatGLMModel", "Phi3VForCausalLM",
                     "ChatGLMForConditionalGeneration", "OlmoeForCausalLM", "GraniteMoeForCausalLM", "DbrxForCausalLM",
                     "Ernie4_5_MoeForCausalLM", "MiniMaxM2ForCausalLM"}
# remote-code class names that end in "Model" but are causal LMs (not embedding models)
CAUSAL_MODEL_CLASSES = {"ChatGLMModel", "QWenLMHeadModel", "TeleFLMModel", "InternVLChatModel", "LlavaLlamaModel"}
#: VILA / NVILA checkpoints: one sub-directory (own config.json + safetensors) per component;
#: tensors are read with the directory name as a prefix (``llm.model.layers.0...``)
NESTED_COMPONENTS = ("llm", "vision_tower", "mm_projector")


def _standard_keys(c: dict[str, Any]) -> dict[str, Any]:
    """Copy of an HF config with the family-specific key spellings (GPT-J ``n_embd``, OPT
    ``ffn_dim``, Falcon ``n_head`` / ``multi_query`` ...) also present under the standard names
    the parser reads.  Existing standard keys win."""
    mt = c.get("model_type", "")
    a: dict[str, Any] = {}
    if mt == "gptj":
        H, nh = c.get("n_embd", 4096), c.get("n_head", 16)
        a = dict(hidden_size=H, num_hidden_layers=c.get("n_layer"), num_attention_heads=nh,
                 intermediate_size=c.get("n_inner") or 4 * H, max_position_embeddings=c.get("n_positions"),
                 partial_rotary_factor=(c.get("rotary_dim") or H // nh) / (H // nh),
                 hidden_act=c.get("activation_function", "gelu_new"), layer_norm_eps=c.get("layer_norm_epsilon"),
                 attention_bias=False, rope_theta=10000.0)
    elif mt == "opt":
        a = dict(intermediate_size=c.get("ffn_dim"), hidden_act=c.get("activation_function", "relu"),
                 partial_rotary_factor=0.0, layer_norm_eps=1e-5, attention_bias=c.get("enable_bias", True),
                 tie_word_embeddings=c.get("tie_word_embeddings", True))
    elif mt == "falcon":
        nh = c.get("num_attention_heads") or c.get("n_head", 71)
        new, mq = c.get("new_decoder_architecture", False), c.get("multi_query", True)
        H = c.get("hidden_size", 4544)
        a = dict(num_attention_heads=nh, num_hidden_layers=c.get("num_hidden_layers") or c.get("n_layer"),
                 num_key_value_heads=(c.get("num_kv_heads") or nh) if new else (1 if mq else nh),
                 intermediate_size=c.get("ffn_hidden_size") or 4 * H, layer_norm_eps=c.get("layer_norm_epsilon"),
                 hidden_act=c.get("activation", "gelu"), attention_bias=c.get("bias", False),
                 tie_word_embeddings=c.get("tie_word_embeddings", True), multi_query=mq)
    elif mt == "bloom":
        H = c.get("hidden_size") or c.get("n_embed", 64)
        a = dict(hidden_size=H, num_hidden_layers=c.get("n_layer"), num_attention_heads=c.get("n_head"),
                 intermediate_size=4 * H, hidden_act="gelu_pytorch_tanh", layer_norm_eps=c.get("layer_norm_epsilon"),
                 partial_rotary_factor=0.0, attention_bias=True, tie_word_embeddings=c.get("tie_word_embeddings", True))
    elif mt == "mpt":
        H = c.get("d_model", 2048)
        ac = c.get("attn_config") or {}
        a = dict(hidden_size=H, num_hidden_layers=c.get("n_layers"), num_attention_heads=c.get("n_heads"),
                 intermediate_size=int(c.get("expansion_ratio", 4) * H), max_position_embeddings=c.get("max_seq_len"),
                 hidden_act="gelu", layer_norm_eps=c.get("layer_norm_epsilon") or 1e-5, partial_rotary_factor=0.0,
                 attention_bias=not c.get("no_bias", True), tie_word_embeddings=c.get("tie_word_embeddings", True),
                 clip_qkv=ac.get("clip_qkv"))
    elif mt == "qwen":  # Qwen (v1): intermediate_size is twice the per-projection width
        nh = c.get("num_attention_heads", 32)
        a = dict(intermediate_size=(c["intermediate_size"] // 2) if c.get("intermediate_size") else None,
                 rope_theta=c.get("rotary_emb_base", 10000.0), rms_norm_eps=c.get("layer_norm_epsilon"),
                 head_dim=c.get("kv_channels"), num_key_value_heads=nh, attention_bias=True,
                 max_position_embeddings=c.get("seq_length"), partial_rotary_factor=c.get("rotary_pct"))
    elif mt == "baichuan":
        a = dict(max_position_embeddings=c.get("model_max_length"), num_key_value_heads=c.get("num_attention_heads"))
    elif mt == "exaone":
        a = dict(num_hidden_layers=c.get("num_layers"), rms_norm_eps=c.get("layer_norm_epsilon"),
                 hidden_act=c.get("activation_function"))
    elif mt == "chatglm":
        mq = c.get("multi_query_attention", False)
        a = dict(num_hidden_layers=c.get("num_layers"), vocab_size=c.get("padded_vocab_size"),
                 head_dim=c.get("kv_channels"), intermediate_size=c.get("ffn_hidden_size"),
                 num_key_value_heads=c.get("multi_query_group_num") if mq else c.get("num_attention_heads"),
                 rms_norm_eps=c.get("layernorm_epsilon"), max_position_embeddings=c.get("seq_length"),
                 rope_theta=10000.0 * float(c.get("rope_ratio", 1.0)), partial_rotary_factor=0.5,
                 attention_bias=c.get("add_qkv_bias", True), tie_word_embeddings=False)
    elif mt == "internlm2":
        a = dict(attention_bias=c.get("bias", False))
    elif mt == "mimo":
        a = dict(attention_bias=True)
    elif mt == "dbrx":
        ac, fc = c.get("attn_config") or {}, c.get("ffn_config") or {}
        a = dict(hidden_size=c.get("d_model"), num_attention_heads=c.get("n_heads"), num_hidden_layers=c.get("n_layers"),
                 max_position_embeddings=c.get("max_seq_len"), num_key_value_heads=ac.get("kv_n_heads"),
                 rope_theta=ac.get("rope_theta"), clip_qkv=ac.get("clip_qkv"),
                 num_local_experts=fc.get("moe_num_experts"), num_experts_per_tok=fc.get("moe_top_k"),
                 intermediate_size=fc.get("ffn_hidden_size"), moe_intermediate_size=fc.get("ffn_hidden_size"),
                 norm_topk_prob=fc.get("moe_normalize_expert_weights") is not None, layer_norm_eps=1e-5,
                 hidden_act=(fc.get("ffn_act_fn") or {}).get("name", "silu"), tie_word_embeddings=False)
    elif mt == "ernie4_5_moe":
        a = dict(num_experts=c.get("moe_num_experts"), num_experts_per_tok=c.get("moe_k"),
                 attention_bias=c.get("use_bias", False), tie_word_embeddings=c.get("tie_word_embeddings", True))
    elif mt == "minimax_m2":
        hd = c.get("head_dim") or c.get("hidden_size", 3072) // c.get("num_attention_heads", 48)
        a = dict(partial_rotary_factor=(c["rotary_dim"] / hd) if c.get("rotary_dim") else None,
                 moe_intermediate_size=c.get("intermediate_size"))
    elif mt == "stablelm":
        a = dict(attention_bias=c.get("use_qkv_bias", False))
    elif mt == "persimmon":
        a = dict(attention_bias=True, hidden_act=c.get("hidden_act", "relu2"))
    elif mt == "phi3small":   # microsoft/Phi-3-small (remote code)
        a = dict(intermediate_size=c.get("ff_intermediate_size"), rope_theta=c.get("rope_embedding_base", 1e6),
                 layer_norm_eps=c.get("layer_norm_epsilon", 1e-5), attention_bias=True, tie_word_embeddings=False)
    elif mt in ("cohere", "olmo"):
        a = dict(layer_norm_eps=c.get("layer_norm_eps") or 1e-5, tie_word_embeddings=c.get("tie_word_embeddings",
                                                                                         mt == "cohere"))
    out = dict(c)
    for k, v in a.items():
        if v is not None and out.get(k) is None:
            out[k] = v
    return out



def _is_fp8_checkpoint(q: dict) -> bool:
    """FP8 weight checkpoints in any of the formats the reference catalog ships, all served as
    W8A8 with dynamic per-token activation scales (``models/quant.py``):
    ``quant_method: fp8`` / ``fbgemm_fp8`` (DeepSeek block scales, Meta per-row scales),
    ``compressed-tensors`` with 8-bit float weights (RedHatAI ``*-FP8-dynamic``: per-channel
    ``weight_scale``), and NVIDIA ModelOpt ``quant_algo: FP8`` (per-tensor ``weight_scale``)."""
    m = str(q.get("quant_method") or q.get("quant_type") or "").lower()
    if m in ("fp8", "fbgemm_fp8"):
        return True
    if m == "compressed-tensors":
        for grp in (q.get("config_groups") or {}).values():
            w = (grp or {}).get("weights") or {}
            if int(w.get("num_bits") or 0) == 8 and str(w.get("type", "")).lower() == "float":
                return True
        return False
    if m == "modelopt":
        algo = q.get("quant_algo") or (q.get("quantization") or {}).get("quant_algo")
        return str(algo or "").upper() == "FP8"
    return False

@dataclass
class ModelConfig:
    architecture: str = "LlamaForCausalLM"
    model_type: str = "llama"
    hidden_size: int = 4096
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    attn_head_dim: int = 0  # true head dim when ``head_dim`` was padded to a kernel tile (Phi-2: 80 -> 128)
    intermediate_size: int = 14336
    vocab_size: int = 128256
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: dict | None = None
    partial_rotary_factor: float = 1.0
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False
    attention_bias: bool = False
    qk_norm: bool = False
    hidden_act: str = "silu"
    sliding_window: int | None = None
    torch_dtype: str = "bfloat16"
    # MoE
    num_experts: int = 0
    num_experts_per_tok: int = 0
    moe_intermediate_size: int = 0
    num_shared_experts: int = 0
    shared_expert_intermediate_size: int = 0
    norm_topk_prob: bool = True
    first_k_dense_replace: int = 0
    moe_layer_freq: int = 1
    routed_scaling_factor: float = 1.0
    scoring_func: str = "softmax"
    n_group: int = 1
    topk_group: int = 1
    # MLA (DeepSeek)
    kv_lora_rank: int = 0
    q_lora_rank: int = 0
    qk_nope_head_dim: int = 0
    qk_rope_head_dim: int = 0
    v_head_dim: int = 0
    quantization: str | None = None
    is_embedding: bool = False
    extra: dict = field(default_factory=dict)

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    @property
    def is_mla(self) -> bool:
        return self.kv_lora_rank > 0

    @property
    def rot_dim(self) -> int:
        return int(self.head_dim * self.partial_rotary_factor)

    def num_params(self) -> int:
        H, L, V = self.hidden_size, self.num_layers, self.vocab_size
        D = self.attn_head_dim or self.head_dim  # checkpoint head dim, not the kernel-tile padding
        attn = H * (self.num_heads * D) * 2 + H * (self.num_kv_heads * D) * 2
        if self.is_moe:
            mlp = self.num_experts * 3 * H * self.moe_intermediate_size + H * self.num_experts
            mlp += self.num_shared_experts * 3 * H * (self.shared_expert_intermediate_size or self.moe_intermediate_size)
        else:  # gated (SwiGLU / GeGLU) MLPs have 3 matrices; the LayerNorm families' fc1/fc2 have 2
            gated = self.architecture not in ("Starcoder2ForCausalLM", "GPTNeoXForCausalLM", "PhiForCausalLM",
                                              "OPTForCausalLM", "GPTJForCausalLM", "FalconForCausalLM",
                                              "RWForCausalLM", "PersimmonForCausalLM", "ArceeForCausalLM",
                                              "BloomForCausalLM", "MptForCausalLM")
            mlp = (3 if gated else 2) * H * self.intermediate_size
        emb = V * H * (1 if self.tie_word_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H

    @classmethod
    def from_hf(cls, cfg: dict[str, Any]) -> "ModelConfig":
        llm_cfg = cfg.get("llm_cfg") if isinstance(cfg.get("llm_cfg"), dict) else None
        if cfg.get("text_config") or cfg.get("llm_config") or cfg.get("language_config") or llm_cfg:
            # llm_config: InternVLChatModel; language_config: Janus / DeepSeek-VL2 originals;
            # llm_cfg: VILA / NVILA (LlavaLlamaModel)
            text = _standard_keys(cfg.get("text_config") or cfg.get("llm_config") or cfg.get("language_config")
                                  or llm_cfg)
        else:  # flat configs: keep the original keys (extra) next to the standard aliases
            cfg = text = _standard_keys(cfg)
        arch = (cfg.get("architectures") or ["LlamaForCausalLM"])[0]
        H = text.get("hidden_size", 4096)
        nh = text.get("num_attention_heads", 32)
        hd = text.get("head_dim") or H // nh
        mt = text.get("model_type", cfg.get("model_type", "llama"))
        rope_theta = text.get("rope_theta", text.get("rotary_emb_base", 10000.0))
        rope_scaling = text.get("rope_scaling")
        prf = text.get("partial_rotary_factor")
        if prf is None:  # 0 is meaningful (no RoPE: OPT's learned positions)
            prf = text.get("rotary_pct") or 1.0
        rp = text.get("rope_parameters")  # transformers >= 5: {rope_type, rope_theta, ...} or per layer type
        if isinstance(rp, dict) and rp:
            glob = rp.get("full_attention", rp) if ("full_attention" in rp or "sliding_attention" in rp) else rp
            rope_theta = glob.get("rope_theta", rope_theta)
            prf = glob.get("partial_rotary_factor") or prf
            if glob.get("rope_type", "default") != "default":
                rope_scaling = dict(glob)
        attn_hd = 0
        if (mt == "phi" or arch in PADDED_HEAD_ARCHS) and hd not in (64, 128, 256):
            # the attention / RoPE-KV kernels tile head_dim in {64, 128, 256}: zero-pad each head
            # (q/k pad dims add 0 to every score, v pad dims feed zero columns of the padded o_proj)
            pad = next(d for d in (64, 128, 256) if d >= hd)
            attn_hd, prf, hd = hd, int(hd * float(prf)) / pad, pad
        c = cls(
            architecture=arch,
            model_type=mt,
            hidden_size=H,
            num_layers=len(text["layers_block_type"]) if text.get("layers_block_type") else
            len(text["hybrid_override_pattern"]) if text.get("hybrid_override_pattern") else
            text.get("num_hidden_layers", 32),
            num_heads=nh,
            num_kv_heads=text.get("num_key_value_heads") or nh,
            head_dim=hd,
            attn_head_dim=attn_hd,
            intermediate_size=text.get("intermediate_size", 4 * H),
            vocab_size=text.get("vocab_size", 32000),
            rms_norm_eps=text.get("rms_norm_eps") or text.get("layer_norm_eps") or text.get("norm_epsilon") or
            text.get("layer_norm_epsilon") or 1e-6,
            rope_theta=rope_theta,
            rope_scaling=rope_scaling,
            partial_rotary_factor=float(prf),
            max_position_embeddings=text.get("max_position_embeddings", 4096),
            tie_word_embeddings=bool(cfg.get("tie_word_embeddings", text.get("tie_word_embeddings", False))),
            attention_bias=bool(text.get("attention_bias", text.get("use_bias", mt in ("qwen2", "qwen2_moe", "qwen2_vl", "qwen2_vl_text", "qwen2_5_vl", "qwen2_5_vl_text", "phi")))),
            qk_norm=mt in ("qwen3", "qwen3_moe", "gemma3", "gemma3_text", "qwen3_vl", "qwen3_vl_text", "qwen3_vl_moe",
                           "qwen3_vl_moe_text", "qwen3_next"),
            hidden_act=text.get("hidden_act", text.get("hidden_activation", "silu")),
            sliding_window=text.get("sliding_window") if text.get("use_sliding_window", mt in ("mistral", "starcoder2", "phi3")) else None,
            torch_dtype=str(text.get("torch_dtype", cfg.get("torch_dtype", "bfloat16"))),
        )
        # MoE variants
        ne = text.get("num_local_experts") or text.get("num_experts") or text.get("n_routed_experts") or 0
        if ne:
            c.num_experts = ne
            c.num_experts_per_tok = text.get("num_experts_per_tok", 2)
            c.moe_intermediate_size = text.get("moe_intermediate_size") or text.get("intermediate_size")
            c.num_shared_experts = text.get("n_shared_experts") or (1 if text.get("shared_expert_intermediate_size") else 0)
            c.shared_expert_intermediate_size = text.get("shared_expert_intermediate_size") or 0
            c.norm_topk_prob = bool(text.get("norm_topk_prob", mt not in ("deepseek_v2",)))
            c.first_k_dense_replace = text.get("first_k_dense_replace", 0)
            c.moe_layer_freq = text.get("moe_layer_freq", 1) or 1
            c.routed_scaling_factor = text.get("routed_scaling_factor", 1.0) or 1.0
            # transformers' DeepSeek-V3 configs omit the key: that model always scores with sigmoid
            c.scoring_func = text.get("scoring_func", "sigmoid" if mt in ("deepseek_v3", "kimi_k2") else "softmax")
            c.n_group = text.get("n_group", 1) or 1
            c.topk_group = text.get("topk_group", 1) or 1
        if text.get("kv_lora_rank"):
            c.kv_lora_rank = text["kv_lora_rank"]
            c.q_lora_rank = text.get("q_lora_rank") or 0
            c.qk_nope_head_dim = text.get("qk_nope_head_dim", 128)
            c.qk_rope_head_dim = text.get("qk_rope_head_dim", 64)
            c.v_head_dim = text.get("v_head_dim", 128)
        q = cfg.get("quantization_config")
        if q:
            c.quantization = "fp8" if _is_fp8_checkpoint(q) else (q.get("quant_method") or q.get("quant_type"))
        c.is_embedding = ("Embedding" in arch) or arch.endswith(("ForSequenceClassification", "RewardModel")) or \
            (arch.endswith("Model") and "ForCausalLM" not in arch and arch not in CAUSAL_MODEL_CLASSES)
        if mt in ("roberta", "xlm-roberta") and c.max_position_embeddings > 2:
            # positions start at padding_idx + 1: the usable length is that much shorter
            c.max_position_embeddings -= int(text.get("pad_token_id", 1)) + 1
        c.extra = {k: v for k, v in cfg.items() if k not in ("text_config",)}
        if text is not cfg:  # multimodal wrappers: the language model's keys win
            c.extra.update({k: v for k, v in text.items() if k != "quantization_config"})
        return c

    @classmethod
    def from_path(cls, path: str | Path) -> "ModelConfig":
        p = Path(path)
        if p.is_dir():
            p = p / "config.json"
        cfg = json.loads(p.read_text())
        for comp in NESTED_COMPONENTS:   # VILA layout: component configs in sub-directories
            sub = p.parent / comp / "config.json"
            if not isinstance(cfg.get(comp + "_cfg"), dict) and sub.exists():
                cfg[comp + "_cfg"] = json.loads(sub.read_text())
        return cls.from_hf(cfg)

    def shrink(self, num_layers: int | None = None, **kw) -> "ModelConfig":
        import dataclasses

        return dataclasses.replace(self, num_layers=num_layers or self.num_layers, **kw)


# Canonical shapes (weights are random-init per BASELINE rules; these are the HF configs of
# the named models, cf. reference testdata pkg/hfutil/modelconfig/testdata/llama3.json etc.).
PRESETS: dict[str, dict] = {
    "llama-3-8b": dict(architectures=["LlamaForCausalLM"], model_type="llama", hidden_size=4096,
                       num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                       intermediate_size=14336, vocab_size=128256, rms_norm_eps=1e-5, rope_theta=500000.0,
                       max_position_embeddings=8192, torch_dtype="bfloat16"),
    "llama-3.1-8b": dict(architectures=["LlamaForCausalLM"], model_type="llama", hidden_size=4096,
                         num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                         intermediate_size=14336, vocab_size=128256, rms_norm_eps=1e-5, rope_theta=500000.0,
                         max_position_embeddings=131072,
                         rope_scaling={"factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                       "original_max_position_embeddings": 8192, "rope_type": "llama3"}),
    "llama-3-70b": dict(architectures=["LlamaForCausalLM"], model_type="llama", hidden_size=8192,
                        num_hidden_layers=80, num_attention_heads=64, num_key_value_heads=8,
                        intermediate_size=28672, vocab_size=128256, rms_norm_eps=1e-5, rope_theta=500000.0,
                        max_position_embeddings=8192),
    "qwen3-8b": dict(architectures=["Qwen3ForCausalLM"], model_type="qwen3", hidden_size=4096, num_hidden_layers=36,
                     num_attention_heads=32, num_key_value_heads=8, head_dim=128, intermediate_size=12288,
                     vocab_size=151936, rms_norm_eps=1e-6, rope_theta=1000000.0, max_position_embeddings=40960),
    "mixtral-8x7b": dict(architectures=["MixtralForCausalLM"], model_type="mixtral", hidden_size=4096,
                         num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                         intermediate_size=14336, num_local_experts=8, num_experts_per_tok=2, vocab_size=32000,
                         rms_norm_eps=1e-5, rope_theta=1000000.0, max_position_embeddings=32768),
    # BASELINE config 1 (operator plumbing on the CPU runtime): facebook/opt-125m
    "opt-125m": dict(architectures=["OPTForCausalLM"], model_type="opt", hidden_size=768, num_hidden_layers=12,
                     num_attention_heads=12, ffn_dim=3072, vocab_size=50272, max_position_embeddings=2048,
                     word_embed_proj_dim=768, do_layer_norm_before=True, activation_function="relu",
                     enable_bias=True, tie_word_embeddings=True, torch_dtype="float16"),
    "tiny-opt": dict(architectures=["OPTForCausalLM"], model_type="opt", hidden_size=256, num_hidden_layers=2,
                     num_attention_heads=4, ffn_dim=512, vocab_size=1024, max_position_embeddings=2048,
                     word_embed_proj_dim=256, do_layer_norm_before=True, activation_function="relu",
                     enable_bias=True, tie_word_embeddings=True),
    "falcon-7b": dict(architectures=["FalconForCausalLM"], model_type="falcon", hidden_size=4544,
                      num_hidden_layers=32, num_attention_heads=71, multi_query=True, parallel_attn=True,
                      new_decoder_architecture=False, bias=False, alibi=False, vocab_size=65024,
                      layer_norm_epsilon=1e-5, rope_theta=10000.0, max_position_embeddings=2048),
    "tiny-llama": dict(architectures=["LlamaForCausalLM"], model_type="llama", hidden_size=256, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, head_dim=128, intermediate_size=512,
                       vocab_size=1024, rms_norm_eps=1e-5, rope_theta=10000.0, max_position_embeddings=2048),
    "gemma-2-9b": dict(architectures=["Gemma2ForCausalLM"], model_type="gemma2", hidden_size=3584,
                       num_hidden_layers=42, num_attention_heads=16, num_key_value_heads=8, head_dim=256,
                       intermediate_size=14336, vocab_size=256000, rms_norm_eps=1e-6, rope_theta=10000.0,
                       max_position_embeddings=8192, sliding_window=4096, query_pre_attn_scalar=256,
                       attn_logit_softcapping=50.0, final_logit_softcapping=30.0, hidden_activation="gelu_pytorch_tanh",
                       tie_word_embeddings=True),
    "tiny-gemma2": dict(architectures=["Gemma2ForCausalLM"], model_type="gemma2", hidden_size=256, num_hidden_layers=2,
                        num_attention_heads=4, num_key_value_heads=2, head_dim=256, intermediate_size=512,
                        vocab_size=1024, rms_norm_eps=1e-6, rope_theta=10000.0, max_position_embeddings=2048,
                        sliding_window=64, query_pre_attn_scalar=256, attn_logit_softcapping=50.0,
                        final_logit_softcapping=30.0, hidden_activation="gelu_pytorch_tanh", tie_word_embeddings=True),
    "gpt-oss-20b": dict(architectures=["GptOssForCausalLM"], model_type="gpt_oss", hidden_size=2880,
                        num_hidden_layers=24, num_attention_heads=64, num_key_value_heads=8, head_dim=64,
                        intermediate_size=2880, num_local_experts=32, num_experts_per_tok=4, vocab_size=201088,
                        rms_norm_eps=1e-5, sliding_window=128, attention_bias=True, max_position_embeddings=131072,
                        rope_parameters={"rope_type": "yarn", "factor": 32.0, "beta_fast": 32.0, "beta_slow": 1.0,
                                         "truncate": False, "original_max_position_embeddings": 4096,
                                         "rope_theta": 150000.0}),
    "tiny-gpt-oss": dict(architectures=["GptOssForCausalLM"], model_type="gpt_oss", hidden_size=256,
                         num_hidden_layers=2, num_attention_heads=8, num_key_value_heads=2, head_dim=64,
                         intermediate_size=256, num_local_experts=8, num_experts_per_tok=2, vocab_size=1024,
                         rms_norm_eps=1e-5, sliding_window=32, attention_bias=True, max_position_embeddings=2048,
                         rope_parameters={"rope_type": "yarn", "factor": 8.0, "beta_fast": 32.0, "beta_slow": 1.0,
                                          "truncate": False, "original_max_position_embeddings": 256,
                                          "rope_theta": 150000.0}),
    "starcoder2-7b": dict(architectures=["Starcoder2ForCausalLM"], model_type="starcoder2", hidden_size=4608,
                          num_hidden_layers=32, num_attention_heads=36, num_key_value_heads=4,
                          intermediate_size=18432, vocab_size=49152, norm_epsilon=1e-5, rope_theta=1000000.0,
                          sliding_window=4096, max_position_embeddings=16384, use_bias=True,
                          hidden_act="gelu_pytorch_tanh", tie_word_embeddings=False),
    "tiny-starcoder2": dict(architectures=["Starcoder2ForCausalLM"], model_type="starcoder2", hidden_size=256,
                            num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                            intermediate_size=512, vocab_size=1024, norm_epsilon=1e-5, rope_theta=10000.0,
                            sliding_window=64, max_position_embeddings=2048, use_bias=True,
                            hidden_act="gelu_pytorch_tanh", tie_word_embeddings=True),
    "pythia-1.4b": dict(architectures=["GPTNeoXForCausalLM"], model_type="gpt_neox", hidden_size=2048,
                        num_hidden_layers=24, num_attention_heads=16, intermediate_size=8192, vocab_size=50304,
                        layer_norm_eps=1e-5, rotary_pct=0.25, rotary_emb_base=10000, use_parallel_residual=True,
                        hidden_act="gelu", max_position_embeddings=2048, attention_bias=True),
    "tiny-neox": dict(architectures=["GPTNeoXForCausalLM"], model_type="gpt_neox", hidden_size=256,
                      num_hidden_layers=2, num_attention_heads=4, intermediate_size=1024, vocab_size=1024,
                      layer_norm_eps=1e-5, rotary_pct=0.25, rotary_emb_base=10000, use_parallel_residual=True,
                      hidden_act="gelu", max_position_embeddings=2048, attention_bias=True),
    "phi-2": dict(architectures=["PhiForCausalLM"], model_type="phi", hidden_size=2560, num_hidden_layers=32,
                  num_attention_heads=32, num_key_value_heads=32, intermediate_size=10240, vocab_size=51200,
                  layer_norm_eps=1e-5, partial_rotary_factor=0.4, rope_theta=10000.0, hidden_act="gelu_new",
                  max_position_embeddings=2048, qk_layernorm=False, tie_word_embeddings=False),
    "tiny-phi": dict(architectures=["PhiForCausalLM"], model_type="phi", hidden_size=256, num_hidden_layers=2,
                     num_attention_heads=4, num_key_value_heads=4, intermediate_size=1024, vocab_size=1024,
                     layer_norm_eps=1e-5, partial_rotary_factor=0.5, rope_theta=10000.0, hidden_act="gelu_new",
                     max_position_embeddings=2048, qk_layernorm=False, tie_word_embeddings=False),
    "llama-4-scout-17b-16e": dict(architectures=["Llama4ForConditionalGeneration"], model_type="llama4",
                                  text_config=dict(model_type="llama4_text", hidden_size=5120, num_hidden_layers=48,
                                                   num_attention_heads=40, num_key_value_heads=8, head_dim=128,
                                                   intermediate_size=8192, intermediate_size_mlp=16384,
                                                   num_local_experts=16, num_experts_per_tok=1, vocab_size=202048,
                                                   rms_norm_eps=1e-5, max_position_embeddings=10485760,
                                                   attention_chunk_size=8192, interleave_moe_layer_step=1,
                                                   use_qk_norm=True, no_rope_layer_interval=4, floor_scale=8192,
                                                   attn_scale=0.1, attn_temperature_tuning=True,
                                                   rope_theta=500000.0,
                                                   rope_scaling={"rope_type": "llama3", "factor": 16.0,
                                                                 "low_freq_factor": 1.0, "high_freq_factor": 1.0,
                                                                 "original_max_position_embeddings": 8192})),
    "qwen2-vl-7b": dict(architectures=["Qwen2VLForConditionalGeneration"], model_type="qwen2_vl", hidden_size=3584,
                        num_hidden_layers=28, num_attention_heads=28, num_key_value_heads=4, intermediate_size=18944,
                        vocab_size=152064, rms_norm_eps=1e-6, rope_theta=1000000.0, max_position_embeddings=32768,
                        rope_scaling={"type": "mrope", "mrope_section": [16, 24, 24]}, image_token_id=151655,
                        video_token_id=151656, vision_start_token_id=151652, vision_end_token_id=151653,
                        vision_config=dict(depth=32, embed_dim=1280, hidden_size=3584, num_heads=16, mlp_ratio=4,
                                           patch_size=14, spatial_merge_size=2, temporal_patch_size=2,
                                           in_channels=3, hidden_act="quick_gelu")),
    # Qwen2.5-VL-7B-Instruct (also Qwen-Image's text encoder)
    "qwen2.5-vl-7b": dict(architectures=["Qwen2_5_VLForConditionalGeneration"], model_type="qwen2_5_vl",
                          hidden_size=3584, num_hidden_layers=28, num_attention_heads=28, num_key_value_heads=4,
                          intermediate_size=18944, vocab_size=152064, rms_norm_eps=1e-6, rope_theta=1000000.0,
                          max_position_embeddings=128000,
                          rope_scaling={"type": "mrope", "mrope_section": [16, 24, 24]}, image_token_id=151655,
                          video_token_id=151656, vision_start_token_id=151652, vision_end_token_id=151653,
                          vision_config=dict(depth=32, hidden_size=1280, num_heads=16, intermediate_size=3420,
                                             patch_size=14, spatial_merge_size=2, temporal_patch_size=2,
                                             in_channels=3, window_size=112, fullatt_block_indexes=[7, 15, 23, 31],
                                             out_hidden_size=3584, hidden_act="silu")),
    "tiny-qwen2-vl": dict(architectures=["Qwen2VLForConditionalGeneration"], model_type="qwen2_vl", hidden_size=256,
                          num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, intermediate_size=512,
                          vocab_size=1024, rms_norm_eps=1e-6, rope_theta=1000000.0, max_position_embeddings=4096,
                          rope_scaling={"type": "mrope", "mrope_section": [8, 12, 12]}, image_token_id=1000,
                          video_token_id=1003, vision_start_token_id=1001, vision_end_token_id=1002,
                          vision_config=dict(depth=2, embed_dim=128, hidden_size=256, num_heads=4, mlp_ratio=2,
                                             patch_size=14, spatial_merge_size=2, temporal_patch_size=2,
                                             in_channels=3, hidden_act="quick_gelu")),
    "nemotron-h-8b": dict(architectures=["NemotronHForCausalLM"], model_type="nemotron_h", hidden_size=4096,
                          hybrid_override_pattern="M-M-M-M*-M-M-M-M-M*-M-M-M-M-M*-M-M-M-M-M*-M-M-M-M-M-",
                          num_attention_heads=32, num_key_value_heads=8, head_dim=128, intermediate_size=21504,
                          mlp_hidden_act="relu2", mamba_num_heads=128, mamba_head_dim=64, ssm_state_size=128,
                          n_groups=8, conv_kernel=4, vocab_size=131072, layer_norm_epsilon=1e-5,
                          max_position_embeddings=8192, time_step_min=0.001, tie_word_embeddings=False),
    "tiny-nemotron-h": dict(architectures=["NemotronHForCausalLM"], model_type="nemotron_h", hidden_size=256,
                            hybrid_override_pattern="M-M*-M", num_attention_heads=4, num_key_value_heads=2,
                            head_dim=64, intermediate_size=512, mlp_hidden_act="relu2", mamba_num_heads=8,
                            mamba_head_dim=64, ssm_state_size=64, n_groups=2, conv_kernel=4, vocab_size=1024,
                            layer_norm_epsilon=1e-5, max_position_embeddings=4096, time_step_min=0.001),
    # Nemotron-3-Nano-30B-A3B shape (52 layers: Mamba-2 / MoE / attention, 128 ReLU^2 experts top-6)
    "nemotron-3-nano-30b-a3b": dict(architectures=["NemotronHForCausalLM"], model_type="nemotron_h",
                                    hidden_size=2688, num_attention_heads=32, num_key_value_heads=2, head_dim=128,
                                    hybrid_override_pattern="MEMEM*EMEMEM*EMEMEM*EMEMEM*EMEMEM*EMEMEMEM*EMEMEMEME",
                                    intermediate_size=1856, mlp_hidden_act="relu2", mamba_num_heads=64,
                                    mamba_head_dim=64, ssm_state_size=128, n_groups=8, conv_kernel=4,
                                    vocab_size=131072, layer_norm_epsilon=1e-5, max_position_embeddings=262144,
                                    time_step_min=0.001, n_routed_experts=128, num_experts_per_tok=6,
                                    moe_intermediate_size=1856, moe_shared_expert_intermediate_size=3712, n_group=1,
                                    topk_group=1, routed_scaling_factor=2.5, norm_topk_prob=True),
    "tiny-nemotron-h-moe": dict(architectures=["NemotronHForCausalLM"], model_type="nemotron_h", hidden_size=256,
                                hybrid_override_pattern="ME*EME", num_attention_heads=4, num_key_value_heads=2,
                                head_dim=64, intermediate_size=512, mlp_hidden_act="relu2", mamba_num_heads=8,
                                mamba_head_dim=64, ssm_state_size=64, n_groups=2, conv_kernel=4, vocab_size=1024,
                                layer_norm_epsilon=1e-5, max_position_embeddings=4096, time_step_min=0.001,
                                n_routed_experts=16, num_experts_per_tok=4, moe_intermediate_size=128,
                                moe_shared_expert_intermediate_size=256, n_group=4, topk_group=2,
                                routed_scaling_factor=2.5, norm_topk_prob=True),
    # NVILA-8B shape (VILA LlavaLlamaModel: Qwen2-7B LM, SigLIP-SO400M 448 px tower, Dynamic-S2 scales
    # 448 / 896 / 1344, mlp_downsample_3x3_fix projector)
    "nvila-8b": dict(architectures=["LlavaLlamaModel"], model_type="llava_llama",
                     llm_cfg=dict(architectures=["Qwen2ForCausalLM"], model_type="qwen2", hidden_size=3584,
                                  intermediate_size=18944, num_hidden_layers=28, num_attention_heads=28,
                                  num_key_value_heads=4, vocab_size=151648, rms_norm_eps=1e-6,
                                  rope_theta=1000000.0, max_position_embeddings=32768),
                     vision_tower_cfg=dict(hidden_size=1152, intermediate_size=4304, num_hidden_layers=27,
                                           num_attention_heads=16, image_size=448, patch_size=14),
                     mm_projector_cfg=dict(mm_projector_type="mlp_downsample_3x3_fix"), mm_vision_select_layer=-2,
                     image_aspect_ratio="dynamic_s2", s2_scales="448,896,1344", s2_max_split_size=448,
                     image_token_id=151649),
    "tiny-nvila": dict(architectures=["LlavaLlamaModel"], model_type="llava_llama",
                       llm_cfg=dict(model_type="qwen2", hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                    num_attention_heads=4, num_key_value_heads=2, vocab_size=1024,
                                    max_position_embeddings=4096),
                       vision_tower_cfg=dict(hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                             num_attention_heads=4, image_size=84, patch_size=14),
                       mm_projector_cfg=dict(mm_projector_type="mlp_downsample_3x3_fix"),
                       image_aspect_ratio="dynamic_s2", s2_scales="84,168,252", s2_max_split_size=84,
                       image_token_id=1000),
    # Jet-Nemotron-2B shape (Qwen2.5-1.5B backbone, 28 layers: JetBlocks + full attention at 15 / 20 and
    # sliding window at 21 / 22; JetBlock shape as published -- the remote config is not available offline)
    "jet-nemotron-2b": dict(architectures=["JetNemotronForCausalLM"], model_type="jet_nemotron", hidden_size=1536,
                            num_hidden_layers=28, num_attention_heads=12, num_key_value_heads=2,
                            intermediate_size=8960, vocab_size=151936, rms_norm_eps=1e-6, rope_theta=1000000.0,
                            max_position_embeddings=65536, tie_word_embeddings=True,
                            efficient_attention_config={"jet": dict(num_heads=6, head_dim=256, expand_v=2.0,
                                                                    conv_size=4, dconv_generator_reduction=8,
                                                                    norm_eps=1e-6),
                                                        "swa": {"window_size": 1152}}),
    "tiny-jet-nemotron": dict(architectures=["JetNemotronForCausalLM"], model_type="jet_nemotron", hidden_size=256,
                              num_hidden_layers=4, num_attention_heads=4, num_key_value_heads=2,
                              intermediate_size=512, vocab_size=1024, rms_norm_eps=1e-6, rope_theta=10000.0,
                              max_position_embeddings=4096, layer_types=["jet", "attn", "jet", "swa"],
                              efficient_attention_config={"jet": dict(num_heads=2, head_dim=128, expand_v=2.0,
                                                                      conv_size=4, dconv_generator_reduction=8),
                                                          "swa": {"window_size": 64}}),
    # Qwen3-Next-80B-A3B shape (48 layers: 3 Gated-DeltaNet + 1 gated attention, 512 experts top-10)
    "qwen3-next-80b-a3b": dict(architectures=["Qwen3NextForCausalLM"], model_type="qwen3_next", hidden_size=2048,
                               num_hidden_layers=48, num_attention_heads=16, num_key_value_heads=2, head_dim=256,
                               intermediate_size=5120, moe_intermediate_size=512,
                               shared_expert_intermediate_size=512, num_experts=512, num_experts_per_tok=10,
                               norm_topk_prob=True, linear_num_key_heads=16, linear_num_value_heads=32,
                               linear_key_head_dim=128, linear_value_head_dim=128, linear_conv_kernel_dim=4,
                               full_attention_interval=4, partial_rotary_factor=0.25, rope_theta=10000000.0,
                               vocab_size=151936, rms_norm_eps=1e-6, max_position_embeddings=262144),
    "tiny-qwen3-next": dict(architectures=["Qwen3NextForCausalLM"], model_type="qwen3_next", hidden_size=256,
                            num_hidden_layers=4, num_attention_heads=4, num_key_value_heads=2, head_dim=128,
                            intermediate_size=512, moe_intermediate_size=128, shared_expert_intermediate_size=128,
                            num_experts=8, num_experts_per_tok=2, norm_topk_prob=True, linear_num_key_heads=2,
                            linear_num_value_heads=4, linear_key_head_dim=128, linear_value_head_dim=128,
                            linear_conv_kernel_dim=4, full_attention_interval=4, partial_rotary_factor=0.25,
                            rope_theta=10000.0, vocab_size=1024, rms_norm_eps=1e-6, max_position_embeddings=4096),
    "tiny-llama4": dict(architectures=["Llama4ForCausalLM"], model_type="llama4_text", hidden_size=256,
                        num_hidden_layers=4, num_attention_heads=4, num_key_value_heads=2, head_dim=128,
                        intermediate_size=256, intermediate_size_mlp=512, num_local_experts=8, num_experts_per_tok=1,
                        vocab_size=1024, rms_norm_eps=1e-5, max_position_embeddings=4096, attention_chunk_size=64,
                        interleave_moe_layer_step=2, use_qk_norm=True, no_rope_layer_interval=4, floor_scale=32,
                        attn_scale=0.1, rope_theta=500000.0,
                        rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                      "high_freq_factor": 4.0, "original_max_position_embeddings": 256}),
    "tiny-moe": dict(architectures=["Qwen3MoeForCausalLM"], model_type="qwen3_moe", hidden_size=256,
                     num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, head_dim=128,
                     intermediate_size=512, moe_intermediate_size=128, num_experts=8, num_experts_per_tok=2,
                     vocab_size=1024, rms_norm_eps=1e-6, rope_theta=10000.0, max_position_embeddings=2048),
    # xai-org Grok-1 (hpcai-tech/grok-1 config.json) and Grok-2 (xai-org/grok-2, SGLang's keys)
    "grok-1": dict(architectures=["Grok1ModelForCausalLM"], model_type="grok-1", hidden_size=6144,
                   num_hidden_layers=64, num_attention_heads=48, num_key_value_heads=8, intermediate_size=32768,
                   num_experts=8, num_experts_per_tok=2, vocab_size=131072, rms_norm_eps=1e-5, rope_theta=10000.0,
                   max_position_embeddings=8192, attn_output_multiplier=0.08838834764831845, max_attn_value=30.0,
                   embedding_multiplier_scale=78.38367176906169, output_multiplier_scale=0.5773502691896257,
                   tie_word_embeddings=True),
    "grok-2": dict(architectures=["Grok1ForCausalLM"], model_type="grok-2", hidden_size=8192, num_hidden_layers=64,
                   num_attention_heads=64, num_key_value_heads=8, head_dim=128, intermediate_size=32768,
                   moe_intermediate_size=16384, num_local_experts=8, num_experts_per_tok=2, vocab_size=131072,
                   rms_norm_eps=1e-5, rope_theta=208533496.0, max_position_embeddings=131072, residual_moe=True,
                   attn_logit_softcapping=30.0, router_logit_softcapping=30.0, final_logit_softcapping=50.0,
                   embedding_multiplier_scale=90.50966799187809, output_multiplier_scale=0.5,
                   tie_word_embeddings=False),
    "tiny-grok1": dict(architectures=["Grok1ModelForCausalLM"], model_type="grok-1", hidden_size=256,
                       num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, intermediate_size=256,
                       num_experts=8, num_experts_per_tok=2, vocab_size=1024, rms_norm_eps=1e-5, rope_theta=10000.0,
                       max_position_embeddings=2048, attn_output_multiplier=0.125, max_attn_value=30.0,
                       embedding_multiplier_scale=16.0, output_multiplier_scale=0.5773502691896257,
                       tie_word_embeddings=True),
    "tiny-grok2": dict(architectures=["Grok1ForCausalLM"], model_type="grok-2", hidden_size=256, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, head_dim=64, intermediate_size=512,
                       moe_intermediate_size=128, num_local_experts=8, num_experts_per_tok=2, vocab_size=1024,
                       rms_norm_eps=1e-5, rope_theta=1000000.0, max_position_embeddings=2048, residual_moe=True,
                       attn_logit_softcapping=30.0, router_logit_softcapping=30.0, final_logit_softcapping=50.0,
                       embedding_multiplier_scale=16.0, output_multiplier_scale=0.5, tie_word_embeddings=False),
    # CofeAI/Tele-FLM (52B, muP multipliers)
    "tele-flm": dict(architectures=["TeleFLMModel"], model_type="teleflm", hidden_size=8192, num_hidden_layers=64,
                     num_attention_heads=64, num_key_value_heads=64, intermediate_size=21824, vocab_size=80000,
                     rms_norm_eps=1e-5, rope_theta=10000.0, max_position_embeddings=4096, use_mup=True,
                     input_mult=1.0, output_mult=1.0, mup_scale_factor=32.0, tie_word_embeddings=False),
    "tiny-teleflm": dict(architectures=["TeleFLMModel"], model_type="teleflm", hidden_size=256, num_hidden_layers=2,
                         num_attention_heads=4, num_key_value_heads=4, intermediate_size=512, vocab_size=1024,
                         rms_norm_eps=1e-5, rope_theta=10000.0, max_position_embeddings=2048, use_mup=True,
                         input_mult=3.0, output_mult=2.0, mup_scale_factor=8.0, tie_word_embeddings=False),
    "deepseek-v3": dict(architectures=["DeepseekV3ForCausalLM"], model_type="deepseek_v3", hidden_size=7168,
                        num_hidden_layers=61, num_attention_heads=128, num_key_value_heads=128,
                        intermediate_size=18432, moe_intermediate_size=2048, n_routed_experts=256,
                        n_shared_experts=1, num_experts_per_tok=8, first_k_dense_replace=3, moe_layer_freq=1,
                        n_group=8, topk_group=4, topk_method="noaux_tc", scoring_func="sigmoid", norm_topk_prob=True,
                        routed_scaling_factor=2.5, kv_lora_rank=512, q_lora_rank=1536, qk_nope_head_dim=128,
                        qk_rope_head_dim=64, v_head_dim=128, vocab_size=129280, rms_norm_eps=1e-6, rope_theta=10000.0,
                        max_position_embeddings=163840,
                        rope_scaling={"type": "yarn", "factor": 40, "original_max_position_embeddings": 4096,
                                      "beta_fast": 32, "beta_slow": 1, "mscale": 1.0, "mscale_all_dim": 1.0}),
    "deepseek-v2-lite": dict(architectures=["DeepseekV2ForCausalLM"], model_type="deepseek_v2", hidden_size=2048,
                             num_hidden_layers=27, num_attention_heads=16, num_key_value_heads=16,
                             intermediate_size=10944, moe_intermediate_size=1408, n_routed_experts=64,
                             n_shared_experts=2, num_experts_per_tok=6, first_k_dense_replace=1, n_group=1,
                             topk_group=1, topk_method="greedy", scoring_func="softmax", norm_topk_prob=False,
                             routed_scaling_factor=1.0, kv_lora_rank=512, q_lora_rank=None, qk_nope_head_dim=128,
                             qk_rope_head_dim=64, v_head_dim=128, vocab_size=102400, rms_norm_eps=1e-6,
                             rope_theta=10000.0, max_position_embeddings=163840),
    "tiny-deepseek": dict(architectures=["DeepseekV3ForCausalLM"], model_type="deepseek_v3", hidden_size=256,
                          num_hidden_layers=3, num_attention_heads=16, num_key_value_heads=16, intermediate_size=512,
                          moe_intermediate_size=64, n_routed_experts=16, n_shared_experts=1, num_experts_per_tok=4,
                          first_k_dense_replace=1, n_group=4, topk_group=2, topk_method="noaux_tc",
                          scoring_func="sigmoid", norm_topk_prob=True, routed_scaling_factor=2.5, kv_lora_rank=512,
                          q_lora_rank=128, qk_nope_head_dim=32, qk_rope_head_dim=64, v_head_dim=32, vocab_size=1024,
                          rms_norm_eps=1e-6, rope_theta=10000.0, max_position_embeddings=2048,
                          rope_scaling={"type": "yarn", "factor": 4, "original_max_position_embeddings": 512,
                                        "beta_fast": 32, "beta_slow": 1, "mscale": 1.0, "mscale_all_dim": 1.0}),
    "tiny-deepseek-v2": dict(architectures=["DeepseekV2ForCausalLM"], model_type="deepseek_v2", hidden_size=256,
                             num_hidden_layers=2, num_attention_heads=16, num_key_value_heads=16,
                             intermediate_size=512, moe_intermediate_size=64, n_routed_experts=16, n_shared_experts=2,
                             num_experts_per_tok=4, first_k_dense_replace=1, n_group=4, topk_group=2,
                             topk_method="group_limited_greedy", scoring_func="softmax", norm_topk_prob=False,
                             routed_scaling_factor=16.0, kv_lora_rank=512, q_lora_rank=None, qk_nope_head_dim=32,
                             qk_rope_head_dim=64, v_head_dim=32, vocab_size=1024, rms_norm_eps=1e-6,
                             rope_theta=10000.0, max_position_embeddings=2048),
}


def preset(name: str) -> ModelConfig:
    return ModelConfig.from_hf(PRESETS[name])


def rope_cos_sin(cfg: ModelConfig, max_pos: int, device=None) -> torch.Tensor:
    """[max_pos, rot_dim] float32 table: cos in the first half, sin in the second.

    Implements the HF rope_type variants used by the catalog: default, linear, dynamic (static
    at max_pos), llama3 (Llama-3.1 wavelength-band scaling) and yarn (DeepSeek / Qwen).
    """
    rot = cfg.rot_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, rot, 2, dtype=torch.float64) / rot))
    sc = cfg.rope_scaling or {}
    rtype = sc.get("rope_type", sc.get("type", "default"))
    mscale = 1.0
    pos = torch.arange(max_pos, dtype=torch.float64)
    if rtype == "linear":
        pos = pos / sc["factor"]
    elif rtype == "llama3":
        factor = sc["factor"]
        lf, hf = sc.get("low_freq_factor", 1.0), sc.get("high_freq_factor", 4.0)
        old = sc.get("original_max_position_embeddings", 8192)
        low_wl, high_wl = old / lf, old / hf
        wl = 2 * math.pi / inv
        smooth = (old / wl - lf) / (hf - lf)
        scaled = torch.where(wl > low_wl, inv / factor, inv)
        mid = (wl <= low_wl) & (wl >= high_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    elif rtype == "yarn":
        factor = sc["factor"]
        old = sc.get("original_max_position_embeddings", 4096)
        bf, bs = sc.get("beta_fast", 32), sc.get("beta_slow", 1)

        def corr(nrot):
            return (rot * math.log(old / (nrot * 2 * math.pi))) / (2 * math.log(cfg.rope_theta))

        if sc.get("truncate", True):
            lo, hi = max(math.floor(corr(bf)), 0), min(math.ceil(corr(bs)), rot - 1)
        else:  # GPT-OSS: unrounded correction range
            lo, hi = max(corr(bf), 0), min(corr(bs), rot - 1)
        ramp = torch.clamp((torch.arange(rot // 2, dtype=torch.float64) - lo) / max(hi - lo, 1e-3), 0, 1)
        extra = 1 - ramp
        inv = inv / factor * (1 - extra) + inv * extra
        ms, msa = sc.get("mscale", 1.0), sc.get("mscale_all_dim", 0.0)

        def ym(s, m):
            return 1.0 if s <= 1 else 0.1 * m * math.log(s) + 1.0

        mscale = ym(factor, ms) / ym(factor, msa) if msa else ym(factor, ms)
    elif rtype in ("longrope", "su"):
        # Phi-3 LongRoPE: per-frequency rescale factors -- the long set when the served context
        # exceeds the pre-training one (a long-context deployment, as HF does for such sequences;
        # one set for every position keeps cached keys consistent), else the short set
        old = sc.get("original_max_position_embeddings") or cfg.extra.get("original_max_position_embeddings") or \
            cfg.max_position_embeddings
        factor = sc.get("factor") or cfg.max_position_embeddings / old
        mscale = sc.get("attention_factor") or (1.0 if factor <= 1.0 else
                                                math.sqrt(1 + math.log(factor) / math.log(old)))
        inv = inv / torch.tensor(sc["long_factor" if max_pos > old else "short_factor"], dtype=torch.float64)
    elif rtype == "dynamic":
        factor = sc["factor"]
        old = cfg.max_position_embeddings
        if max_pos > old:
            base = cfg.rope_theta * ((factor * max_pos / old) - (factor - 1)) ** (rot / (rot - 2))
            inv = 1.0 / (base ** (torch.arange(0, rot, 2, dtype=torch.float64) / rot))
    freqs = torch.outer(pos, inv)
    cs = torch.cat([freqs.cos() * mscale, freqs.sin() * mscale], dim=-1).float()
    return cs.to(device) if device is not None else cs

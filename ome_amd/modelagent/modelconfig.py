"""Hugging Face model-config introspection (parity with ``pkg/hfutil/modelconfig``).

The reference keeps ~35 per-architecture Go loaders (``llama.go``, ``qwen3_moe.go``,
``deepseek_v3.go``, ...) that mostly map (hidden, layers) to nominal parameter counts.  Here a
single architecture-generic counter derives the **exact** parameter count from the config
fields every decoder family uses (with the per-family field-name aliases: ``n_embd`` /
``d_model`` / ``hidden_size``, ``multi_query_group_num``, ``ffn_config``, MLA ranks, MoE
expert counts, shared experts, ``first_k_dense_replace`` ...), plus nested ``text_config`` /
``vision_config`` for multimodal models.  When safetensors headers are present their tensor
shapes win (``safetensors.go:67-195`` semantics: sum of shape products, sharded via
``model.safetensors.index.json``).

Also provides ``format_param_count`` (``interface.go:170``), ``estimate_size_bytes``
(``interface.go:212``), capability detection (``config_parser.go:513``) and the
``ModelMetadata`` extraction the model agent writes into node ConfigMaps
(``config_parser.go:274-380``).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

from ome_amd.io.safetensors import count_params_in_dir

DTYPE_BYTES = {"float32": 4.0, "fp32": 4.0, "float16": 2.0, "fp16": 2.0, "half": 2.0, "bfloat16": 2.0, "bf16": 2.0,
               "float8_e4m3fn": 1.0, "float8_e5m2": 1.0, "fp8": 1.0, "int8": 1.0, "uint8": 1.0, "int4": 0.5,
               "float64": 8.0}

VISION_TYPES = ("vl", "vision", "llava", "mllama", "multi_modality", "phi3_v", "gemma3", "qwen3_5", "llama4",
                "janus", "deepseek_vl")


def format_param_count(n: int) -> str:
    for div, suf in ((10 ** 12, "T"), (10 ** 9, "B"), (10 ** 6, "M"), (10 ** 3, "K")):
        if n >= div:
            v = n / div
            if v == int(v):
                return f"{int(v)}{suf}"
            if round(v * 100) == v * 100:
                return f"{v:.1f}{suf}"
            return f"{v:.2f}{suf}"
    return str(n)


def format_size(n: int) -> str:
    for div, suf in ((1 << 40, "TB"), (1 << 30, "GB"), (1 << 20, "MB"), (1 << 10, "KB")):
        if n >= div:
            return f"{n / div:.2f} {suf}"
    return f"{n} B"


def estimate_size_bytes(params: int, dtype: str | None) -> int:
    return int(params * DTYPE_BYTES.get((dtype or "float32").lower(), 4.0))


def _g(cfg: dict, *names, default=None):
    for n in names:
        v = cfg.get(n)
        if v is not None:
            return v
    return default


# transformers defaults for fields that sub-configs commonly omit
TEXT_DEFAULTS = {
    "llama": {"hidden_size": 4096, "num_hidden_layers": 32, "num_attention_heads": 32, "intermediate_size": 11008,
              "vocab_size": 32000, "max_position_embeddings": 4096},
    "gemma3_text": {"max_position_embeddings": 131072, "vocab_size": 262208},
    "mistral": {"hidden_size": 4096, "num_hidden_layers": 32, "num_attention_heads": 32, "num_key_value_heads": 8,
                "intermediate_size": 14336, "vocab_size": 32000, "max_position_embeddings": 32768},
}


def text_params(cfg: dict) -> int:
    """Parameter count of a decoder/encoder LM described by ``cfg`` (text part only)."""
    H = int(_g(cfg, "hidden_size", "n_embd", "d_model", "dim", default=0))
    L = int(_g(cfg, "num_hidden_layers", "n_layer", "n_layers", "num_layers", default=0))
    if not H or not L:
        return 0
    V = int(_g(cfg, "padded_vocab_size", "vocab_size", default=32000))
    nh = int(_g(cfg, "num_attention_heads", "n_head", "n_heads", default=max(1, H // 128)))
    attn_cfg = cfg.get("attn_config") or {}
    nkv = int(_g(cfg, "num_key_value_heads", "multi_query_group_num", "n_kv_heads", default=None)
              or attn_cfg.get("kv_n_heads") or nh)
    if cfg.get("multi_query_attention") is False:
        nkv = nh
    hd = int(_g(cfg, "head_dim", "kv_channels", default=H // nh) or H // nh)
    ffn_cfg = cfg.get("ffn_config") or {}
    inter = int(_g(cfg, "intermediate_size", "ffn_hidden_size", "n_inner", "ffn_dim", default=0)
                or ffn_cfg.get("ffn_hidden_size") or 4 * H)
    mt = (cfg.get("model_type") or "").lower()
    if mt == "qwen":  # Qwen v1 stores 2x the per-projection width
        inter //= 2
    gated = mt not in ("bert", "roberta", "xlm-roberta", "gpt2", "gpt_neox", "phi", "stablelm_epoch", "clip_vision_model",
                       "starcoder2", "falcon", "opt", "gptj", "persimmon", "arcee")
    if mt in ("stablelm",):
        gated = True
    # attention
    inter_bias = 0
    q_lora = cfg.get("q_lora_rank")
    kv_lora = cfg.get("kv_lora_rank")
    if kv_lora:  # multi-head latent attention (DeepSeek-V2/V3, Kimi-K2, MiniCPM3)
        rope_d = int(cfg.get("qk_rope_head_dim", 64))
        nope_d = int(cfg.get("qk_nope_head_dim", 128))
        v_d = int(cfg.get("v_head_dim", 128))
        qk_d = rope_d + nope_d
        q = (H * q_lora + q_lora + q_lora * nh * qk_d) if q_lora else H * nh * qk_d
        kv = H * (kv_lora + rope_d) + kv_lora + kv_lora * nh * (nope_d + v_d)
        attn = q + kv + nh * v_d * H
    else:
        attn = H * nh * hd + 2 * H * nkv * hd + nh * hd * H
        if cfg.get("attention_bias") or cfg.get("qkv_bias") or mt in ("qwen2", "qwen", "bert", "chatglm"):
            attn += nh * hd + 2 * nkv * hd
        if mt == "opt" and cfg.get("enable_bias", True):  # every projection biased (q/k/v/out, fc1/fc2)
            attn += 3 * nh * hd + H
            inter_bias = inter + H
    # MLP / MoE
    n_exp = int(_g(cfg, "num_local_experts", "num_experts", "n_routed_experts", default=0) or ffn_cfg.get("moe_num_experts") or 0)
    mlp_dense = (3 if gated else 2) * H * inter + inter_bias
    if n_exp:
        moe_inter = int(_g(cfg, "moe_intermediate_size", default=0) or inter)
        shared = int(_g(cfg, "n_shared_experts", default=0) or 0) * 3 * H * moe_inter
        if cfg.get("shared_expert_intermediate_size"):
            shared = 3 * H * int(cfg["shared_expert_intermediate_size"]) + H
        moe = n_exp * 3 * H * moe_inter + H * n_exp + shared
        if cfg.get("interleave_moe_layer_step"):  # Llama-4: MoE every k-th layer + shared expert
            shared = 3 * H * moe_inter
            mlp_dense = 3 * H * int(cfg.get("intermediate_size_mlp") or inter)
            moe = n_exp * 3 * H * moe_inter + H * n_exp + shared
        k_dense = int(cfg.get("first_k_dense_replace", 0) or 0)
        step = int(cfg.get("decoder_sparse_step", 0) or cfg.get("interleave_moe_layer_step", 0) or 1)
        moe_layers = [i for i in range(k_dense, L) if (i + 1) % step == 0] if step > 1 else list(range(k_dense, L))
        mlp_total = len(moe_layers) * moe + (L - len(moe_layers)) * mlp_dense
    else:
        mlp_total = L * mlp_dense
    norms = 4 * H if mt in ("opt", "bert") else 2 * H  # LayerNorm weight + bias
    total = L * (attn + norms) + mlp_total
    total += V * H + H  # embeddings + final norm
    tied = cfg.get("tie_word_embeddings", cfg.get("tie_embeddings", mt in ("bert", "gemma", "gemma2", "gemma3_text")))
    if not tied and "Model" != (cfg.get("architectures") or [""])[0][-5:] and mt not in ("bert",):
        total += V * H
    if mt == "opt":  # learned positions (offset 2) and the final LayerNorm bias
        total += (int(cfg.get("max_position_embeddings", 2048)) + 2) * H + H
    if mt == "bert":
        total += int(cfg.get("max_position_embeddings", 512)) * H + int(cfg.get("type_vocab_size", 2)) * H
    return int(total)


def vision_params(vc: dict) -> int:
    H = int(_g(vc, "embed_dim", "width", "hidden_size", default=0))
    L = int(_g(vc, "num_hidden_layers", "depth", "layers", default=0))
    if not H or not L:
        return 0
    inter = int(_g(vc, "intermediate_size", default=4 * H))
    patch = int(_g(vc, "patch_size", default=14))
    per = 4 * H * H + 2 * H * inter + 4 * H
    return int(L * per + 3 * patch * patch * H)


@dataclass
class ModelInfo:
    model_type: str = ""
    architecture: str = ""
    context_length: int = 0
    param_count: int = 0
    torch_dtype: str = ""
    transformers_version: str = ""
    quantization: str = ""
    has_vision: bool = False
    is_embedding: bool = False
    size_bytes: int = 0
    diffusion: dict | None = None
    raw: dict = field(default_factory=dict)

    @property
    def parameter_size(self) -> str:
        return format_param_count(self.param_count)


def _context_length(cfg: dict) -> int:
    tc = cfg.get("text_config") or {}
    tc = {**TEXT_DEFAULTS.get(str(tc.get("model_type") or "").lower(), {}), **tc} if tc else tc
    for c in (cfg, tc):
        v = _g(c, "max_position_embeddings", "max_sequence_length", "seq_length", "n_positions", "model_max_length",
               "max_seq_len", default=None)
        if v:
            return int(v)
    return 0


def info_from_config(cfg: dict, model_dir: str | None = None) -> ModelInfo:
    archs = cfg.get("architectures") or []
    arch = archs[0] if archs else (cfg.get("_class_name") or "")
    mt = cfg.get("model_type") or ""
    tc = cfg.get("text_config") or cfg.get("language_config") or {}
    vc = cfg.get("vision_config") or cfg.get("vision_tower_config") or {}
    text = {**{k: v for k, v in cfg.items() if k not in ("text_config", "vision_config")}, **tc}
    if tc and not tc.get("model_type"):
        text["model_type"] = mt
    text = {**TEXT_DEFAULTS.get(str(text.get("model_type") or "").lower(), {}), **text}
    params = text_params(text) + (vision_params(vc) if vc else 0)
    if model_dir:
        st = count_params_in_dir(model_dir)
        if st:
            params = st
    dtype = str(cfg.get("torch_dtype") or tc.get("torch_dtype") or cfg.get("dtype") or "bfloat16")
    qc = cfg.get("quantization_config") or tc.get("quantization_config") or {}
    quant = str(qc.get("quant_method") or qc.get("quant_type") or "")
    if quant == "fp8" or "float8" in dtype or qc.get("fmt") == "e4m3":
        quant = "fp8"
    if qc.get("bits") == 4 or "int4" in str(qc).lower() or quant in ("awq", "gptq"):
        quant = quant or "int4"
    lo = (arch + " " + mt).lower()
    has_vision = bool(vc) or any(t in mt.lower() for t in VISION_TYPES) and "text" not in mt.lower()
    is_emb = (("embedding" in lo or "sentence" in lo or mt.lower() in ("bert", "roberta", "xlm-roberta"))
              or (mt.lower() == "mistral" and arch.lower() == "mistralmodel"))
    if model_dir and os.path.exists(os.path.join(model_dir, "config_sentence_transformers.json")):
        is_emb = True
    size_dtype = "fp8" if quant == "fp8" else ("int4" if quant in ("int4", "awq", "gptq") else dtype)
    return ModelInfo(model_type=mt, architecture=arch, context_length=_context_length(cfg), param_count=params,
                     torch_dtype=dtype, transformers_version=str(cfg.get("transformers_version") or ""),
                     quantization=quant, has_vision=has_vision, is_embedding=is_emb,
                     size_bytes=estimate_size_bytes(params, size_dtype), raw=cfg)


def load_model_config(path: str) -> ModelInfo:
    """``path`` is a model directory (``config.json`` / ``model_index.json``) or a config file."""
    if os.path.isdir(path):
        mi = os.path.join(path, "model_index.json")
        cj = os.path.join(path, "config.json")
        if not os.path.exists(cj) and os.path.exists(mi):
            with open(mi) as f:
                idx = json.load(f)
            info = ModelInfo(model_type="diffusers", architecture=idx.get("_class_name", ""),
                             transformers_version="", diffusion=idx, raw=idx)
            info.param_count = count_params_in_dir(path, recursive=True)
            info.size_bytes = estimate_size_bytes(info.param_count, "bfloat16")
            return info
        if not os.path.exists(cj):
            raise FileNotFoundError(f"no config.json or model_index.json under {path}")
        with open(cj) as f:
            return info_from_config(json.load(f), path)
    with open(path) as f:
        return info_from_config(json.load(f), None)


def capabilities(info: ModelInfo) -> list[str]:
    """``config_parser.go:513`` decision order: diffusion -> vision -> omni -> embedding -> text."""
    a = info.architecture.lower()
    if info.diffusion is not None:
        if any(k in a for k in ("imageedit", "pix2pix", "img2img", "inpaint")):
            return ["IMAGE_TEXT_TO_IMAGE"]
        if any(k in a for k in ("image", "pix", "stablediffusion")):
            return ["TEXT_TO_IMAGE"]
        if "texttovideo" in a or "t2v" in a:
            return ["TEXT_TO_VIDEO"]
        if "video" in a:
            return ["IMAGE_TEXT_TO_VIDEO"]
        return []
    if info.has_vision:
        return ["IMAGE_TEXT_TO_TEXT"]
    if "omni" in a:
        return ["TEXT_TO_AUDIO", "IMAGE_TEXT_TO_AUDIO", "VIDEO_TEXT_TO_AUDIO", "AUDIO_TO_TEXT", "AUDIO_TO_AUDIO"]
    if info.is_embedding:
        return ["EMBEDDING"]
    return ["TEXT_TO_TEXT"]


def model_metadata(info: ModelInfo) -> dict:
    """The ``ModelMetadata`` JSON stored in node ConfigMap entries (``model_data.go:45-67``)."""
    md = {"modelType": info.model_type, "modelArchitecture": info.architecture,
          "modelParameterSize": info.parameter_size, "maxTokens": info.context_length,
          "modelCapabilities": capabilities(info)}
    if info.diffusion is not None:
        ver = info.diffusion.get("_diffusers_version", "")
        md["modelFormat"] = {"name": "diffusers", "version": ver}
        md["modelFramework"] = {"name": "diffusers", "version": ver}
    else:
        md["modelFormat"] = {"name": "safetensors", "version": "1.0.0"}
        md["modelFramework"] = {"name": "transformers", **({"version": info.transformers_version}
                                                          if info.transformers_version else {})}
    q = info.quantization.lower()
    if "int4" in q or q in ("awq", "gptq"):
        md["quantization"] = "int4"
    elif "fp8" in q:
        md["quantization"] = "fp8"
    md["modelConfiguration"] = {"model_type": info.model_type, "architecture": info.architecture,
                                "context_length": info.context_length, "parameter_count": info.parameter_size,
                                "has_vision": info.has_vision, "is_embedding": info.is_embedding,
                                "transformers_version": info.transformers_version, "torch_dtype": info.torch_dtype,
                                "model_size_bytes": info.size_bytes}
    return md

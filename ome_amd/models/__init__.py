"""Model registry for the first-party runtime.

Architectures served (the HF ``architectures[0]`` names used by the reference's
ClusterServingRuntime catalog, ``config/runtimes/**``): dense Llama-family decoders and MoE
decoders.  ``load_format``: ``auto`` (safetensors if present, else random), ``safetensors``,
``dummy`` (random-init weights of the architecture — the BASELINE benchmark rule).
"""
from __future__ import annotations

from pathlib import Path

import torch

from ome_amd.models.config import ModelConfig

DENSE_ARCHS = {
    "LlamaForCausalLM", "MistralForCausalLM", "Qwen2ForCausalLM", "Qwen3ForCausalLM",
    "LlamaModel", "MistralModel", "Qwen2Model", "Qwen3Model",
}
GEMMA_ARCHS = {"GemmaForCausalLM", "Gemma2ForCausalLM", "Gemma3ForCausalLM", "Gemma3ForConditionalGeneration",
               "Gemma2ForSequenceClassification"}
LAYERNORM_ARCHS = {"Starcoder2ForCausalLM", "GPTNeoXForCausalLM", "PhiForCausalLM"}
LLAMA4_ARCHS = {"Llama4ForCausalLM", "Llama4ForConditionalGeneration"}
QWEN2_VL_ARCHS = {"Qwen2VLForConditionalGeneration", "Qwen2_5_VLForConditionalGeneration",
                  "Qwen3VLForConditionalGeneration", "Qwen3VLMoeForConditionalGeneration"}
NEMOTRON_H_ARCHS = {"NemotronHForCausalLM"}
from ome_amd.models.config import PADDED_HEAD_ARCHS as DECODER_ARCHS  # noqa: E402  (models/decoder.py)

ENCODER_ARCHS = {"BertModel", "BertForSequenceClassification", "RobertaModel", "RobertaForSequenceClassification",
                 "XLMRobertaModel", "XLMRobertaForSequenceClassification"}  # models/bert.py
MOE_ARCHS = {"MixtralForCausalLM", "Qwen2MoeForCausalLM", "Qwen3MoeForCausalLM", "DeepseekV2ForCausalLM",
             "DeepseekV3ForCausalLM", "PhiMoEForCausalLM"}


def model_class(cfg: ModelConfig):
    if cfg.architecture in ("Grok1ModelForCausalLM", "Grok1ForCausalLM") or cfg.model_type in ("grok-1", "grok1"):
        from ome_amd.models.grok import GrokForCausalLM

        return GrokForCausalLM
    if cfg.architecture in ("NemotronH_Nano_VL_V2", "NemotronVLForConditionalGeneration"):
        from ome_amd.models.nemotron_vl import nemotron_vl_class

        return nemotron_vl_class(cfg)
    if cfg.architecture in ("DotsOCRForConditionalGeneration", "DotsVLMForConditionalGeneration"):
        from ome_amd.models.dots import dots_class

        return dots_class(cfg)
    if cfg.architecture == "DeepseekVLV2ForCausalLM":
        from ome_amd.models.deepseek_vl2 import DeepseekVLV2ForCausalLM

        return DeepseekVLV2ForCausalLM
    if cfg.architecture == "MiniCPMV" or cfg.model_type == "minicpmv":
        from ome_amd.models.minicpmv import MiniCPMV

        return MiniCPMV
    if cfg.architecture == "Phi3VForCausalLM" or cfg.model_type == "phi3_v":
        from ome_amd.models.phi3v import Phi3VForCausalLM

        return Phi3VForCausalLM
    if cfg.architecture in ("TeleFLMModel", "TeleFLMForCausalLM") or cfg.model_type == "teleflm":
        from ome_amd.models.teleflm import TeleFLMForCausalLM

        return TeleFLMForCausalLM
    if cfg.architecture == "GptOssForCausalLM" or cfg.model_type == "gpt_oss":
        from ome_amd.models.gpt_oss import GptOssForCausalLM

        return GptOssForCausalLM
    if cfg.architecture == "Gemma3ForConditionalGeneration" and (cfg.extra or {}).get("vision_config"):
        from ome_amd.models.gemma3_vision import Gemma3ForConditionalGeneration

        return Gemma3ForConditionalGeneration
    if cfg.architecture in GEMMA_ARCHS or cfg.model_type in ("gemma", "gemma2", "gemma3", "gemma3_text"):
        from ome_amd.models.gemma import GemmaForCausalLM

        return GemmaForCausalLM
    if cfg.architecture in NEMOTRON_H_ARCHS or cfg.model_type == "nemotron_h":
        from ome_amd.models.nemotron_h import NemotronHForCausalLM

        return NemotronHForCausalLM
    if cfg.architecture == "JetNemotronForCausalLM" or cfg.model_type == "jet_nemotron":
        from ome_amd.models.jet_nemotron import JetNemotronForCausalLM

        return JetNemotronForCausalLM
    if cfg.architecture == "Qwen3NextForCausalLM" or cfg.model_type == "qwen3_next":
        from ome_amd.models.qwen3_next import Qwen3NextForCausalLM

        return Qwen3NextForCausalLM
    if cfg.architecture == "Glm4vMoeForConditionalGeneration" or cfg.model_type == "glm4v_moe":
        from ome_amd.models.glm4v import Glm4vMoeForConditionalGeneration

        return Glm4vMoeForConditionalGeneration
    if cfg.architecture in ("Qwen3VLForConditionalGeneration", "Qwen3VLMoeForConditionalGeneration"):
        from ome_amd.models.qwen3_vl import Qwen3VLForConditionalGeneration, Qwen3VLMoeForConditionalGeneration

        return Qwen3VLMoeForConditionalGeneration if cfg.is_moe else Qwen3VLForConditionalGeneration
    if cfg.architecture == "Qwen2_5_VLForConditionalGeneration" or cfg.model_type == "qwen2_5_vl":
        from ome_amd.models.qwen2_vl import Qwen2_5_VLForConditionalGeneration

        return Qwen2_5_VLForConditionalGeneration
    if cfg.architecture in QWEN2_VL_ARCHS or cfg.model_type == "qwen2_vl":
        from ome_amd.models.qwen2_vl import Qwen2VLForConditionalGeneration

        return Qwen2VLForConditionalGeneration
    if cfg.architecture == "Llama4ForConditionalGeneration" and (cfg.extra or {}).get("vision_config"):
        from ome_amd.models.llama4_vision import Llama4ForConditionalGeneration

        return Llama4ForConditionalGeneration
    if cfg.architecture in LLAMA4_ARCHS or cfg.model_type in ("llama4", "llama4_text"):
        from ome_amd.models.llama4 import Llama4ForCausalLM

        return Llama4ForCausalLM
    if cfg.architecture == "MllamaForConditionalGeneration" or cfg.model_type == "mllama":
        from ome_amd.models.mllama import MllamaForConditionalGeneration

        return MllamaForConditionalGeneration
    if cfg.architecture == "XverseMoeForCausalLM" or cfg.model_type == "xverse_moe":
        from ome_amd.models.xverse import XverseMoeForCausalLM

        return XverseMoeForCausalLM
    if cfg.architecture == "BailingMoeForCausalLM" or cfg.model_type == "bailing_moe":
        from ome_amd.models.bailing import BailingMoeForCausalLM

        return BailingMoeForCausalLM
    if cfg.architecture == "LlavaLlamaModel":
        from ome_amd.models.nvila import NVILAForCausalLM

        return NVILAForCausalLM
    if cfg.architecture in ("LlavaQwenForCausalLM", "LlavaOnevisionForConditionalGeneration"):
        from ome_amd.models.llava_onevision import LlavaOnevisionForConditionalGeneration

        return LlavaOnevisionForConditionalGeneration
    if cfg.architecture in ("JanusForConditionalGeneration", "MultiModalityCausalLM", "JanusMultiModalityCausalLM"):
        from ome_amd.models.janus import JanusForConditionalGeneration

        return JanusForConditionalGeneration
    if cfg.architecture in ("InternVLChatModel", "InternVLForConditionalGeneration"):
        from ome_amd.models.internvl import internvl_class

        return internvl_class(cfg)
    if cfg.architecture == "Mistral3ForConditionalGeneration" or cfg.model_type == "mistral3":
        from ome_amd.models.mistral3 import Mistral3ForConditionalGeneration

        return Mistral3ForConditionalGeneration
    if cfg.architecture == "CLIPModel":
        from ome_amd.models.clip import CLIPModel

        return CLIPModel
    if cfg.architecture == "LlavaNextForConditionalGeneration" or \
            (cfg.architecture == "LlavaLlamaForCausalLM" and "anyres" in str((cfg.extra or {}).get("image_aspect_ratio", ""))):
        from ome_amd.models.llava_next import LlavaNextForConditionalGeneration

        return LlavaNextForConditionalGeneration
    if cfg.architecture in ("LlavaForConditionalGeneration", "LlavaLlamaForCausalLM"):
        from ome_amd.models.llava import LlavaForConditionalGeneration

        return LlavaForConditionalGeneration
    if cfg.architecture == "DeciLMForCausalLM" or cfg.model_type == "nemotron-nas":
        from ome_amd.models.decilm import DeciLMForCausalLM

        return DeciLMForCausalLM
    if cfg.architecture in ENCODER_ARCHS:
        from ome_amd.models.bert import EncoderModel

        return EncoderModel
    if cfg.architecture in DECODER_ARCHS:
        from ome_amd.models.decoder_moe import DECODER_MOE_ARCHS, DecoderMoEForCausalLM

        if cfg.architecture in DECODER_MOE_ARCHS:
            return DecoderMoEForCausalLM
        if cfg.architecture == "QWenLMHeadModel" and (cfg.extra or {}).get("visual"):
            from ome_amd.models.qwen_vl import QwenVLForCausalLM

            return QwenVLForCausalLM
        if cfg.architecture == "Phi3SmallForCausalLM":
            from ome_amd.models.phi3small import Phi3SmallForCausalLM

            return Phi3SmallForCausalLM
        from ome_amd.models.decoder import DecoderForCausalLM

        return DecoderForCausalLM
    if cfg.architecture in LAYERNORM_ARCHS or cfg.model_type in ("starcoder2", "gpt_neox", "phi"):
        from ome_amd.models.layernorm_lm import LayerNormForCausalLM

        return LayerNormForCausalLM
    if cfg.architecture == "MiniCPM3ForCausalLM" or cfg.model_type == "minicpm3":
        from ome_amd.models.minicpm3 import MiniCPM3ForCausalLM

        return MiniCPM3ForCausalLM
    if cfg.architecture in ("Phi4MMForCausalLM", "Phi4MultimodalForCausalLM") or cfg.model_type == "phi4_multimodal":
        from ome_amd.models.phi4mm import Phi4MMForCausalLM

        return Phi4MMForCausalLM
    if cfg.architecture in ("KimiVLForConditionalGeneration", "Kimi_K25ForConditionalGeneration") or \
            cfg.model_type in ("kimi_vl", "kimi_k25"):
        from ome_amd.models.kimi_vl import KimiVLForConditionalGeneration

        return KimiVLForConditionalGeneration
    if cfg.is_mla:
        from ome_amd.models.deepseek import DeepseekForCausalLM

        return DeepseekForCausalLM
    if cfg.is_moe:
        from ome_amd.models.moe import MoEForCausalLM

        return MoEForCausalLM
    from ome_amd.models.llama import LlamaForCausalLM

    return LlamaForCausalLM


def supported(arch: str) -> bool:
    return arch in DENSE_ARCHS or arch in MOE_ARCHS or arch in GEMMA_ARCHS or arch in LAYERNORM_ARCHS or arch in LLAMA4_ARCHS or arch in QWEN2_VL_ARCHS or arch in NEMOTRON_H_ARCHS or \
        arch in DECODER_ARCHS or arch in ENCODER_ARCHS or arch == "MllamaForConditionalGeneration" or \
        arch == "DeciLMForCausalLM" or arch in ("LlavaForConditionalGeneration", "LlavaLlamaForCausalLM") or \
        arch == "LlavaNextForConditionalGeneration" or \
        arch == "CLIPModel" or arch == "Qwen3NextForCausalLM" or arch == "JetNemotronForCausalLM" or \
        arch == "LlavaLlamaModel" or \
        arch == "Mistral3ForConditionalGeneration" or arch == "MiniCPM3ForCausalLM" or \
        arch in ("InternVLChatModel", "InternVLForConditionalGeneration") or \
        arch in ("JanusForConditionalGeneration", "MultiModalityCausalLM", "JanusMultiModalityCausalLM") or \
        arch in ("LlavaQwenForCausalLM", "LlavaOnevisionForConditionalGeneration") or \
        arch in ("BailingMoeForCausalLM", "XverseMoeForCausalLM", "Glm4vMoeForConditionalGeneration") or \
        arch == "GptOssForCausalLM" or arch in ("KimiVLForConditionalGeneration", "Kimi_K25ForConditionalGeneration") or \
        arch in ("Phi4MMForCausalLM", "Phi4MultimodalForCausalLM") or \
        arch in ("Grok1ModelForCausalLM", "Grok1ForCausalLM") or arch in ("TeleFLMModel", "TeleFLMForCausalLM") or \
        arch == "Phi3VForCausalLM" or arch in ("NemotronH_Nano_VL_V2", "NemotronVLForConditionalGeneration") or \
        arch == "MiniCPMV" or arch == "DeepseekVLV2ForCausalLM" or \
        arch in ("DotsOCRForConditionalGeneration", "DotsVLMForConditionalGeneration") or \
        arch in ("QwenImagePipeline", "QwenImageEditPipeline", "QwenImageEditPlusPipeline")   # ome_amd.diffusion


def build_model(cfg: ModelConfig, device, dtype=torch.bfloat16, max_positions: int | None = None,
                model_path: str | None = None, load_format: str = "auto", seed: int = 0):
    if model_path:   # models that read side files of the checkpoint (tokenizer special-token ids)
        cfg.extra = {**(cfg.extra or {}), "_model_path": str(model_path)}
    cls = model_class(cfg)
    m = cls(cfg, device=device, dtype=dtype, max_positions=max_positions)
    fmt = load_format
    if fmt == "auto":
        from ome_amd.models.loader import has_checkpoint

        fmt = "safetensors" if model_path and has_checkpoint(model_path) else "dummy"
    if fmt == "dummy":
        m.init_random(seed)
    elif fmt == "safetensors":
        from ome_amd.models.loader import iter_safetensors

        plan = m.shard_plan if hasattr(m, "sharded") and m.sharded() else None
        if plan is not None:
            m._presliced = True   # every tensor arrives as this rank's shard
        m.load_hf_weights(iter_safetensors(model_path, device=device, plan=plan))
    else:
        raise ValueError(f"unknown load_format {load_format}")
    return m

"""Model + runtime catalog generator (reference: ``config/runtimes/**`` — 205 ClusterServingRuntimes —
and ``config/models/**`` — 205 ClusterBaseModels).

The reference hand-maintains one SGLang/vLLM runtime YAML per model and GPU count.  Here the
catalog is generated from one table of the model families the first-party runtime serves
(:data:`FAMILIES`), sized for MI355X: tensor parallelism is the smallest power of two that leaves
~40 % of each GPU's 288 GB HBM3E for the KV cache (Llama-3-70B bf16 and smaller run on ONE GPU,
Llama-4-Scout bf16 on two, Maverick / DeepSeek-V3 on a full 8-GPU xGMI node), plus
prefill/decode-disaggregated variants for the dense headline models and a two-node
leader/worker variant for DeepSeek-V3 bf16.  ``python -m ome_amd.catalog --out config`` writes
``config/runtimes/ome-amd/*.yaml`` and ``config/models/<vendor>/*.yaml``; ``tests/test_catalog_cpu.py``
checks every entry parses into the v1beta1 API types, names a supported architecture, passes the
runtime server's own flag parser, and is what the RuntimeSelector picks for its base model.
"""
from __future__ import annotations

import argparse
import copy
from dataclasses import dataclass, field
from pathlib import Path

import yaml

HBM_GB = 288.0
KV_HEADROOM = 0.6      # weights may use at most this fraction of a GPU
IMAGE = "ome-amd/runtime:rocm7.2-gfx950"


@dataclass
class Family:
    name: str                 # runtime / base model name stem
    vendor: str
    hf: str                   # hf:// repo of the real weights
    arch: str                 # HF architectures[0]
    params_b: float           # billions of parameters
    preset: str | None = None  # ome_amd preset for random:// (offline) weights
    bytes_per_param: float = 2.0
    capabilities: list[str] = field(default_factory=lambda: ["TEXT_TO_TEXT"])
    args: list[str] = field(default_factory=list)
    pd: bool = False          # also emit a prefill/decode-disaggregated runtime
    multinode: int = 0        # also emit a leader/worker runtime over this many nodes (bf16)
    quantization: str | None = None
    min_tp: int = 1           # e.g. DP attention over a whole node
    diffusion: str | None = None   # diffusers pipeline class: served by ome_amd.diffusion.server
    runtime: bool | None = None    # emit a runtime; None = only if no earlier family's runtime covers it
    grpc: bool = False        # also emit a gRPC-mode runtime (engine --grpc-mode, grpc.health.v1 probes)


FAMILIES: list[Family] = [
    Family("llama-3-8b-instruct", "meta", "meta-llama/Meta-Llama-3-8B-Instruct", "LlamaForCausalLM", 8.0,
           "llama-3-8b", pd=True),
    Family("llama-3-1-8b-instruct", "meta", "meta-llama/Llama-3.1-8B-Instruct", "LlamaForCausalLM", 8.0,
           "llama-3.1-8b", args=['--tool-call-parser', 'llama3_json'], pd=True, grpc=True),
    Family("llama-3-70b-instruct", "meta", "meta-llama/Meta-Llama-3-70B-Instruct", "LlamaForCausalLM", 70.6,
           "llama-3-70b", pd=True),
    Family("llama-3-1-405b-instruct-fp8", "meta", "meta-llama/Llama-3.1-405B-Instruct-FP8", "LlamaForCausalLM",
           405.0, None, 1.0, quantization="fp8", args=['--tool-call-parser', 'llama3_json'], multinode=2),
    Family("llama-4-scout-17b-16e-instruct", "meta", "meta-llama/Llama-4-Scout-17B-16E-Instruct",
           "Llama4ForConditionalGeneration", 109.0, "llama-4-scout-17b-16e",
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"], args=['--tool-call-parser', 'pythonic'], pd=True),
    Family("llama-4-maverick-17b-128e-instruct-fp8", "meta", "meta-llama/Llama-4-Maverick-17B-128E-Instruct-FP8",
           "Llama4ForConditionalGeneration", 402.0, None, 1.0, quantization="fp8",
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"], args=['--tool-call-parser', 'pythonic'], pd=True,
           grpc=True),
    Family("mistral-7b-instruct", "mistralai", "mistralai/Mistral-7B-Instruct-v0.3", "MistralForCausalLM", 7.2, pd=True),
    Family("mixtral-8x7b-instruct", "mistralai", "mistralai/Mixtral-8x7B-Instruct-v0.1", "MixtralForCausalLM",
           46.7, "mixtral-8x7b", pd=True),
    Family("qwen2-5-7b-instruct", "qwen", "Qwen/Qwen2.5-7B-Instruct", "Qwen2ForCausalLM", 7.6),
    Family("qwen2-5-72b-instruct", "qwen", "Qwen/Qwen2.5-72B-Instruct", "Qwen2ForCausalLM", 72.7),
    Family("qwen3-8b", "qwen", "Qwen/Qwen3-8B", "Qwen3ForCausalLM", 8.2, "qwen3-8b"),
    Family("qwen3-30b-a3b", "qwen", "Qwen/Qwen3-30B-A3B", "Qwen3MoeForCausalLM", 30.5),
    Family("qwen2-vl-7b-instruct", "qwen", "Qwen/Qwen2-VL-7B-Instruct", "Qwen2VLForConditionalGeneration", 8.3,
           "qwen2-vl-7b", capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("qwen2-5-vl-7b-instruct", "qwen", "Qwen/Qwen2.5-VL-7B-Instruct", "Qwen2_5_VLForConditionalGeneration", 8.3,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("mimo-vl-7b-rl", "xiaomimimo", "XiaomiMiMo/MiMo-VL-7B-RL", "Qwen2_5_VLForConditionalGeneration", 8.3,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("nvila-8b", "Efficient-Large-Model", "Efficient-Large-Model/NVILA-8B", "LlavaLlamaModel", 8.0, "nvila-8b",
           capabilities=["IMAGE_TEXT_TO_TEXT", "VIDEO_TEXT_TO_TEXT"]),
    Family("jet-nemotron-2b", "jet-ai", "jet-ai/Jet-Nemotron-2B", "JetNemotronForCausalLM", 2.0, "jet-nemotron-2b"),
    Family("qwen3-next-80b-a3b-instruct", "qwen", "Qwen/Qwen3-Next-80B-A3B-Instruct", "Qwen3NextForCausalLM", 81.3,
           "qwen3-next-80b-a3b", args=['--tool-call-parser', 'hermes']),
    Family("qwen3-next-80b-a3b-thinking", "qwen", "Qwen/Qwen3-Next-80B-A3B-Thinking", "Qwen3NextForCausalLM", 81.3,
           "qwen3-next-80b-a3b", args=['--reasoning-parser', 'deepseek-r1']),
    Family("mistral-small-3-1-24b-instruct-2503", "mistralai", "mistralai/Mistral-Small-3.1-24B-Instruct-2503",
           "Mistral3ForConditionalGeneration", 24.0, capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"],
           args=['--tool-call-parser', 'mistral']),
    Family("minicpm-v-2-6", "openbmb", "openbmb/MiniCPM-V-2_6", "MiniCPMV", 8.1,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("minicpm3-4b", "openbmb", "openbmb/MiniCPM3-4B", "MiniCPM3ForCausalLM", 4.1),
    Family("internvl2-5-8b", "opengvlab", "OpenGVLab/InternVL2_5-8B", "InternVLChatModel", 8.1,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("janus-pro-7b", "deepseek-ai", "deepseek-ai/Janus-Pro-7B", "JanusMultiModalityCausalLM", 7.4,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("llava-onevision-qwen2-7b-ov", "lmms-lab", "lmms-lab/llava-onevision-qwen2-7b-ov", "LlavaQwenForCausalLM",
           8.0, capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("llava-next-72b", "lmms-lab", "lmms-lab/llava-next-72b", "LlavaQwenForCausalLM", 72.7,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("ling-lite", "inclusionai", "inclusionAI/Ling-lite", "BailingMoeForCausalLM", 16.8),
    Family("ling-plus", "inclusionai", "inclusionAI/Ling-plus", "BailingMoeForCausalLM", 290.0),
    Family("xverse-moe-a36b", "xverse", "xverse/XVERSE-MoE-A36B", "XverseMoeForCausalLM", 255.0),
    Family("phi-4-multimodal-instruct", "microsoft", "microsoft/Phi-4-multimodal-instruct", "Phi4MMForCausalLM", 5.6,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("kimi-vl-a3b-instruct", "moonshotai", "moonshotai/Kimi-VL-A3B-Instruct", "KimiVLForConditionalGeneration",
           16.4, capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("glm-4-5v", "zai-org", "zai-org/GLM-4.5V", "Glm4vMoeForConditionalGeneration", 108.0,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("qwen3-vl-8b-instruct", "qwen", "Qwen/Qwen3-VL-8B-Instruct", "Qwen3VLForConditionalGeneration", 8.8,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("qwen3-vl-235b-a22b-instruct", "qwen", "Qwen/Qwen3-VL-235B-A22B-Instruct",
           "Qwen3VLMoeForConditionalGeneration", 236.0, None, 1.0, quantization="fp8",
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("llava-v1-5-13b", "liuhaotian", "liuhaotian/llava-v1.5-13b", "LlavaLlamaForCausalLM", 13.4,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("llava-1-5-7b-hf", "llava-hf", "llava-hf/llava-1.5-7b-hf", "LlavaForConditionalGeneration", 7.1,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("llama-3-2-11b-vision-instruct", "meta", "meta-llama/Llama-3.2-11B-Vision-Instruct",
           "MllamaForConditionalGeneration", 10.7, capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"], args=['--tool-call-parser', 'llama3_json']),
    Family("llama-3-2-90b-vision-instruct", "meta", "meta-llama/Llama-3.2-90B-Vision-Instruct",
           "MllamaForConditionalGeneration", 88.6, capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("deepseek-v2-lite-chat", "deepseek-ai", "deepseek-ai/DeepSeek-V2-Lite-Chat", "DeepseekV2ForCausalLM",
           15.7, "deepseek-v2-lite"),
    Family("deepseek-vl2", "deepseek-ai", "deepseek-ai/deepseek-vl2", "DeepseekVLV2ForCausalLM", 27.5,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("dots-ocr", "rednote-hilab", "rednote-hilab/dots.ocr", "DotsOCRForConditionalGeneration", 3.0,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("dots-vlm1-inst", "rednote-hilab", "rednote-hilab/dots.vlm1.inst", "DotsVLMForConditionalGeneration",
           672.0, capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"], min_tp=8),
    Family("deepseek-v3", "deepseek-ai", "deepseek-ai/DeepSeek-V3", "DeepseekV3ForCausalLM", 671.0, None, 1.0,
           args=["--enable-dp-attention", "--dp", "8"], quantization="fp8", multinode=2, min_tp=8, pd=True),
    Family("kimi-k2-instruct", "moonshotai", "moonshotai/Kimi-K2-Instruct", "DeepseekV3ForCausalLM", 1026.0, None,
           1.0, quantization="fp8", pd=True, multinode=2),
    Family("gpt-oss-20b", "openai", "openai/gpt-oss-20b", "GptOssForCausalLM", 20.9, "gpt-oss-20b", args=['--tool-call-parser', 'gpt-oss', '--reasoning-parser', 'gpt-oss'], grpc=True),
    Family("gpt-oss-120b", "openai", "openai/gpt-oss-120b", "GptOssForCausalLM", 117.0, args=['--tool-call-parser', 'gpt-oss', '--reasoning-parser', 'gpt-oss'], grpc=True),
    Family("gemma-2-9b-it", "google", "google/gemma-2-9b-it", "Gemma2ForCausalLM", 9.2, "gemma-2-9b"),
    Family("gemma-3-27b-it", "google", "google/gemma-3-27b-it", "Gemma3ForConditionalGeneration", 27.4,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("gemma-3-1b-it", "google", "google/gemma-3-1b-it", "Gemma3ForCausalLM", 1.0),
    Family("grok-1", "xai-org", "xai-org/grok-1", "Grok1ModelForCausalLM", 316.0, "grok-1"),
    Family("grok-2", "xai-org", "xai-org/grok-2", "Grok1ForCausalLM", 314.0, "grok-2"),
    Family("tele-flm", "cofeai", "CofeAI/Tele-FLM", "TeleFLMModel", 52.0, "tele-flm"),
    Family("phi-3-vision-128k-instruct", "microsoft", "microsoft/Phi-3-vision-128k-instruct", "Phi3VForCausalLM", 4.2,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("phi-3-mini-4k-instruct", "microsoft", "microsoft/Phi-3-mini-4k-instruct", "Phi3ForCausalLM", 3.8),
    Family("phi-3-small-8k-instruct", "microsoft", "microsoft/Phi-3-small-8k-instruct", "Phi3SmallForCausalLM", 7.4),
    Family("phi-3-5-moe-instruct", "microsoft", "microsoft/Phi-3.5-MoE-instruct", "PhiMoEForCausalLM", 41.9),
    Family("starcoder2-7b", "bigcode", "bigcode/starcoder2-7b", "Starcoder2ForCausalLM", 7.2, "starcoder2-7b"),
    Family("pythia-1-4b", "eleutherai", "EleutherAI/pythia-1.4b", "GPTNeoXForCausalLM", 1.4, "pythia-1.4b"),
    Family("phi-2", "microsoft", "microsoft/phi-2", "PhiForCausalLM", 2.8, "phi-2"),
    Family("internlm2-7b-chat", "internlm", "internlm/internlm2-chat-7b", "InternLM2ForCausalLM", 7.7),
    Family("granite-3-1-8b-instruct", "ibm-granite", "ibm-granite/granite-3.1-8b-instruct", "GraniteForCausalLM",
           8.2),
    Family("smollm3-3b", "huggingfacetb", "HuggingFaceTB/SmolLM3-3B", "SmolLM3ForCausalLM", 3.1),
    Family("nvidia-nemotron-nano-9b-v2", "nvidia", "nvidia/NVIDIA-Nemotron-Nano-9B-v2", "NemotronHForCausalLM", 8.9,
           args=['--reasoning-parser', 'nano_v3', '--tool-call-parser', 'nano_v3']),
    Family("nvidia-nemotron-3-nano-30b-a3b-bf16", "nvidia", "nvidia/NVIDIA-Nemotron-3-Nano-30B-A3B-BF16",
           "NemotronHForCausalLM", 31.6, "nemotron-3-nano-30b-a3b",
           args=['--reasoning-parser', 'nano_v3', '--tool-call-parser', 'qwen3_coder']),
    Family("nvidia-nemotron-nano-12b-v2-vl-bf16", "nvidia", "nvidia/NVIDIA-Nemotron-Nano-12B-v2-VL-BF16",
           "NemotronVLForConditionalGeneration", 12.6, capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("nemotron-h-8b-base", "nvidia", "nvidia/Nemotron-H-8B-Base-8K", "NemotronHForCausalLM", 8.1,
           "nemotron-h-8b"),
    Family("opt-125m", "facebook", "facebook/opt-125m", "OPTForCausalLM", 0.125, "opt-125m"),
    Family("falcon-7b-instruct", "tiiuae", "tiiuae/falcon-7b-instruct", "FalconForCausalLM", 7.2, "falcon-7b"),
    Family("gpt-j-6b", "eleutherai", "EleutherAI/gpt-j-6b", "GPTJForCausalLM", 6.1),
    Family("stablelm-2-12b-chat", "stabilityai", "stabilityai/stablelm-2-12b-chat", "StableLmForCausalLM", 12.1),
    Family("persimmon-8b-chat", "adept", "adept/persimmon-8b-chat", "PersimmonForCausalLM", 9.4),
    Family("c4ai-command-r-v01", "cohereforai", "CohereForAI/c4ai-command-r-v01", "CohereForCausalLM", 35.0),
    Family("glm-4-9b-chat", "zhipuai", "THUDM/glm-4-9b-chat-hf", "GlmForCausalLM", 9.4),
    Family("olmo-2-1124-7b-instruct", "allenai", "allenai/OLMo-2-1124-7B-Instruct", "Olmo2ForCausalLM", 7.3),
    Family("afm-4-5b-base", "arcee-ai", "arcee-ai/AFM-4.5B-Base", "ArceeForCausalLM", 4.6),
    Family("bloomz-7b1", "bigscience", "bigscience/bloomz-7b1", "BloomForCausalLM", 7.1),
    Family("mpt-7b", "mosaicml", "mosaicml/mpt-7b", "MPTForCausalLM", 6.7),
    Family("internlm2-7b-reward", "internlm", "internlm/internlm2-7b-reward", "InternLM2ForRewardModel", 7.7,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("qwen-7b-chat", "qwen", "Qwen/Qwen-7B-Chat", "QWenLMHeadModel", 7.7),
    Family("qwen-vl-chat", "qwen", "Qwen/Qwen-VL-Chat", "QWenLMHeadModel", 9.6,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"], runtime=True),
    Family("qwen-vl", "qwen", "Qwen/Qwen-VL", "QWenLMHeadModel", 9.6,
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("baichuan2-7b-chat", "baichuan-inc", "baichuan-inc/Baichuan2-7B-Chat", "BaichuanForCausalLM", 7.5),
    Family("baichuan2-13b-chat", "baichuan-inc", "baichuan-inc/Baichuan2-13B-Chat", "BaichuanForCausalLM", 13.9),
    Family("exaone-3-5-7-8b-instruct", "lgai-exaone", "LGAI-EXAONE/EXAONE-3.5-7.8B-Instruct", "ExaoneForCausalLM",
           7.8),
    Family("orion-14b-base", "orionstarai", "OrionStarAI/Orion-14B-Base", "OrionForCausalLM", 14.5),
    Family("minicpm-2b-sft-bf16", "openbmb", "openbmb/MiniCPM-2B-sft-bf16", "MiniCPMForCausalLM", 2.7),
    Family("chatglm2-6b", "thudm", "THUDM/chatglm2-6b", "ChatGLMModel", 6.2),
    Family("mimo-7b-rl", "xiaomimimo", "XiaomiMiMo/MiMo-7B-RL", "MiMoForCausalLM", 7.8),
    Family("olmoe-1b-7b-0924", "allenai", "allenai/OLMoE-1B-7B-0924", "OlmoeForCausalLM", 6.9),
    Family("granite-3-0-3b-a800m-instruct", "ibm-granite", "ibm-granite/granite-3.0-3b-a800m-instruct",
           "GraniteMoeForCausalLM", 3.3),
    Family("dbrx-instruct", "databricks", "databricks/dbrx-instruct", "DbrxForCausalLM", 132.0),
    Family("ernie-4-5-21b-a3b-pt", "baidu", "baidu/ERNIE-4.5-21B-A3B-PT", "Ernie4_5_MoeForCausalLM", 21.8),
    Family("minimax-m2", "minimax", "MiniMaxAI/MiniMax-M2", "MiniMaxM2ForCausalLM", 229.0, None, 1.0,
           quantization="fp8"),
    Family("qwen-image", "qwen", "Qwen/Qwen-Image", "QwenImagePipeline", 28.9, "qwen-image",
           capabilities=["TEXT_TO_IMAGE"], diffusion="QwenImagePipeline"),
    Family("qwen-image-edit", "qwen", "Qwen/Qwen-Image-Edit", "QwenImageEditPipeline", 28.9, "qwen-image",
           capabilities=["IMAGE_TEXT_TO_IMAGE"], diffusion="QwenImageEditPipeline"),
    Family("qwen-image-edit-plus", "qwen", "Qwen/Qwen-Image-Edit-2511", "QwenImageEditPlusPipeline", 28.9, "qwen-image",
           capabilities=["IMAGE_TEXT_TO_IMAGE"], diffusion="QwenImageEditPlusPipeline"),
    Family("bge-large-en-v1-5", "baai", "BAAI/bge-large-en-v1.5", "BertModel", 0.335,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("bge-m3", "baai", "BAAI/bge-m3", "XLMRobertaModel", 0.568,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("bge-reranker-v2-m3", "baai", "BAAI/bge-reranker-v2-m3", "XLMRobertaForSequenceClassification", 0.568,
           capabilities=["TEXT_RERANK"], args=["--is-embedding"]),
    Family("llama-3-3-nemotron-super-49b-v1", "nvidia", "nvidia/Llama-3_3-Nemotron-Super-49B-v1", "DeciLMForCausalLM",
           49.9),
    Family("llama-3-1-nemotron-ultra-253b-v1", "nvidia", "nvidia/Llama-3_1-Nemotron-Ultra-253B-v1", "DeciLMForCausalLM",
           253.0, None, 1.0, quantization="fp8"),
    Family("clip-vit-large-patch14-336", "openai", "openai/clip-vit-large-patch14-336", "CLIPModel", 0.428,
           capabilities=["TEXT_EMBEDDINGS", "EMBEDDING"], args=["--is-embedding"]),
    Family("e5-mistral-7b-instruct", "intfloat", "intfloat/e5-mistral-7b-instruct", "MistralModel", 7.1,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    # embedding / reward checkpoints of generative architectures (pooled or scored, --is-embedding)
    Family("qwen3-embedding-0-6b", "qwen", "Qwen/Qwen3-Embedding-0.6B", "Qwen3ForCausalLM", 0.6,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("qwen3-embedding-4b", "qwen", "Qwen/Qwen3-Embedding-4B", "Qwen3ForCausalLM", 4.0,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("qwen3-embedding-8b", "qwen", "Qwen/Qwen3-Embedding-8B", "Qwen3ForCausalLM", 7.6,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("gte-qwen2-7b-instruct", "alibaba-nlp", "Alibaba-NLP/gte-Qwen2-7B-instruct", "Qwen2ForCausalLM", 7.6,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("gme-qwen2-vl-2b-instruct", "alibaba-nlp", "Alibaba-NLP/gme-Qwen2-VL-2B-Instruct",
           "Qwen2VLForConditionalGeneration", 2.2, capabilities=["TEXT_EMBEDDINGS", "EMBEDDING"],
           args=["--is-embedding"]),
    Family("skywork-reward-llama-3-1-8b-v0-2", "skywork", "Skywork/Skywork-Reward-Llama-3.1-8B-v0.2",
           "LlamaForSequenceClassification", 7.5, capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("skywork-reward-gemma-2-27b-v0-2", "skywork", "Skywork/Skywork-Reward-Gemma-2-27B-v0.2",
           "Gemma2ForSequenceClassification", 27.2, capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("qwen2-5-math-rm-72b", "qwen", "Qwen/Qwen2.5-Math-RM-72B", "Qwen2ForRewardModel", 72.7,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    Family("qwen2-5-1-5b-apeach", "jason9693", "jason9693/Qwen2.5-1.5B-apeach", "Qwen2ForSequenceClassification", 1.5,
           capabilities=["TEXT_EMBEDDINGS"], args=["--is-embedding"]),
    # fp8 checkpoints of served architectures (dequantised per 128x128 block at load, fp8 GEMMs)
    Family("llama-3-3-70b-instruct-fp8-dynamic", "redhatai", "RedHatAI/Llama-3.3-70B-Instruct-FP8-dynamic",
           "LlamaForCausalLM", 70.6, None, 1.0, quantization="fp8"),
    Family("nvidia-nemotron-3-nano-30b-a3b-fp8", "nvidia", "nvidia/NVIDIA-Nemotron-3-Nano-30B-A3B-FP8",
           "NemotronHForCausalLM", 31.6, None, 1.0, quantization="fp8"),
    # compressed-tensors (RedHatAI FP8-dynamic) and NVIDIA ModelOpt FP8 vision-language checkpoints
    Family("llama-3-2-90b-vision-instruct-fp8", "meta", "RedHatAI/Llama-3.2-90B-Vision-Instruct-FP8-dynamic",
           "MllamaForConditionalGeneration", 88.6, None, 1.0, quantization="fp8",
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
    Family("nvidia-nemotron-nano-12b-v2-vl-fp8", "nvidia", "nvidia/NVIDIA-Nemotron-Nano-12B-v2-VL-FP8",
           "NemotronH_Nano_VL_V2", 12.6, None, 1.0, quantization="fp8",
           capabilities=["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"]),
]


# More checkpoints of supported architectures (the rest of the reference's model catalog,
# ``config/models/**``): base models whose runtime is an earlier family's when one of the same
# architecture / quantisation already covers the size, otherwise a runtime of their own.
_C, _I, _V = ["TEXT_TO_TEXT"], ["TEXT_TO_TEXT", "IMAGE_TEXT_TO_TEXT"], ["IMAGE_TO_TEXT"]
_L, _Q2, _Q3 = "LlamaForCausalLM", "Qwen2ForCausalLM", "Qwen3ForCausalLM"
_MORE = [
    ("deepseek-coder-7b-instruct-v1-5", "deepseek", "deepseek-ai/deepseek-coder-7b-instruct-v1.5", _L, 6.9),
    ("deepseek-llm-7b-chat", "deepseek", "deepseek-ai/deepseek-llm-7b-chat", _L, 6.9),
    ("deepseek-r1-distill-llama-8b", "deepseek", "deepseek-ai/DeepSeek-R1-Distill-Llama-8B", _L, 8.0),
    ("deepseek-r1-distill-llama-70b", "deepseek", "deepseek-ai/DeepSeek-R1-Distill-Llama-70B", _L, 70.6),
    ("deepseek-r1-distill-qwen-1-5b", "deepseek", "deepseek-ai/DeepSeek-R1-Distill-Qwen-1.5B", _Q2, 1.8),
    ("deepseek-r1-distill-qwen-7b", "deepseek", "deepseek-ai/DeepSeek-R1-Distill-Qwen-7B", _Q2, 7.6),
    ("deepseek-r1-distill-qwen-14b", "deepseek", "deepseek-ai/DeepSeek-R1-Distill-Qwen-14B", _Q2, 14.8),
    ("deepseek-r1-distill-qwen-32b", "deepseek", "deepseek-ai/DeepSeek-R1-Distill-Qwen-32B", _Q2, 32.8),
    ("deepseek-v2", "deepseek", "deepseek-ai/DeepSeek-V2", "DeepseekV2ForCausalLM", 236.0),
    ("deepseek-v2-5", "deepseek", "deepseek-ai/DeepSeek-V2.5", "DeepseekV2ForCausalLM", 236.0),
    ("dolly-v2-12b", "databricks", "databricks/dolly-v2-12b", "GPTNeoXForCausalLM", 12.0),
    ("stablelm-tuned-alpha-7b", "stabilityai", "stabilityai/stablelm-tuned-alpha-7b", "GPTNeoXForCausalLM", 7.9),
    ("falcon3-10b-instruct", "tiiuae", "tiiuae/Falcon3-10B-Instruct", _L, 10.3),
    ("gemma-2b", "google", "google/gemma-2b", "GemmaForCausalLM", 2.5),
    ("gemma-7b", "google", "google/gemma-7b", "GemmaForCausalLM", 8.5),
    ("gemma-2-2b", "google", "google/gemma-2-2b", "Gemma2ForCausalLM", 2.6),
    ("gemma-2-2b-it", "google", "google/gemma-2-2b-it", "Gemma2ForCausalLM", 2.6),
    ("gemma-2-9b", "google", "google/gemma-2-9b", "Gemma2ForCausalLM", 9.2),
    ("gemma-2-27b", "google", "google/gemma-2-27b", "Gemma2ForCausalLM", 27.2),
    ("gemma-2-27b-it", "google", "google/gemma-2-27b-it", "Gemma2ForCausalLM", 27.2),
    ("gemma-3-4b-it", "google", "google/gemma-3-4b-it", "Gemma3ForConditionalGeneration", 4.3, _I),
    ("gemma-3-12b-it", "google", "google/gemma-3-12b-it", "Gemma3ForConditionalGeneration", 12.2, _I),
    ("granite-3-0-2b-instruct", "ibm", "ibm-granite/granite-3.0-2b-instruct", "GraniteForCausalLM", 2.6),
    ("granite-3-1-2b-instruct", "ibm", "ibm-granite/granite-3.1-2b-instruct", "GraniteForCausalLM", 2.5),
    ("granite-3-0-8b-instruct", "ibm", "ibm-granite/granite-3.0-8b-instruct", "GraniteForCausalLM", 8.2),
    ("hermes-2-pro-llama-3-8b", "nousresearch", "NousResearch/Hermes-2-Pro-Llama-3-8B", _L, 8.0),
    ("internlm2-7b", "internlm", "internlm/internlm2-7b", "InternLM2ForCausalLM", 7.7),
    ("internlm2-20b", "internlm", "internlm/internlm2-20b", "InternLM2ForCausalLM", 19.9),
    ("llama-2-7b", "meta", "meta-llama/Llama-2-7b-hf", _L, 6.7),
    ("llama-2-7b-chat-hf", "meta", "meta-llama/Llama-2-7b-chat-hf", _L, 6.7),
    ("llama-2-13b-hf", "meta", "meta-llama/Llama-2-13b-hf", _L, 13.0),
    ("llama-2-13b-chat-hf", "meta", "meta-llama/Llama-2-13b-chat-hf", _L, 13.0),
    ("llama-2-70b-hf", "meta", "meta-llama/Llama-2-70b-hf", _L, 69.0),
    ("llama-2-70b-chat-hf", "meta", "meta-llama/Llama-2-70b-chat-hf", _L, 69.0),
    ("llama-3-1-70b-instruct", "meta", "meta-llama/Meta-Llama-3.1-70B-Instruct", _L, 70.6),
    ("llama-3-3-70b-instruct", "meta", "meta-llama/Llama-3.3-70B-Instruct", _L, 70.6),
    ("llama-3-1-nemotron-70b-instruct-hf", "nvidia", "nvidia/Llama-3.1-Nemotron-70B-Instruct-HF", _L, 70.6),
    ("llama-3-1-nemotron-nano-8b-v1", "nvidia", "nvidia/Llama-3.1-Nemotron-Nano-8B-v1", _L, 8.0),
    ("llama-3-2-1b-instruct", "meta", "meta-llama/Llama-3.2-1B-Instruct", _L, 1.2),
    ("llama-3-2-3b-instruct", "meta", "meta-llama/Llama-3.2-3B-Instruct", _L, 3.2),
    ("llama-guard-3-8b", "meta", "meta-llama/Llama-Guard-3-8B", _L, 8.0),
    ("llama-4-maverick-17b-128e-instruct", "meta", "meta-llama/Llama-4-Maverick-17B-128E-Instruct",
     "Llama4ForConditionalGeneration", 402.0, _I),
    ("unsloth-llama-3-2-11b-vision-instruct", "unsloth", "unsloth/Llama-3.2-11B-Vision-Instruct",
     "MllamaForConditionalGeneration", 10.7, _I),
    ("llava-v1-5-7b", "llava", "liuhaotian/llava-v1.5-7b", "LlavaLlamaForCausalLM", 7.1, _V),
    # LLaVA-1.6 / NeXT (anyres): same original layout, the model class follows the checkpoint config
    ("llava-v1-6-vicuna-7b", "liuhaotian", "liuhaotian/llava-v1.6-vicuna-7b", "LlavaLlamaForCausalLM", 7.1, _V),
    ("llava-v1-6-vicuna-13b", "liuhaotian", "liuhaotian/llava-v1.6-vicuna-13b", "LlavaLlamaForCausalLM", 13.4, _V),
    ("llava-next-8b", "lmms-lab", "lmms-lab/llava-next-8b", "LlavaLlamaForCausalLM", 8.4, _V),
    ("mistral-7b-instruct-v0-2", "mistralai", "mistralai/Mistral-7B-Instruct-v0.2", "MistralForCausalLM", 7.2),
    ("mistral-7b-instruct-v0-3", "mistral", "mistralai/Mistral-7B-Instruct-v0.3", "MistralForCausalLM", 7.2),
    ("mistral-7b-v0-1", "mistral", "mistralai/Mistral-7B-v0.1", "MistralForCausalLM", 7.2),
    ("mistral-nemo-instruct-2407", "mistral", "mistralai/Mistral-Nemo-Instruct-2407", "MistralForCausalLM", 12.2),
    ("mixtral-8x7b-instruct-v0-1", "mistral", "mistralai/Mixtral-8x7B-Instruct-v0.1", "MixtralForCausalLM", 46.7),
    ("mixtral-8x7b-v0-1", "mistral", "mistralai/Mixtral-8x7B-v0.1", "MixtralForCausalLM", 46.7),
    ("mixtral-8x22b-v0-1", "mistral", "mistralai/Mixtral-8x22B-v0.1", "MixtralForCausalLM", 141.0),
    ("nvidia-nemotron-3-nano-30b-a3b-base-bf16", "nvidia", "nvidia/NVIDIA-Nemotron-3-Nano-30B-A3B-Base-BF16",
     "NemotronHForCausalLM", 31.6),
    ("phi-1-5", "microsoft", "microsoft/phi-1_5", "PhiForCausalLM", 1.4),
    ("phi-3-mini-128k-instruct", "microsoft", "microsoft/Phi-3-mini-128k-instruct", "Phi3ForCausalLM", 3.8),
    ("phi-3-5-mini-instruct", "microsoft", "microsoft/Phi-3.5-mini-instruct", "Phi3ForCausalLM", 3.8),
    ("phi-4-mini-instruct", "microsoft", "microsoft/Phi-4-mini-instruct", "Phi3ForCausalLM", 3.8),
    ("phi-3-medium-4k-instruct", "microsoft", "microsoft/Phi-3-medium-4k-instruct", "Phi3ForCausalLM", 14.0),
    ("phi-4", "microsoft", "microsoft/phi-4", "Phi3ForCausalLM", 14.7),
    ("qwen1-5-7b-chat", "qwen", "Qwen/Qwen1.5-7B-Chat", _Q2, 7.7),
    ("qwen1-5-32b-chat", "qwen", "Qwen/Qwen1.5-32B-Chat", _Q2, 32.5),
    ("qwen1-5-72b-chat", "qwen", "Qwen/Qwen1.5-72B-Chat", _Q2, 72.3),
    ("qwen1-5-110b-chat", "qwen", "Qwen/Qwen1.5-110B-Chat", _Q2, 111.0),
    ("qwen2-7b-instruct", "qwen", "Qwen/Qwen2-7B-Instruct", _Q2, 7.6),
    ("qwen2-72b-instruct", "qwen", "Qwen/Qwen2-72B-Instruct", _Q2, 72.7),
    ("qwen2-5-0-5b", "qwen", "Qwen/Qwen2.5-0.5B", _Q2, 0.5),
    ("qwen2-5-1-5b", "qwen", "Qwen/Qwen2.5-1.5B", _Q2, 1.5),
    ("qwen2-5-3b", "qwen", "Qwen/Qwen2.5-3B", _Q2, 3.1),
    ("qwen2-5-3b-instruct", "qwen", "Qwen/Qwen2.5-3B-Instruct", _Q2, 3.1),
    ("qwen2-5-7b", "qwen", "Qwen/Qwen2.5-7B", _Q2, 7.6),
    ("qwen2-5-14b", "qwen", "Qwen/Qwen2.5-14B", _Q2, 14.8),
    ("qwen2-5-14b-instruct", "qwen", "Qwen/Qwen2.5-14B-Instruct", _Q2, 14.8),
    ("qwen2-5-32b", "qwen", "Qwen/Qwen2.5-32B", _Q2, 32.8),
    ("qwen2-5-32b-instruct", "qwen", "Qwen/Qwen2.5-32B-Instruct", _Q2, 32.8),
    ("qwen2-5-72b", "qwen", "Qwen/Qwen2.5-72B", _Q2, 72.7),
    ("qwen2-5-coder-7b-instruct", "qwen", "Qwen/Qwen2.5-Coder-7B-Instruct", _Q2, 7.6),
    ("qwen2-5-coder-32b-instruct", "qwen", "Qwen/Qwen2.5-Coder-32B-Instruct", _Q2, 32.8),
    ("skywork-or1-7b-preview", "skywork", "Skywork/Skywork-OR1-7B-Preview", _Q2, 7.6),
    ("qwen2-vl-2b-instruct", "qwen", "Qwen/Qwen2-VL-2B-Instruct", "Qwen2VLForConditionalGeneration", 2.2, _I),
    ("qwen2-vl-72b-instruct", "qwen", "Qwen/Qwen2-VL-72B-Instruct", "Qwen2VLForConditionalGeneration", 73.4, _I),
    ("qwen3-0-6b", "qwen", "Qwen/Qwen3-0.6B", _Q3, 0.75),
    ("qwen3-1-7b", "qwen", "Qwen/Qwen3-1.7B", _Q3, 2.0),
    ("qwen3-4b", "qwen", "Qwen/Qwen3-4B", _Q3, 4.0),
    ("qwen3-14b", "qwen", "Qwen/Qwen3-14B", _Q3, 14.8),
    ("qwen3-32b", "qwen", "Qwen/Qwen3-32B", _Q3, 32.8),
    ("smollm-135m", "huggingface", "HuggingFaceTB/SmolLM-135M", _L, 0.135),
    ("smollm-360m", "huggingface", "HuggingFaceTB/SmolLM-360M", _L, 0.36),
    ("smollm-1-7b", "huggingfacetb", "HuggingFaceTB/SmolLM-1.7B", _L, 1.7),
    ("smollm2-1-7b-instruct", "huggingfacetb", "HuggingFaceTB/SmolLM2-1.7B-Instruct", _L, 1.7),
    ("solar-10-7b-instruct-v1-0", "upstage", "upstage/SOLAR-10.7B-Instruct-v1.0", _L, 10.7),
    ("starcoder2-3b", "bigcode", "bigcode/starcoder2-3b", "Starcoder2ForCausalLM", 3.0),
    ("starcoder2-15b", "bigcode", "bigcode/starcoder2-15b", "Starcoder2ForCausalLM", 16.0),
    ("vicuna-7b-v1-5", "lmsys", "lmsys/vicuna-7b-v1.5", _L, 6.7),
    ("vicuna-13b-v1-5", "lmsys", "lmsys/vicuna-13b-v1.5", _L, 13.0),
    ("xgen-7b-8k-inst", "salesforce", "Salesforce/xgen-7b-8k-inst", _L, 6.7),
]
_FP8 = [   # the reference's DeepSeek-V3-architecture fp8 checkpoints, served like deepseek-v3
    ("deepseek-v3-0324", "deepseek-ai/DeepSeek-V3-0324"), ("deepseek-r1", "deepseek-ai/DeepSeek-R1"),
    ("deepseek-r1-zero", "deepseek-ai/DeepSeek-R1-Zero"),
]


_PD_MORE = {"llama-3-1-70b-instruct", "llama-3-3-70b-instruct", "llama-3-2-1b-instruct", "llama-3-2-3b-instruct"}


def _covers(g: Family, f: Family) -> bool:
    return (g.arch == f.arch and g.quantization == f.quantization and g.diffusion == f.diffusion
            and g.params_b * 0.85 <= f.params_b <= g.params_b * 1.15)


def _extend() -> None:
    for f in FAMILIES:   # the hand-picked families above all carry their own runtimes
        if f.runtime is None:
            f.runtime = True
    for row in _MORE:
        name, vendor, hf, arch, b = row[:5]
        FAMILIES.append(Family(name, vendor, hf, arch, b, capabilities=list(row[5]) if len(row) > 5 else list(_C)))
    for name, hf in _FP8:
        FAMILIES.append(Family(name, "deepseek-ai", hf, "DeepseekV3ForCausalLM", 671.0, None, 1.0,
                               args=["--enable-dp-attention", "--dp", "8"], quantization="fp8", min_tp=8))
    for f in FAMILIES:
        # every catalog model carries its own runtime, as in the reference catalog (look-alikes of
        # one size class are opt-in by name, see _lookalike); the reference's PD
        # runtimes exist for these too
        if f.runtime is None:
            f.runtime = True
        if f.name in _PD_MORE:
            f.pd = True


_extend()


def tp_for(f: Family) -> int:
    gb = f.params_b * f.bytes_per_param
    tp = f.min_tp
    while gb / tp > KV_HEADROOM * HBM_GB and tp < 8:
        tp *= 2
    return tp


def size_label(b: float) -> str:
    return f"{b:.0f}B" if b >= 10 else f"{b:.1f}B".replace(".0B", "B")


def _probes() -> dict:
    def get(path, **kw):
        return {"httpGet": {"path": path, "port": 8080}, **kw}

    return {"readinessProbe": get("/health_generate", failureThreshold=3, successThreshold=1, periodSeconds=30,
                                  timeoutSeconds=60),
            "livenessProbe": get("/health", failureThreshold=5, successThreshold=1, periodSeconds=30,
                                 timeoutSeconds=30),
            "startupProbe": get("/health_generate", failureThreshold=150, successThreshold=1, periodSeconds=6,
                                initialDelaySeconds=10, timeoutSeconds=30)}


def server_args(f: Family, tp: int, extra: list[str] | None = None) -> list[str]:
    if f.diffusion:
        return ["--host", "0.0.0.0", "--port", "8080", "--enable-metrics", "--model-path", "$(MODEL_PATH)",
                "--served-model-name", f.hf, "--pipeline", f.diffusion, "--tp-size", "1"]
    a = ["--host", "0.0.0.0", "--port", "8080", "--enable-metrics", "--model-path", "$(MODEL_PATH)",
         "--tp-size", str(tp), "--mem-frac", "0.9", "--served-model-name", f.hf]
    if f.quantization:
        a += ["--quantization", f.quantization]
    return a + list(f.args) + list(extra or [])


def _container(f: Family, tp: int, args: list[str], name: str = "ome-container") -> dict:
    cpu, mem = 16 * tp, f"{64 * tp}Gi"
    return {"name": name, "image": IMAGE, "ports": [{"containerPort": 8080, "name": "http1", "protocol": "TCP"}],
            "command": ["python3", "-m", "ome_amd.diffusion.server" if f.diffusion else "ome_amd.runtime.server"],
            "args": args,
            "env": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}, {"name": "GPU_MAX_HW_QUEUES", "value": "4"}],
            "volumeMounts": [{"mountPath": "/dev/shm", "name": "dshm"}],
            "resources": {"requests": {"cpu": cpu, "memory": mem, "amd.com/gpu": tp},
                          "limits": {"cpu": cpu, "memory": mem, "amd.com/gpu": tp}},
            **(_diffusion_probes() if f.diffusion else _probes())}


def _diffusion_probes() -> dict:
    def get(path, **kw):
        return {"httpGet": {"path": path, "port": 8080}, **kw}

    return {"readinessProbe": get("/health", failureThreshold=5, successThreshold=1, periodSeconds=60,
                                  timeoutSeconds=200),
            "livenessProbe": get("/health", failureThreshold=5, successThreshold=1, periodSeconds=60,
                                 timeoutSeconds=200),
            "startupProbe": get("/health", failureThreshold=150, successThreshold=1, periodSeconds=6,
                                initialDelaySeconds=10, timeoutSeconds=30)}


def _router() -> dict:
    return {"runner": {"name": "router", "image": "ome-amd/router:latest",
                       "ports": [{"containerPort": 8080, "name": "http"}],
                       "command": ["python3", "-m", "ome_amd.router", "--host", "0.0.0.0", "--port", "8080",
                                   "--policy", "cache_aware", "--service-discovery", "--selector",
                                   "component=engine", "ome.io/inferenceservice=$(INFERENCESERVICE_NAME)",
                                   "--service-discovery-namespace", "$(NAMESPACE)"],
                       "env": [{"name": "INFERENCESERVICE_NAME",
                                "valueFrom": {"fieldRef": {"fieldPath": "metadata.labels['ome.io/inferenceservice']"}}},
                               {"name": "NAMESPACE", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}}],
                       "resources": {"limits": {"cpu": "2", "memory": "2Gi"}}}}


def _formats(f: Family, priority: int = 2) -> list[dict]:
    if f.diffusion:
        return [{"modelFramework": {"name": "diffusers", "version": "0.34.0", "operator": "GreaterThanOrEqual"},
                 "modelFormat": {"name": "diffusers", "version": "0.34.0"}, "modelArchitecture": f.arch,
                 "autoSelect": True, "priority": priority, "version": "1.0.0"}]
    return [{"modelFramework": {"name": "transformers", "version": "5.0.0", "operator": "GreaterThanOrEqual"},
             "modelFormat": {"name": "safetensors", "version": "1.0.0"}, "modelArchitecture": f.arch,
             "autoSelect": True, "priority": priority, "version": "1.0.0",
             **({"quantization": f.quantization} if f.quantization else {})}]


def _lookalike(f: Family) -> int:
    """Position of ``f`` among the runtime families of its format / architecture / size range.
    Two auto-selecting runtimes of one such class would need distinct priorities (the
    ServingRuntime admission rule, ``servingruntime_webhook.go:202``), and the higher one would
    then win for every model of the class.  So the first family of a class auto-selects and its
    look-alikes (e.g. Llama-3.1 8B next to Llama-3 8B, Vicuna next to Llama-2 13B) are opt-in by
    runtime name -- every model still lands on a runtime of its own size class."""
    def key(g: Family):
        return (g.arch, g.quantization, size_label(g.params_b * 0.85), size_label(g.params_b * 1.15))

    k = key(f)
    same = [g.name for g in FAMILIES if g.runtime and key(g) == k and not _pooled_twin(g)]
    return same.index(f.name) if f.name in same else 0


def _pooled_twin(f: Family) -> bool:
    """An embedding / reward checkpoint of an architecture that also has generative runtimes:
    runtime selection does not look at capabilities, so its (pooling) runtime is opt-in by name
    and never captures the generative models of its size class."""
    return "--is-embedding" in f.args and any(g.arch == f.arch and "--is-embedding" not in g.args
                                              for g in FAMILIES if g.runtime)


def _spec_base(f: Family) -> dict:
    lo, hi = f.params_b * 0.85, f.params_b * 1.15
    fmts = _formats(f, 2)
    if _lookalike(f) or _pooled_twin(f):
        fmts[0]["autoSelect"] = False
    return {"disabled": False, "supportedModelFormats": fmts, "protocolVersions": ["openAI"],
            "modelSizeRange": {"min": size_label(lo), "max": size_label(hi)},
            "acceleratorRequirements": {"acceleratorClasses": ["amd-mi355x", "amd-mi300x"]}}


def runtime(f: Family) -> dict:
    tp = tp_for(f)
    spec = _spec_base(f)
    spec["engineConfig"] = {"annotations": {"prometheus.io/scrape": "true", "prometheus.io/port": "8080",
                                            "prometheus.io/path": "/metrics"},
                            "volumes": [{"name": "dshm", "emptyDir": {"medium": "Memory"}}],
                            "runner": _container(f, tp, server_args(f, tp))}
    if not f.diffusion:
        spec["routerConfig"] = _router()
    return {"apiVersion": "ome.io/v1beta1", "kind": "ClusterServingRuntime",
            "metadata": {"name": f"ome-amd-{f.name}-tp{tp}"}, "spec": spec}


def pd_runtime(f: Family) -> dict:
    """Prefill (engine) + decode (decoder) pods on one xGMI node; KV pages move GPU to GPU."""
    tp = tp_for(f)
    spec = _spec_base(f)
    spec["supportedModelFormats"][0]["priority"] = 1
    spec["supportedModelFormats"][0]["autoSelect"] = False  # opt-in via the ISVC's runtime name
    vol = [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]
    spec["engineConfig"] = {"volumes": vol, "runner": _container(
        f, tp, server_args(f, tp, ["--disaggregation-mode", "prefill", "--disaggregation-bootstrap-port", "8998"]))}
    spec["decoderConfig"] = {"volumes": vol, "runner": _container(f, tp, server_args(f, tp, ["--disaggregation-mode",
                                                                                             "decode"]))}
    r = _router()
    r["runner"]["command"] += ["--pd-disaggregation"]
    spec["routerConfig"] = r
    return {"apiVersion": "ome.io/v1beta1", "kind": "ClusterServingRuntime",
            "metadata": {"name": f"ome-amd-{f.name}-pd-tp{tp}"}, "spec": spec}


GRPC_SERVICE = "sglang.grpc.scheduler.SglangScheduler"


def _grpc_container(f: Family, tp: int, args: list[str]) -> dict:
    """The engine container of a gRPC-mode runtime (reference ``srt/gpt-oss-120b-rt.yaml:61-130``):
    port ``grpc1``; grpc.health.v1 probes -- service "" for liveness / startup, the scheduler
    service for readiness (runtime/grpc_server.py)."""
    c = _container(f, tp, args + ["--grpc-mode"])
    c["ports"] = [{"containerPort": 8080, "name": "grpc1", "protocol": "TCP"}]

    def g(service, **kw):
        return {"grpc": {"port": 8080, "service": service}, **kw}

    c["livenessProbe"] = g("", failureThreshold=5, successThreshold=1, periodSeconds=60, timeoutSeconds=60)
    c["readinessProbe"] = g(GRPC_SERVICE, initialDelaySeconds=60, failureThreshold=3, successThreshold=1,
                            periodSeconds=60, timeoutSeconds=200)
    c["startupProbe"] = g("", failureThreshold=150, successThreshold=1, periodSeconds=6, initialDelaySeconds=60,
                          timeoutSeconds=30)
    return c


def _grpc_router(pd: bool = False) -> dict:
    r = _router()
    r["runner"]["command"] += ["--health-check-endpoint", "/HealthCheck"] + (["--pd-disaggregation"] if pd else [])
    return r


def grpc_runtime(f: Family) -> dict:
    """Engine behind gRPC (``--grpc-mode``), reached by the router over gRPC (opt-in by name)."""
    tp = tp_for(f)
    spec = _spec_base(f)
    spec["supportedModelFormats"][0]["autoSelect"] = False
    spec["engineConfig"] = {"volumes": [{"name": "dshm", "emptyDir": {"medium": "Memory"}}],
                            "runner": _grpc_container(f, tp, server_args(f, tp))}
    spec["routerConfig"] = _grpc_router()
    return {"apiVersion": "ome.io/v1beta1", "kind": "ClusterServingRuntime",
            "metadata": {"name": f"ome-amd-{f.name}-grpc-tp{tp}"}, "spec": spec}


def pd_grpc_runtime(f: Family) -> dict:
    """PD disaggregation with both roles behind gRPC (reference ``...-fp8-pd-grpc-rt.yaml``)."""
    tp = tp_for(f)
    spec = _spec_base(f)
    spec["supportedModelFormats"][0]["priority"] = 1
    spec["supportedModelFormats"][0]["autoSelect"] = False
    vol = [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]
    spec["engineConfig"] = {"volumes": vol, "runner": _grpc_container(
        f, tp, server_args(f, tp, ["--disaggregation-mode", "prefill", "--disaggregation-bootstrap-port", "8998"]))}
    spec["decoderConfig"] = {"volumes": vol, "runner": _grpc_container(
        f, tp, server_args(f, tp, ["--disaggregation-mode", "decode"]))}
    spec["routerConfig"] = _grpc_router(pd=True)
    return {"apiVersion": "ome.io/v1beta1", "kind": "ClusterServingRuntime",
            "metadata": {"name": f"ome-amd-{f.name}-pd-grpc-tp{tp}"}, "spec": spec}


def multinode_runtime(f: Family) -> dict:
    """Leader/worker (LeaderWorkerSet) serving over ``f.multinode`` nodes of 8 GPUs (TP across the
    nodes, the checkpoint's own precision: the family's model must admit to it)."""
    g = copy.copy(f)
    g.args = []
    n = f.multinode
    tp = 8 * n
    spec = _spec_base(g)
    spec["supportedModelFormats"][0]["autoSelect"] = False
    vol = [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]
    dist = ["--dist-init-addr", "$(LWS_LEADER_ADDRESS):5000", "--nnodes", str(n)]
    leader = _container(g, 8, server_args(g, tp, dist + ["--node-rank", "0"]))
    worker = _container(g, 8, server_args(g, tp, dist + ["--node-rank", "$(LWS_WORKER_INDEX)"]))
    for c in (leader, worker):
        c["resources"] = {"requests": {"cpu": 128, "memory": "1024Gi", "amd.com/gpu": 8},
                          "limits": {"cpu": 128, "memory": "1024Gi", "amd.com/gpu": 8}}
    spec["engineConfig"] = {"volumes": vol, "leader": {"runner": leader}, "worker": {"size": n - 1, "runner": worker}}
    spec["routerConfig"] = _router()
    return {"apiVersion": "ome.io/v1beta1", "kind": "ClusterServingRuntime",
            "metadata": {"name": f"ome-amd-{f.name}-{n}node"}, "spec": spec}


def base_model(f: Family) -> dict:
    uri = f"random://{f.preset}" if f.preset else f"hf://{f.hf}"
    spec = {"vendor": f.vendor, "disabled": False, "version": "1.0.0", "displayName": f"{f.vendor}.{f.name}",
            "modelCapabilities": list(f.capabilities), "modelArchitecture": f.arch,
            "modelParameterSize": size_label(f.params_b),
            "modelFormat": {"name": "diffusers", "version": "0.34.0"} if f.diffusion else
            {"name": "safetensors", "version": "1.0.0"},
            "modelFramework": {"name": "diffusers", "version": "0.34.0"} if f.diffusion else
            {"name": "transformers", "version": "4.46.0"},
            "storage": {"storageUri": uri, "path": f"/raid/models/{f.vendor}/{f.name}"}}
    if f.quantization:
        spec["quantization"] = f.quantization
    if not f.preset:
        spec["storage"]["key"] = "hf-token"
    return {"apiVersion": "ome.io/v1beta1", "kind": "ClusterBaseModel", "metadata": {"name": f.name}, "spec": spec}


def isvc_samples(f: Family) -> dict[str, dict]:
    """InferenceService samples for a family (``config/samples/isvc/<vendor>/*.yaml``): the
    default runtime, plus the PD-disaggregated and multi-node runtimes where the family has them."""
    def isvc(name: str, rt: dict, extra: dict | None = None) -> dict:
        spec = {"model": {"name": f.name}, "runtime": {"name": rt["metadata"]["name"]},
                "engine": {"minReplicas": 1, "maxReplicas": 1}}
        if "TEXT_TO_TEXT" in f.capabilities or "IMAGE_TEXT_TO_TEXT" in f.capabilities:
            spec["router"] = {"minReplicas": 1, "maxReplicas": 1}
        spec.update(extra or {})
        return {"apiVersion": "ome.io/v1beta1", "kind": "InferenceService",
                "metadata": {"name": name, "namespace": name}, "spec": spec}

    out = {f.name: isvc(f.name, runtime(f))}
    if f.pd:
        out[f"{f.name}-pd"] = isvc(f"{f.name}-pd", pd_runtime(f),
                                   {"decoder": {"minReplicas": 1, "maxReplicas": 1},
                                    "router": {"minReplicas": 1, "maxReplicas": 1}})
    if f.multinode:
        out[f"{f.name}-{f.multinode}node"] = isvc(f"{f.name}-{f.multinode}node", multinode_runtime(f))
    return out


SCENARIOS = ["N(480,240)/(300,150)", "D(100,100)", "D(100,1000)", "D(2000,200)", "D(7800,200)"]
CONCURRENCY = [1, 2, 4, 8, 16, 32, 64, 128, 256]


def benchmark_samples() -> dict[str, list[dict]]:
    """BenchmarkJob samples: the protocol sweep on a text model, an embeddings run, the PD
    DeepSeek deployment and the Hugging Face secret the tokenizer download uses."""
    def job(name, isvc, task, scenarios, conc, ns, extra=None):
        spec = {"huggingFaceSecretReference": {"name": "huggingface-secret"},
                "endpoint": {"inferenceService": {"name": isvc, "namespace": isvc}}, "task": task,
                "trafficScenarios": scenarios, "numConcurrency": conc, "maxTimePerIteration": 15,
                "maxRequestsPerIteration": 100, "additionalRequestParams": {"temperature": "0.0"},
                "outputLocation": {"storageUri": f"oci://n/ome-ns/b/ome-benchmark-results/o/{name}",
                                   "parameters": {"auth": "instance_principal"}}}
        spec.update(extra or {})
        return {"apiVersion": "ome.io/v1beta1", "kind": "BenchmarkJob", "metadata": {"name": name, "namespace": ns},
                "spec": spec}

    secret = {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "huggingface-secret", "namespace": "default"},
              "type": "Opaque", "data": {"HUGGINGFACE_API_KEY": "cmVwbGFjZS1tZQ=="}}
    return {
        "llama3-8b-instruct": [job("llama-3-8b-benchmark", "llama-3-8b-instruct", "text-to-text", SCENARIOS,
                                   CONCURRENCY, "llama-3-8b-instruct")],
        "llama3-70b-instruct-pd": [job("llama-3-70b-pd-benchmark", "llama-3-70b-instruct-pd", "text-to-text",
                                       SCENARIOS, CONCURRENCY, "llama-3-70b-instruct-pd")],
        "e5-mistral-7b-instruct": [job("e5-mistral-7b-benchmark", "e5-mistral-7b-instruct", "text-to-embeddings",
                                       ["E(64)", "E(512)", "E(1024)"], [1, 8, 32, 128], "e5-mistral-7b-instruct")],
        "deepseek-v3": [job("deepseek-v3-benchmark", "deepseek-v3", "text-to-text", SCENARIOS[:3],
                            [1, 16, 64, 256], "deepseek-v3", {"maxTimePerIteration": 30})],
        "huggingface-secret": [secret],
    }


def generate() -> tuple[dict[str, list[dict]], dict[str, list[dict]]]:
    """-> ({runtime file stem: docs}, {vendor: base model docs})."""
    rts: dict[str, list[dict]] = {}
    models: dict[str, list[dict]] = {}
    for f in FAMILIES:
        models.setdefault(f.vendor, []).append(base_model(f))
        if not f.runtime:   # served by an earlier family's runtime (same architecture and size class)
            continue
        docs = [runtime(f)]
        if f.pd:
            docs.append(pd_runtime(f))
        if f.multinode:
            docs.append(multinode_runtime(f))
        if f.grpc:
            docs.append(grpc_runtime(f))
            if f.pd:
                docs.append(pd_grpc_runtime(f))
        rts[f.name] = docs
    return rts, models


def write(out: Path) -> list[Path]:
    rts, models = generate()
    paths = []
    hdr = "# Generated by `python -m ome_amd.catalog --out config` -- edit ome_amd/catalog.py, not this file.\n"
    for stem, docs in rts.items():
        p = out / "runtimes" / "ome-amd" / f"{stem}-rt.yaml"
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(hdr + yaml.safe_dump_all(docs, sort_keys=False))
        paths.append(p)
    for vendor, docs in models.items():
        p = out / "models" / vendor / "catalog.yaml"
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(hdr + yaml.safe_dump_all(docs, sort_keys=False))
        paths.append(p)
    for f in FAMILIES:
        if not f.runtime:
            continue
        for stem, doc in isvc_samples(f).items():
            p = out / "samples" / "isvc" / f.vendor / f"{stem}.yaml"
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_text(hdr + yaml.safe_dump(doc, sort_keys=False))
            paths.append(p)
    for stem, docs in benchmark_samples().items():
        p = out / "samples" / "benchmark" / f"{stem}.yaml"
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(hdr + yaml.safe_dump_all(docs, sort_keys=False))
        paths.append(p)
    return paths


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--out", default="config")
    a = ap.parse_args(argv)
    for p in write(Path(a.out)):
        print(p)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

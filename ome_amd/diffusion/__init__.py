"""Diffusion serving (text-to-image / image editing): the Qwen-Image pipelines on the ome_amd
kernels -- MMDiT (``qwen_image_dit``), VAE (``vae``), flow-matching sampler (``scheduler``),
pipelines (``pipeline``) and the OpenAI-images HTTP server (``server``)."""
from ome_amd.diffusion.pipeline import PIPELINES, QwenImagePipeline  # noqa: F401

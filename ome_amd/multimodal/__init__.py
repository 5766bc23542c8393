"""Multimodal inputs for the first-party runtime: image loading / preprocessing, prompt expansion
(image placeholder tokens -> one token per merged vision patch), M-RoPE positions.

Reference: the vision-language runtimes of the catalog (``config/runtimes/srt/qwen/qwen2-vl-*``,
``MllamaForConditionalGeneration`` / ``Llama4ForConditionalGeneration`` runtimes) served through
SGLang's OpenAI-compatible ``image_url`` chat content; this package is the MI355X runtime's own
implementation of that input path.
"""
from ome_amd.multimodal.inputs import MMInput, expand_image_tokens, mrope_positions  # noqa: F401

"""FP8 checkpoint formats of the reference catalog beyond DeepSeek block scales:

* compressed-tensors ``float-quantized`` (RedHatAI ``*-FP8-dynamic``: per-channel ``weight_scale``),
  here on Llama 3.2 Vision (``config/models/meta/Llama-3.2-90B-Vision-Instruct-FP8.yaml``);
* NVIDIA ModelOpt ``quant_algo: FP8`` (per-tensor ``weight_scale`` + ``input_scale``), here on
  NemotronH (``config/models/nvidia/NVIDIA-Nemotron-Nano-12B-v2-VL-FP8.yaml``'s language model).

A tiny random HF model is quantised into each format on disk; the loaded model must match HF run on
the same DEQUANTISED weights (Mllama: W8A8 projections -> cosine check; NemotronH: dequantised to
bf16/fp32 -> logits match)."""
import json

import pytest
import torch
import torch.nn.functional as F

transformers = pytest.importorskip("transformers")

from safetensors.torch import load_file  # noqa: E402

from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models.config import _is_fp8_checkpoint  # noqa: E402
from ome_amd.models.quant import Fp8Weight  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402

FP8_MAX = 448.0


def test_fp8_config_detection():
    ct = {"quant_method": "compressed-tensors", "format": "float-quantized",
          "config_groups": {"group_0": {"targets": ["Linear"], "weights": {"num_bits": 8, "type": "float",
                                                                           "strategy": "channel"},
                                        "input_activations": {"num_bits": 8, "type": "float", "dynamic": True}}}}
    assert _is_fp8_checkpoint(ct)
    assert not _is_fp8_checkpoint({**ct, "config_groups": {"g": {"weights": {"num_bits": 4, "type": "int"}}}})
    assert _is_fp8_checkpoint({"quant_method": "modelopt", "quant_algo": "FP8"})
    assert not _is_fp8_checkpoint({"quant_method": "modelopt", "quant_algo": "NVFP4"})
    assert _is_fp8_checkpoint({"quant_method": "fp8", "weight_block_size": [128, 128]})
    assert not _is_fp8_checkpoint({"quant_method": "awq"})


def _quantize_dir(path, keep, per_channel: bool, cfg_patch: dict):
    """Rewrite path/model.safetensors: every 2-D weight for which ``keep(name)`` is False becomes
    e4m3 + ``weight_scale`` ([N, 1] per channel, or a scalar + ``input_scale``); returns the
    dequantised state dict (what HF must run to be comparable)."""
    sd = {k: v.clone() for k, v in load_file(path / "model.safetensors").items()}   # not backed by the file we rewrite
    out, deq = {}, {}
    for n, w in sd.items():
        if n.endswith(".weight") and w.dim() == 2 and not keep(n):
            wf = w.float()
            s = (wf.abs().amax(1, keepdim=True) if per_channel else wf.abs().amax()).clamp_min(1e-8) / FP8_MAX
            q = (wf / s).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
            out[n] = q
            out[n[:-len("weight")] + "weight_scale"] = s.reshape(-1, 1) if per_channel else s.reshape(())
            if not per_channel:
                out[n[:-len("weight")] + "input_scale"] = torch.tensor(1.0)
            deq[n] = (q.float() * s).to(w.dtype)
        else:
            out[n] = w
            deq[n] = w
    save_file({k: v.contiguous() for k, v in out.items()}, path / "model.safetensors")
    cfg = json.loads((path / "config.json").read_text())
    cfg.update(cfg_patch)
    (path / "config.json").write_text(json.dumps(cfg))
    return deq


def test_compressed_tensors_mllama(tmp_path):
    from tests.test_mllama_cpu import CASES, _prefill_logits
    from tests.test_mllama_cpu import _hf as mllama_hf

    hf = mllama_hf(tmp_path)
    ct = {"quantization_config": {
        "quant_method": "compressed-tensors", "format": "float-quantized", "ignore": ["lm_head", "re:.*vision.*"],
        "config_groups": {"group_0": {"targets": ["Linear"],
                                      "weights": {"num_bits": 8, "type": "float", "strategy": "channel"},
                                      "input_activations": {"num_bits": 8, "type": "float", "dynamic": True,
                                                            "strategy": "token"}}}}}
    deq = _quantize_dir(tmp_path, lambda n: "vision" in n or "embed" in n or "lm_head" in n or
                        "multi_modal_projector" in n, True, ct)
    # checkpoint names (legacy layout) -> this transformers version's module names
    hf_names = set(hf.state_dict())

    def hf_name(k):
        for a, b in (("language_model.model.", "model.language_model."), ("language_model.lm_head.", "lm_head."),
                     ("vision_model.", "model.vision_model."),
                     ("multi_modal_projector.", "model.multi_modal_projector.")):
            if k.startswith(a) and b + k[len(a):] in hf_names:
                return b + k[len(a):]
        return k

    res = hf.load_state_dict({hf_name(k): v for k, v in deq.items()}, strict=False)
    assert not [k for k in res.missing_keys if "language_model" in k], res.missing_keys[:4]
    ids, _ = CASES["text"]
    with torch.no_grad():
        want = hf(input_ids=torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=256))
    m = eng.runner.model
    assert m.fp8 and type(m).__name__ == "MllamaForConditionalGeneration"
    assert any(isinstance(m.w_gu[i], Fp8Weight) for i in m.layers)
    got = _prefill_logits(eng, ids, None)
    assert F.cosine_similarity(got, want, dim=-1).min().item() > 0.99


def test_modelopt_fp8_nemotron_h(tmp_path):
    from tests.test_nemotron_h_cpu import _hf_model, _prefill_logits

    hf = _hf_model(tmp_path)
    deq = _quantize_dir(tmp_path, lambda n: "embed" in n or "lm_head" in n or "norm" in n or "conv1d" in n, False,
                        {"quantization_config": {"quant_method": "modelopt", "quant_algo": "FP8"}})
    # the checkpoint keeps the remote-code names (backbone.*, embedding); HF's module names differ
    ren = {k.replace("backbone.", "model.").replace("model.embedding.", "model.embeddings."): v for k, v in deq.items()}
    res = hf.load_state_dict(ren, strict=False)
    assert not res.missing_keys, res.missing_keys[:4]
    ids = [(7 * i + 3) % 500 + 3 for i in range(24)]
    with torch.no_grad():
        want = hf(torch.tensor([ids])).logits[0].float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=256))
    assert eng.runner.model.fp8
    got = _prefill_logits(eng, ids, [24])
    assert (got - want).abs().max().item() < 2e-3 * max(1.0, want.abs().max().item())

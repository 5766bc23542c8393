"""Rank-aware loading straight into HBM (libomeio omeio_load_ranges / omeio_load_strided): a TP
rank's shards loaded on the GPU equal the CPU shards, byte for byte."""
import json

import pytest
import torch

from ome_amd.io import native as nio
from ome_amd.models import build_model
from ome_amd.models.config import PRESETS, ModelConfig
from ome_amd.parallel import state as pstate
from tests.test_sharded_load_cpu import _hf_checkpoint

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tp,rank", [(2, 1), (4, 2)])
def test_gpu_shards_match_cpu(tmp_path, tp, rank):
    hf = dict(PRESETS["tiny-llama"])
    hf.update(num_key_value_heads=4, num_attention_heads=4)
    cfg = ModelConfig.from_hf(hf)
    (tmp_path / "config.json").write_text(json.dumps(hf))
    _hf_checkpoint(tmp_path, cfg, seed=7)
    prev = pstate.get()
    pstate.set_state(pstate.ParallelState(tp_size=tp, tp_rank=rank, world_size=tp, rank=rank))
    try:
        cpu = build_model(cfg, "cpu", torch.bfloat16, model_path=str(tmp_path), load_format="safetensors")
        b0 = nio.bytes_read()
        gpu = build_model(cfg, "cuda", torch.bfloat16, model_path=str(tmp_path), load_format="safetensors")
        torch.cuda.synchronize()
        nbytes = nio.bytes_read() - b0
    finally:
        pstate.set_state(prev)
    assert gpu._presliced
    for i in range(cfg.num_layers):
        for a, b in ((cpu.w_qkv[i], gpu.w_qkv[i]), (cpu.w_o[i], gpu.w_o[i]), (cpu.w_gu[i], gpu.gate_up_weight(i)),
                     (cpu.w_d[i], gpu.w_d[i])):
            assert torch.equal(a, b.cpu())
    assert torch.equal(cpu.embed, gpu.embed.cpu()) and torch.equal(cpu.lm_head, gpu.lm_head.cpu())
    full = (tmp_path / "model.safetensors").stat().st_size
    assert nbytes < full / tp * 1.1

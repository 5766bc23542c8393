"""Qwen2-VL class model on gfx950: vision tower (ome_layernorm HIP kernel + hipBLASLt GEMMs) vs an
fp32 CPU copy of the same weights, and an image request served with HIP-graph decode (M-RoPE
``rope_delta`` on the decode rows) agreeing with the eager (row-indexed M-RoPE table) path."""
import numpy as np
import pytest
import torch

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams

pytestmark = pytest.mark.gpu


def _img():
    from PIL import Image

    return Image.fromarray(np.random.default_rng(1).integers(0, 255, (112, 140, 3), dtype=np.uint8))


def test_qwen2_vl_vision_tower_matches_fp32():
    from ome_amd.multimodal.inputs import preprocess_image
    from ome_amd.models.qwen2_vl import Qwen2VisionTower
    from ome_amd.models.config import PRESETS

    vc = PRESETS["tiny-qwen2-vl"]["vision_config"]
    g = Qwen2VisionTower(vc, 256, torch.device("cuda"), torch.bfloat16)
    g.init_random(torch.Generator(device="cuda").manual_seed(0), std=0.05)
    c = Qwen2VisionTower(vc, 256, torch.device("cpu"), torch.float32)
    c.w = {k: v.float().cpu() for k, v in g.w.items()}
    pv, grid = preprocess_image(_img())
    pv = torch.from_numpy(pv)
    got = g.forward(pv, [grid]).float().cpu()
    want = c.forward(pv, [grid])
    assert got.shape == want.shape == (grid[1] * grid[2] // 4, 256)
    err = (got - want).abs().max().item()
    assert err < 3e-2 * max(1.0, want.abs().max().item()), err


def test_qwen2_vl_image_request_graph_vs_eager():
    outs = []
    for graph in (True, False):
        eng = Engine(EngineArgs(model="tiny-qwen2-vl", device="cuda", max_running_requests=8, context_length=512,
                                cuda_graph=graph))
        m = eng.runner.model
        assert eng.runner.use_graph == graph
        prompt = [5, 9, 17, m.vision_start_id, m.image_token_id, m.vision_end_id, 33, 41, 12, 7]
        reqs = [eng.make_mm_request(prompt, [_img()], SamplingParams(max_new_tokens=16, ignore_eos=True)),
                eng.make_request([11 + j for j in range(40)], SamplingParams(max_new_tokens=16, ignore_eos=True))]
        for r in reqs:
            eng.add_request(r)
        while not all(r.finished for r in reqs):
            eng.step()
        assert reqs[0].mm.rope_delta != 0
        outs.append([r.output_ids for r in reqs])
        del eng
        torch.cuda.empty_cache()
    for a, b in zip(*outs):
        assert sum(int(x == y) for x, y in zip(a, b)) >= 14, (a, b)

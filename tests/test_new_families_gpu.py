"""Round-4 model families on MI355X (bf16, HIP kernels) against their CPU fp32 runs: Grok-1/2 and
Tele-FLM engines with HIP-graph decode, the VLM image encoders (Phi-3-V, MiniCPM-V, Nemotron VL,
DeepSeek-VL2, dots.ocr) on checkpoints built by their CPU tests, and the Qwen-Image MMDiT / VAE /
pipeline."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).abs().max() / (b.float().abs().max() + 1e-6)).item()


@pytest.mark.parametrize("preset", ["tiny-grok1", "tiny-grok2", "tiny-teleflm"])
def test_engine_graphs_match_eager(preset):
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    g = Engine(EngineArgs(model=preset, device="cuda", max_running_requests=8, context_length=512))
    e = Engine(EngineArgs(model=preset, device="cuda", max_running_requests=8, context_length=512,
                          cuda_graph=False, overlap_schedule=False))
    prompts = [[3 + (i * 37 + j) % 900 for j in range(9 + 5 * i)] for i in range(5)]
    sp = SamplingParams(max_new_tokens=12, ignore_eos=True)
    a = [r.output_ids for r in g.generate(prompts, sp)]
    b = [r.output_ids for r in e.generate(prompts, sp)]
    assert sum(x == y for x, y in zip(a, b)) >= 4, (a, b)


def _engine_pair(path):
    from ome_amd.runtime.engine import Engine, EngineArgs

    cpu = Engine(EngineArgs(model_path=str(path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=512))
    gpu = Engine(EngineArgs(model_path=str(path), device="cuda", dtype="bfloat16", max_running_requests=2,
                            context_length=512, cuda_graph=False))
    return cpu.runner.model, gpu.runner.model


def _image(h, w, seed=0):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def test_phi3v_features(tmp_path):
    import test_phi3v_cpu as t
    from ome_amd.models.phi3v import preprocess_phi3v

    t._build(tmp_path)
    c, g = _engine_pair(tmp_path)
    px, grid = preprocess_phi3v(_image(80, 60), 4, t.CROP)
    assert _rel(g.encode_images(px, [grid]), c.encode_images(px, [grid])) < 3e-2


def test_minicpmv_features(tmp_path):
    import test_minicpmv_cpu as t
    from ome_amd.models.minicpmv import preprocess_minicpmv

    t._build(tmp_path)
    c, g = _engine_pair(tmp_path)
    rows, grids, _ = preprocess_minicpmv(_image(60, 100), 4, t.SCALE, t.PS)
    grids = [(1, h, w) for h, w in grids]
    assert _rel(g.encode_images(rows, grids), c.encode_images(rows, grids)) < 3e-2


def test_nemotron_vl_features(tmp_path):
    import test_nemotron_vl_cpu as t
    from ome_amd.models.internvl import preprocess_internvl

    t._build(tmp_path, "NemotronH_Nano_VL_V2")
    c, g = _engine_pair(tmp_path)
    px = preprocess_internvl(_image(70, 130), t.SIZE, 4, True, t.MEAN, t.STD)
    assert _rel(g.encode_images(px), c.encode_images(px)) < 3e-2


def test_deepseek_vl2_features(tmp_path):
    import test_deepseek_vl2_cpu as t
    from ome_amd.models.deepseek_vl2 import preprocess_deepseek_vl2

    t._build(tmp_path)
    c, g = _engine_pair(tmp_path)
    px, grid = preprocess_deepseek_vl2(_image(40, 100, 1), t.SIZE, True, t.CANDS)
    assert _rel(g.encode_images(px, [grid]), c.encode_images(px, [grid])) < 3e-2


def test_qwen_image_dit_vae_on_gpu():
    from ome_amd.diffusion.qwen_image_dit import QwenImageDiT
    from ome_amd.diffusion.vae import QwenImageVAE

    cfg = dict(num_layers=2, num_attention_heads=2, attention_head_dim=128, joint_attention_dim=256, in_channels=64,
               out_channels=16, patch_size=2, axes_dims_rope=[16, 56, 56])
    cpu = QwenImageDiT(cfg, "cpu", torch.float32).init_random(2, std=0.05)
    gpu = QwenImageDiT(cfg, "cuda", torch.bfloat16)
    gpu.w = {k: v.to("cuda", torch.bfloat16) for k, v in cpu.w.items()}
    shapes = [(1, 16, 16)]
    g = torch.Generator().manual_seed(0)
    img = torch.randn(1, 256, 64, generator=g).expand(2, 256, 64).contiguous()
    txts = [torch.randn(40, 256, generator=g), torch.randn(9, 256, generator=g)]
    t = torch.tensor([0.5, 0.5])
    want = cpu.forward(img, txts, t, shapes)
    got = gpu.forward(img.cuda(), [x.cuda() for x in txts], t.cuda(), shapes)
    assert _rel(got, want) < 4e-2
    vc = dict(base_dim=32, z_dim=16, dim_mult=[1, 2, 4, 4], num_res_blocks=2)
    v0 = QwenImageVAE(vc, "cpu", torch.float32).init_random(1)
    v1 = QwenImageVAE(vc, "cuda", torch.bfloat16)
    v1.w = {k: v.to("cuda", torch.bfloat16) for k, v in v0.w.items()}
    z = torch.randn(1, 16, 16, 16, generator=g)
    got, want = v1.decode(z.cuda()).float().cpu(), v0.decode(z)
    assert (got - want).abs().mean().item() < 1e-2 and _rel(got, want) < 1e-1   # bf16 through ~30 convolutions


def test_qwen_image_pipeline_on_gpu():
    from ome_amd.diffusion.pipeline import QwenImagePipeline

    p = QwenImagePipeline.random("tiny-qwen-image", "t2i", device="cuda", dtype=torch.bfloat16)
    a = p("a lighthouse at dusk", negative_prompt=" ", width=128, height=96, steps=4, seed=1)
    b = p("a lighthouse at dusk", negative_prompt=" ", width=128, height=96, steps=4, seed=1)
    assert a.shape == (96, 128, 3) and np.array_equal(a, b)

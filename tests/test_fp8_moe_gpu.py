"""FP8 block-scaled grouped MoE GEMM (csrc/kernels/moe.hip ome_moe_gemm_fp8) through
ops.fused_moe with Fp8Experts, against the fp32 emulation of the same quantisation
(ops.reference.fused_moe_fp8) and against the bf16 MoE within fp8 tolerance."""
import pytest
import torch

from ome_amd import ops
from ome_amd.models.quant import quantize_experts
from ome_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.mark.parametrize("T,E,k,H,I", [(1, 8, 2, 256, 128), (37, 16, 4, 1024, 512), (256, 64, 8, 1024, 256),
                                       (600, 8, 2, 512, 384)])
@pytest.mark.parametrize("tile", ["auto", "64", "128"])
def test_fused_moe_fp8_matches_emulation(T, E, k, H, I, tile, monkeypatch):
    if tile != "auto":   # both row tiles of ome_moe_gemm_fp8_tile, whatever the heuristic picks
        monkeypatch.setenv("OME_MOE_FP8_TILE", tile)
    torch.manual_seed(T + E)
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    w13 = (torch.randn(E, 2 * I, H, device=DEV) * H ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device=DEV) * I ** -0.5).to(torch.bfloat16)
    logits = torch.randn(T, E, device=DEV)
    tw, tid = ops.moe_route(logits, k)
    q13, q2 = quantize_experts(w13), quantize_experts(w2)
    got = ops.fused_moe(x, tw, tid, q13, q2, 0, 1.0)
    want = ref.fused_moe_fp8(x.cpu(), tw.cpu(), tid.cpu(), q13.q.cpu(), q13.scale.cpu(), q2.q.cpu(), q2.scale.cpu())
    err = (got.float().cpu() - want.float()).abs().max().item()
    assert err <= 2e-2 * want.float().abs().max().item() + 1e-3, err
    bf = ops.fused_moe(x, tw, tid, w13, w2, 0, 1.0)
    rel = ((got.float() - bf.float()).norm() / bf.float().norm()).item()
    assert rel < 0.08, rel   # e4m3 weights + activations vs bf16


def test_fp8_experts_stay_fp8_in_model():
    from ome_amd.models import build_model
    from ome_amd.models.config import preset
    from ome_amd.models.quant import Fp8Experts

    cfg = preset("tiny-moe")
    cfg.quantization = "fp8"
    m = build_model(cfg, DEV, torch.bfloat16, load_format="dummy", seed=1)
    assert all(isinstance(m.w13[i], Fp8Experts) and isinstance(m.w2[i], Fp8Experts) for i in m.moe_layers)
    assert m.w13[sorted(m.moe_layers)[0]].q.dtype == torch.float8_e4m3fn


@pytest.mark.parametrize("fp8", [False, True])
def test_fused_moe_combine_adds_shared_output(fp8):
    """``add=``: the shared expert's output summed inside the combine kernel, in place."""
    torch.manual_seed(3)
    T, E, k, H, I = 45, 16, 4, 512, 256
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    w13 = (torch.randn(E, 2 * I, H, device=DEV) * H ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(E, H, I, device=DEV) * I ** -0.5).to(torch.bfloat16)
    tw, tid = ops.moe_route(torch.randn(T, E, device=DEV), k)
    if fp8:
        w13, w2 = quantize_experts(w13), quantize_experts(w2)
    sh = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    plain = ops.fused_moe(x, tw, tid, w13, w2, 0, 2.5)
    acc = sh.clone()
    got = ops.fused_moe(x, tw, tid, w13, w2, 0, 2.5, add=acc)
    assert got.data_ptr() == acc.data_ptr()
    want = sh.float() + plain.float()
    assert (got.float() - want).abs().max().item() <= 2e-2 * want.abs().max().item()

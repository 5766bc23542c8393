"""``ome_gemv`` (batch-1..8 weight-streaming GEMV, ``csrc/kernels/gemv.hip``) vs an fp32 PyTorch
reference: every row count, N not a multiple of the 16-row workgroup span, K tails below one
512-element step, bias, strided activations and output."""
import pytest
import torch

from ome_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("N,K", [(4096, 4096), (6144, 4096), (4096, 14336), (1000, 1032), (37, 200), (16, 8),
                                 (2048, 2560)])
def test_gemv_matches_reference(M, N, K):
    torch.manual_seed(0)
    xs = torch.randn(M, K + 64, device="cuda").to(torch.bfloat16)
    x = xs[:, 16:16 + K]
    w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    want = x.float() @ w.float().t()
    big = torch.full((M, N + 8), 7.0, device="cuda", dtype=torch.bfloat16)
    for bias in (None, b):
        ref = want if bias is None else want + b.float()
        got = ops.gemv(x, w, bias, out=big[:, :N]).float()
        assert (got - ref).abs().max().item() < 1e-2 * max(1.0, ref.abs().max().item())
        assert (big[:, N:] == 7.0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,I", [(4096, 14336), (2048, 8192), (1024, 512)])
def test_gemv_act_equals_act_then_gemv(M, N, I):
    """Down projection with SwiGLU folded into the operand load: bit-identical to act_and_mul
    followed by the plain GEMV (same bf16 rounding of the activation), close to fp32."""
    from ome_amd import ops
    from ome_amd.ops import reference as ref

    torch.manual_seed(M * 7 + N)
    gu = torch.randn(M, 2 * I, device="cuda", dtype=torch.bfloat16) * 2
    w = torch.randn(N, I, device="cuda", dtype=torch.bfloat16) * 0.05
    fused = ops.gemv_act(gu, w)
    two = ops.gemv(ops.act_and_mul(gu, 0), w)
    assert torch.equal(fused, two)
    want = torch.nn.functional.linear(ref.act_and_mul(gu.float().cpu(), 0), w.float().cpu())
    assert torch.allclose(fused.float().cpu(), want, atol=2e-2 * want.abs().max().item(), rtol=2e-2)

"""``ome_skinny_gemm`` (decode-shaped MFMA GEMM, ``csrc/kernels/skinny_gemm.hip``) vs an fp32 PyTorch
reference: row counts that are not multiples of 16, bias, strided activations, split-K with the
last-block reduction (counters re-armed: two back-to-back launches)."""
import pytest
import torch

from ome_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K,splits", [(1, 128, 256, 1), (37, 512, 1024, 1), (100, 256, 2048, 4),
                                          (256, 192, 640, 2), (200, 4096, 4096, 1)])
def test_skinny_gemm_matches_reference(M, N, K, splits):
    torch.manual_seed(0)
    xs = (torch.randn(M, K + 64, device="cuda")).to(torch.bfloat16)
    x = xs[:, 32:32 + K]                                  # strided rows
    w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    want = x.float() @ w.float().t() + b.float()
    for _ in range(2):
        got = ops.skinny_gemm(x, w, b, splits=splits).float()
        assert (got - want).abs().max().item() < 2e-2 * max(1.0, want.abs().max().item())

"""csrc/kernels/gemm.hip (256x256 MFMA tile, global_load_lds double buffer, XOR-swizzled LDS,
XCD-aware tile order, split-K, fused SiLU*mul epilogue) against an fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

from ome_amd import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ref(x, w):
    return x.float() @ w.float().t()


def _rel(a, b):
    return ((a.float() - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("M", [1, 37, 256, 300, 913])
@pytest.mark.parametrize("N,K", [(256, 64), (512, 4096), (6144, 4096), (4096, 14336)])
@pytest.mark.parametrize("splits", [1, 2, 4])
def test_gemm_plain(M, N, K, splits):
    if K % (64 * splits):
        pytest.skip("K not divisible")
    torch.manual_seed(M + N + K + splits)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    y = ops.gemm(x, w, splits=splits)
    assert y.shape == (M, N)
    assert _rel(y, _ref(x, w)) < 1e-2


def test_gemm_asymmetric_identity():
    """A = I-like selector with an asymmetric B: catches a transposed / permuted C write."""
    M, N, K = 256, 512, 256
    x = torch.zeros(M, K, device=DEV, dtype=torch.bfloat16)
    x[torch.arange(M), torch.arange(M) % K] = 1
    w = (torch.arange(N, device=DEV).view(N, 1) * 1000 + torch.arange(K, device=DEV).view(1, K)).to(torch.float32)
    w = (w % 251).to(torch.bfloat16)
    y = ops.gemm(x, w)
    assert torch.equal(y.float(), _ref(x, w))


@pytest.mark.parametrize("M", [1, 64, 256, 700])
@pytest.mark.parametrize("splits", [1, 2])
def test_gemm_silu_mul_epilogue(M, splits):
    I, H = 1792, 1024
    torch.manual_seed(M)
    x = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(2 * I, H, device=DEV, dtype=torch.bfloat16) / H ** 0.5
    y = ops.gemm(x, ops.interleave_gate_up(w), epi=2, splits=splits)
    g, u = _ref(x, w[:I]), _ref(x, w[I:])
    assert y.shape == (M, I)
    assert _rel(y, F.silu(g) * u) < 1e-2


def test_gemm_strided_activation_view():
    M, N, K = 300, 512, 1024
    big = torch.randn(M, K + 128, device=DEV, dtype=torch.bfloat16)
    x = big[:, 64:64 + K]
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    assert _rel(ops.gemm(x, w), _ref(x, w)) < 1e-2

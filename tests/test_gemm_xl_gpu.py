"""csrc/kernels/gemm_xl.hip (round-6 large-tile experiment, not routed): 256 x BN tiles on
32x32x16 MFMAs, persistent per-XCD stream-K, against an fp32 PyTorch reference -- every staging
variant (probe 3 register staging, 4 LDS-DMA, 5 warp-specialised), both epilogues, row tails."""
import pytest
import torch
import torch.nn.functional as F

from ome_amd import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ref(x, w, b=None):
    y = x.float() @ w.float().t()
    return y + b.float() if b is not None else y


def _rel(a, b):
    return ((a.float() - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("M", [256, 700, 1024])
@pytest.mark.parametrize("bn,nwg", [(256, 256), (128, 256), (128, 192)])
@pytest.mark.parametrize("probe", [0, 3, 4])
def test_gemm_xl_plain(M, bn, nwg, probe):
    N, K = 2048, 1024
    torch.manual_seed(M + bn + nwg)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    assert ops.gemm_xl_ok(M, N, K, bn, nwg)
    y = ops.gemm_xl(x, w, bn=bn, nwg=nwg, probe=probe)
    assert _rel(y, _ref(x, w)) < 1e-2


@pytest.mark.parametrize("M", [512, 777])
def test_gemm_xl_warp_specialised(M):
    N, K = 1024, 2048
    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    y = ops.gemm_xl(x, w, bn=128, nwg=256, probe=5)
    assert _rel(y, _ref(x, w)) < 1e-2


def test_gemm_xl_bias_and_silu():
    M, H, I = 640, 1024, 2048
    torch.manual_seed(0)
    x = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(1024, H, device=DEV, dtype=torch.bfloat16) / H ** 0.5
    b = torch.randn(1024, device=DEV, dtype=torch.bfloat16)
    assert _rel(ops.gemm_xl(x, w, b, bn=256), _ref(x, w, b)) < 1e-2
    wgu = torch.randn(2 * I, H, device=DEV, dtype=torch.bfloat16) / H ** 0.5
    y = ops.gemm_xl(x, ops.interleave_gate_up(wgu), epi=2, bn=256)
    assert y.shape == (M, I)
    assert _rel(y, F.silu(_ref(x, wgu[:I])) * _ref(x, wgu[I:])) < 1e-2


def test_gemm_xl_identity_asymmetric():
    """Exact-integer selector: a permuted C write or a mis-staged K-tile changes whole rows."""
    M, N, K = 512, 1024, 512
    x = torch.zeros(M, K, device=DEV, dtype=torch.bfloat16)
    x[torch.arange(M), (torch.arange(M) * 7) % K] = 1
    w = (torch.arange(N, device=DEV).view(N, 1) * 1000 + torch.arange(K, device=DEV).view(1, K)).float()
    w = (w % 251).to(torch.bfloat16)
    assert torch.equal(ops.gemm_xl(x, w, bn=256).float(), _ref(x, w))

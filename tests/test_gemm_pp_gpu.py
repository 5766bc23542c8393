"""csrc/kernels/gemm_pp.hip: ping-pong 256 x 256 MFMA GEMM (two wave groups one barrier apart,
LDS-DMA staging split by group) against an fp32 PyTorch reference, every epilogue."""
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


@pytest.mark.parametrize("M", [1, 100, 256, 257, 913, 2304])
@pytest.mark.parametrize("N,K", [(256, 64), (512, 128), (6144, 4096), (4096, 14336), (2048, 192)])
def test_gemm_pp_plain(M, N, K):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    y = ops.gemm_pp(x, w)
    assert y.shape == (M, N)
    assert _rel(y, _ref(x, w)) < 1e-2


def test_gemm_pp_identity_asymmetric():
    """Exact-integer selector with an asymmetric W: a transposed / permuted C write, a wrong
    swizzle or a mis-staged K-tile changes whole rows, not rounding."""
    M, N, K = 768, 1024, 512
    x = torch.zeros(M, K, device=DEV, dtype=torch.bfloat16)
    x[torch.arange(M), (torch.arange(M) * 7) % K] = 1
    w = (torch.arange(N, device=DEV).view(N, 1) * 1000 + torch.arange(K, device=DEV).view(1, K)).float()
    w = (w % 251).to(torch.bfloat16)
    assert torch.equal(ops.gemm_pp(x, w).float(), _ref(x, w))


@pytest.mark.parametrize("M", [7, 256, 700])
def test_gemm_pp_bias_strided_and_residual(M):
    N, K = 768, 1024
    torch.manual_seed(M)
    big = torch.randn(M, K + 128, device=DEV, dtype=torch.bfloat16)
    x = big[:, 64:64 + K]
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    out_big = torch.zeros(M, N + 64, device=DEV, dtype=torch.bfloat16)
    y = ops.gemm_pp(x, w, b, out=out_big[:, :N])
    assert _rel(y, _ref(x, w, b)) < 1e-2
    assert out_big[:, N:].abs().max().item() == 0
    r = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    want = _ref(x, w, b) + r.float()
    got = ops.gemm_pp(x, w, b, epi=1, res=r)
    assert _rel(got, want) < 1e-2
    r2 = r.clone()   # residual updated in place (res aliases out)
    ops.gemm_pp(x, w, None, out=r2, epi=1, res=r2)
    assert _rel(r2, _ref(x, w) + r.float()) < 1e-2


@pytest.mark.parametrize("M", [1, 256, 1000])
def test_gemm_pp_silu_mul(M):
    I, H = 1792, 1024
    torch.manual_seed(M)
    x = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(2 * I, H, device=DEV, dtype=torch.bfloat16) / H ** 0.5
    y = ops.gemm_pp(x, ops.interleave_gate_up(w), epi=2)
    assert y.shape == (M, I)
    assert _rel(y, F.silu(_ref(x, w[:I])) * _ref(x, w[I:])) < 1e-2


def test_gemm_pp_graph_replay_and_rejects():
    M, N, K = 512, 1024, 1024
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.gemm_pp(x, w, out=out)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.gemm_pp(x, w, out=out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert _rel(out, _ref(x, w)) < 1e-2
    with pytest.raises(ops.NativeError):
        ops.gemm_pp(x, w[:1000], out=out[:, :1000])   # N % 256

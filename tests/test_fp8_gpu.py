"""FP8 W8A8 kernels (csrc/kernels/fp8.hip) vs the plain-PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.quant import Fp8Weight, linear, quantize_weight
from ome_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("group", [0, 128])
@pytest.mark.parametrize("M,K", [(1, 128), (37, 4096), (300, 14336)])
def test_fp8_quant(group, M, K):
    torch.manual_seed(0)
    x = (torch.randn(M, K, device=DEV) * torch.rand(M, 1, device=DEV) * 4).to(torch.bfloat16)
    q, s = ops.fp8_quant(x, group)
    qr, sr = ref.fp8_quant(x.cpu(), group)
    assert torch.allclose(s.cpu(), sr, rtol=1e-6)
    # x * (1/s) on the device vs x * (1/s) on the host: identical except rare 1-ulp rounding ties
    same = (q.cpu().view(torch.uint8) == qr.view(torch.uint8)).float().mean().item()
    assert same > 0.999, same
    assert torch.allclose(q.cpu().float(), qr.float(), rtol=0.13, atol=2 ** -9)


@pytest.mark.parametrize("block", [0, 128])
@pytest.mark.parametrize("M,N,K", [(1, 64, 128), (5, 6144, 4096), (64, 128, 256), (257, 4096, 14336),
                                   (1000, 512, 1024), (700, 6144, 4096), (129, 768, 384), (66, 256, 128)])
@pytest.mark.parametrize("mx_tiles", [112, 1])   # 1: force the 256x256 MX tile wherever it applies
def test_fp8_gemm(block, M, N, K, mx_tiles, monkeypatch):
    monkeypatch.setattr(ops, "FP8_MX_MIN_TILES", mx_tiles)
    torch.manual_seed(1)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(torch.bfloat16)
    qw = quantize_weight(w, block)
    qa, sa = ops.fp8_quant(x, block)
    bias = torch.randn(N, device=DEV).to(torch.bfloat16)
    got = ops.fp8_gemm(qa, sa, qw.q, qw.scale, block, bias)
    want = ref.fp8_gemm(qa.cpu(), sa.cpu(), qw.q.cpu(), qw.scale.cpu(), block, bias.cpu(), torch.float32)
    err = (got.float().cpu() - want).abs().max().item()
    assert err <= 1e-2 * want.abs().max().item() + 1e-3, err


def test_fp8_linear_vs_bf16():
    torch.manual_seed(2)
    x = torch.randn(128, 4096, device=DEV).to(torch.bfloat16)
    w = (torch.randn(1024, 4096, device=DEV) * 0.02).to(torch.bfloat16)
    for block in (0, 128):
        y = linear(x, quantize_weight(w, block))
        want = F.linear(x.float(), w.float())
        assert ((y.float() - want).norm() / want.norm()).item() < 0.05


def test_fp8_engine_decode_graphs():
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model="tiny-llama", max_running_requests=8, context_length=256, quantization="fp8"))
    assert isinstance(eng.runner.model.w_gu[0], Fp8Weight)
    reqs = eng.generate([[5, 6, 7, 8] * 5, [9, 10, 11]] * 3,
                        SamplingParams(max_new_tokens=12, temperature=0.0, ignore_eos=True))
    eng.flush()
    assert all(len(r.output_ids) == 12 for r in reqs)
    assert reqs[0].output_ids == reqs[2].output_ids  # same prompt, greedy


@pytest.mark.parametrize("block", [0, 128])
@pytest.mark.parametrize("M,N,K", [(1, 6144, 4096), (3, 1536, 7168), (8, 576, 7168), (5, 64, 128),
                                   (9, 4096, 14336), (32, 6144, 4096), (64, 128, 256), (100, 1536, 7168),
                                   (128, 4096, 4096), (200, 576, 7168), (256, 6144, 4096)])
@pytest.mark.parametrize("splits", [None, 1])
def test_w8a16_gemm(block, M, N, K, splits):
    """fp8 weight x bf16 activation (csrc/kernels/w8a16.hip) vs the fp32 reference on the
    dequantised weight: GEMV rows (M <= 8) and the skinny MFMA tile with and without split-K."""
    if (M <= 8 and splits == 1) or (block and K % 128):
        pytest.skip("GEMV has no split-K / block 128 needs K % 128 == 0")
    torch.manual_seed(3)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(torch.bfloat16)
    qw = quantize_weight(w, block)
    bias = torch.randn(N, device=DEV).to(torch.bfloat16)
    got = ops.w8a16_gemm(x, qw.q, qw.scale, block, bias, splits=splits)
    wd = ref.fp8_dequant_weight(qw.q.cpu(), qw.scale.cpu(), block).float()
    want = F.linear(x.float().cpu(), wd, bias.float().cpu())
    err = (got.float().cpu() - want).abs().max().item()
    assert err <= 1e-2 * want.abs().max().item() + 1e-2, err
    # graph replay of the split-K path re-arms its tile counters
    if M > 8:
        out = torch.empty_like(got)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ops.w8a16_gemm(x, qw.q, qw.scale, block, bias, out=out, splits=splits)
            with torch.cuda.graph(g, stream=s):
                ops.w8a16_gemm(x, qw.q, qw.scale, block, bias, out=out, splits=splits)
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            out.zero_()
            g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, got)

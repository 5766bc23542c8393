"""csrc/kernels/gemm_sk.hip: per-XCD stream-K MFMA GEMM (fragment-order fp32 slabs, last-arriver
in-launch reduction, 2-, 3- and 4-stage global_load_lds pipelines, 256- and 128-row tiles, bf16+bias
and SiLU*mul epilogues) against an fp32 PyTorch reference."""
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


TILES = [(256, 128), (256, 256), (128, 256), (128, 128)]   # (bm, bn)


def _nwgs(M, N, K, bn, bm=256):
    T = ops.gemm_sk_tiles(M, N, bn, bm)
    cands = {8, 64, 128, 200, 256}
    if T % 8 == 0 and T <= 256:
        cands.add(T)
    return sorted(c for c in cands if ops.gemm_sk_ok(M, N, K, bn, c, bm))


@pytest.mark.parametrize("M", [1, 37, 256, 300, 913])
@pytest.mark.parametrize("N,K", [(256, 64), (512, 4096), (6144, 4096), (4096, 14336)])
@pytest.mark.parametrize("bm,bn", TILES)
def test_gemm_sk_plain(M, N, K, bm, bn):
    torch.manual_seed(M + N + K + bn + bm)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    ref = _ref(x, w)
    for nwg in _nwgs(M, N, K, bn, bm):
        y = ops.gemm_sk(x, w, bn=bn, nwg=nwg, bm=bm)
        assert y.shape == (M, N)
        assert _rel(y, ref) < 1e-2, (nwg, _rel(y, ref))


def test_gemm_sk_identity_asymmetric():
    """A = I-like selector with an asymmetric B: catches a transposed / permuted C write, in every
    decomposition (whole tiles, split tiles, partial slabs of several arrivers)."""
    M, N, K = 512, 1024, 512
    x = torch.zeros(M, K, device=DEV, dtype=torch.bfloat16)
    x[torch.arange(M), torch.arange(M) % K] = 1
    w = (torch.arange(N, device=DEV).view(N, 1) * 1000 + torch.arange(K, device=DEV).view(1, K)).float()
    w = (w % 251).to(torch.bfloat16)
    ref = _ref(x, w)
    for bm, bn in TILES:
        for nwg in _nwgs(M, N, K, bn, bm):
            assert torch.equal(ops.gemm_sk(x, w, bn=bn, nwg=nwg, bm=bm).float(), ref), (bm, bn, nwg)


@pytest.mark.parametrize("M", [1, 64, 256, 700])
@pytest.mark.parametrize("bm,bn", TILES)
def test_gemm_sk_silu_mul(M, bm, bn):
    I, H = 1792, 1024
    torch.manual_seed(M)
    x = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(2 * I, H, device=DEV, dtype=torch.bfloat16) / H ** 0.5
    wi = ops.interleave_gate_up(w)
    g, u = _ref(x, w[:I]), _ref(x, w[I:])
    ref = F.silu(g) * u
    for nwg in _nwgs(M, 2 * I, H, bn, bm):
        y = ops.gemm_sk(x, wi, epi=2, bn=bn, nwg=nwg, bm=bm)
        assert y.shape == (M, I)
        assert _rel(y, ref) < 1e-2, nwg


def test_gemm_sk_bias_and_strided():
    M, N, K = 300, 768, 1024
    big = torch.randn(M, K + 128, device=DEV, dtype=torch.bfloat16)
    x = big[:, 64:64 + K]
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    out_big = torch.zeros(M, N + 64, device=DEV, dtype=torch.bfloat16)
    for bm, bn in TILES:
        for nwg in _nwgs(M, N, K, bn, bm):
            y = ops.gemm_sk(x, w, b, out=out_big[:, :N], bn=bn, nwg=nwg, bm=bm)
            assert _rel(y, _ref(x, w, b)) < 1e-2
    assert out_big[:, N:].abs().max().item() == 0   # nothing written past the output view


def test_gemm_sk_repeat_and_graph_replay():
    """Tickets are re-armed by each tile's last arriver: repeated launches and HIP-graph replays
    of a split decomposition give the same result."""
    M, N, K = 256, 6144, 4096
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    ref = _ref(x, w)
    y0 = ops.gemm_sk(x, w, bn=128, nwg=256)
    for _ in range(5):
        assert _rel(ops.gemm_sk(x, w, bn=128, nwg=256), ref) < 1e-2
    out = torch.empty_like(y0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.gemm_sk(x, w, out=out, bn=128, nwg=256)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.gemm_sk(x, w, out=out, bn=128, nwg=256)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert _rel(out, ref) < 1e-2


def test_gemm_sk_two_streams_concurrently():
    """Stream-K GEMMs on two streams at once (side-stream overlap, TBO halves) must not share
    partial slabs or tickets: each stream gets its own workspace (ops._sk_workspace)."""
    M, N, K = 256, 6144, 4096
    torch.manual_seed(1)
    xs = [torch.randn(M, K, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
    ws = [torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5 for _ in range(2)]
    refs = [_ref(x, w) for x, w in zip(xs, ws)]
    outs = [[torch.empty(M, N, device=DEV, dtype=torch.bfloat16) for _ in range(8)] for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    for i in range(8):   # interleaved issue: the two streams' launches overlap on the device
        for k, s in enumerate(streams):
            with torch.cuda.stream(s):
                ops.gemm_sk(xs[k], ws[k], out=outs[k][i], bn=128, nwg=256)
    torch.cuda.synchronize()
    for k in range(2):
        for o in outs[k]:
            assert _rel(o, refs[k]) < 1e-2
    keys = {key for key in ops._SK_WS if key[1] in (streams[0].cuda_stream, streams[1].cuda_stream)}
    assert len(keys) == 2


def test_gemm_sk_rejects_bad_arguments():
    x = torch.randn(16, 64, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(256, 64, device=DEV, dtype=torch.bfloat16)
    assert not ops.gemm_sk_ok(16, 256, 64, 256, 12)      # nwg not a multiple of 8
    assert not ops.gemm_sk_ok(16, 200, 64, 128, 8)       # N not a multiple of bn
    for bn, nwg in ((256, 12), (64, 8)):
        with pytest.raises(ops.NativeError):
            ops.gemm_sk(x, w, bn=bn, nwg=nwg)


def test_gemm_sk_more_blocks_than_units():
    """Tiny K: fewer (tile, k-step) units than blocks in a group -- empty blocks exit and the
    ticket count only includes blocks that own units."""
    for M, N, K in ((16, 256, 64), (300, 512, 128), (513, 1024, 192)):
        x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
        for bm, bn in TILES:
            for nwg in (16, 64, 256):
                assert _rel(ops.gemm_sk(x, w, bn=bn, nwg=nwg, bm=bm), _ref(x, w)) < 1e-2, (M, N, K, bm, bn, nwg)


# ---------------------------------------------------------------- fp8 W8A8 (Q = 1 per-channel, Q = 2 block 128)
def _fp8_case(M, N, K, block, seed):
    from ome_amd.models.quant import quantize_weight

    torch.manual_seed(seed)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    qa, sa = ops.fp8_quant(x, block)
    fw = quantize_weight(w, block)
    ref = ops.reference.fp8_gemm(qa.cpu(), sa.cpu(), fw.q.cpu(), fw.scale.cpu(), block, out_dtype=torch.float32)
    return qa, sa, fw.q, fw.scale, ref.to(DEV)


@pytest.mark.parametrize("M", [1, 37, 128, 256, 300])
@pytest.mark.parametrize("N,K", [(256, 128), (1024, 4096), (6144, 4096), (4096, 14336)])
@pytest.mark.parametrize("block,bn", [(0, 128), (0, 256), (128, 128)])
def test_gemm_sk_fp8(M, N, K, block, bn):
    qa, sa, qw, sw, ref = _fp8_case(M, N, K, block, M + N + K + block + bn)
    for nwg in (8, 64, 256):
        if not ops.gemm_sk_fp8_ok(M, N, K, bn, nwg):
            continue
        y = ops.gemm_sk_fp8(qa, sa, qw, sw, block, bn=bn, nwg=nwg)
        assert y.shape == (M, N) and y.dtype == torch.bfloat16
        assert _rel(y, ref) < 1e-2, (nwg, _rel(y, ref))


def test_gemm_sk_fp8_identity_block_scales():
    """Selector activations with distinct per-(row, K-group) and per-(N-block, K-block) scales:
    a scale applied to the wrong K-tile, row or W block changes exact small-integer results."""
    M, N, K = 256, 512, 512
    qa = torch.zeros(M, K, device=DEV)
    qa[torch.arange(M), (torch.arange(M) * 7) % K] = 1
    qa = qa.to(torch.float8_e4m3fn)
    qw = ((torch.arange(N, device=DEV).view(N, 1) + 3 * torch.arange(K, device=DEV).view(1, K)) % 13 - 6).float()
    qw = qw.to(torch.float8_e4m3fn)
    sa = (2.0 ** (torch.arange(M * (K // 128), device=DEV) % 3)).float().view(M, K // 128)
    sw = (2.0 ** -(torch.arange((N // 128) * (K // 128), device=DEV) % 4)).float().view(N // 128, K // 128)
    ref = ops.reference.fp8_gemm(qa.cpu(), sa.cpu(), qw.cpu(), sw.cpu(), 128, out_dtype=torch.float32).to(DEV)
    for nwg in (8, 16, 256):
        assert torch.equal(ops.gemm_sk_fp8(qa, sa, qw, sw, 128, nwg=nwg).float(), ref), nwg


@pytest.mark.parametrize("M", [1, 64, 256])
def test_gemm_sk_fp8_silu_mul(M):
    from ome_amd.models.quant import quantize_weight

    I, H = 1792, 1024
    torch.manual_seed(M)
    x = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(2 * I, H, device=DEV, dtype=torch.bfloat16) / H ** 0.5
    qa, sa = ops.fp8_quant(x, 0)
    fw = quantize_weight(ops.interleave_gate_up(w), 0)
    y = ops.gemm_sk_fp8(qa, sa, fw.q, fw.scale, 0, epi=2)
    full = ops.reference.fp8_gemm(qa.cpu(), sa.cpu(), fw.q.cpu(), fw.scale.cpu(), 0, out_dtype=torch.float32)
    g, u = ops.deinterleave_gate_up(full)
    ref = (F.silu(g) * u).to(DEV)
    assert y.shape == (M, I) and _rel(y, ref) < 1e-2


def test_fp8_gemm_routes_decode_rows_to_stream_k():
    """ops.fp8_gemm: decode-sized M goes to the stream-K kernel and matches the library-free reference."""
    for block in (0, 128):
        qa, sa, qw, sw, ref = _fp8_case(200, 2048, 1024, block, 5)
        assert _rel(ops.fp8_gemm(qa, sa, qw, sw, block), ref) < 1e-2

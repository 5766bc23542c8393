"""Varlen bidirectional attention kernel (``varlen_attn.hip``) against the fp32 reference, and the
BERT / XLM-RoBERTa encoders served in bf16 on gfx950 against transformers' fp32 forward."""
import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D", [64, 80, 88, 128])
@pytest.mark.parametrize("causal", [False, True])
def test_varlen_attention_kernel(D, causal):
    torch.manual_seed(D)
    lens = [1, 127, 128, 129, 300, 17]
    T, Hq, Hkv = sum(lens), 8, (2 if D == 128 else 8)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()  # fused projection, read in place
    q = qkv[:, :Hq * D].view(T, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].view(T, Hkv, D)
    got = ops.varlen_attention(q, k, v, lens, D ** -0.5, causal).float()
    want = ref.varlen_attention(q.float(), k.float(), v.float(), lens, D ** -0.5, causal)
    err = (got - want).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("D", [80, 128])
def test_varlen_attention_fast_rescale_paths(D):
    """Fast bidirectional body: long sequences (the two-register-stage ring runs many stages), key
    norms that grow along the sequence (the lazy O / l rescale fires mid-sequence, > 2^8 growth),
    and a tail that is not a multiple of 32 or 64 keys."""
    torch.manual_seed(7 + D)
    lens = [1000, 333, 64, 65]
    T, Hq, Hkv = sum(lens), 4, 2
    q = torch.randn(T, Hq, D, device="cuda")
    k = torch.randn(T, Hkv, D, device="cuda")
    v = torch.randn(T, Hkv, D, device="cuda")
    s0 = 0
    for n in lens:   # key scale ramps 0.2 -> 3: row maxima keep growing by several powers of two
        k[s0:s0 + n] *= torch.linspace(0.2, 3.0, n, device="cuda")[:, None, None]
        s0 += n
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    got = ops.varlen_attention(q, k, v, lens, D ** -0.5).float()
    want = ref.varlen_attention(q.float(), k.float(), v.float(), lens, D ** -0.5)
    err = (got - want).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("D", [64, 72, 128])
def test_varlen_cross_attention_kernel(D):
    """Cross lengths (MiniCPM-V resampler, Phi-4-MM padding queries, Mllama padding rows): query
    sequence s attends to its own packed key rows; an empty key set gives zeros."""
    torch.manual_seed(D)
    lq, lk = [64, 0, 5, 129, 64], [300, 7, 0, 1, 37]
    Hq, Hkv = 4, 2
    q = torch.randn(sum(lq), Hq, D, device="cuda").bfloat16()
    kv = torch.randn(sum(lk), 2, Hkv, D, device="cuda").bfloat16()
    got = ops.varlen_attention(q, kv[:, 0], kv[:, 1], lq, D ** -0.5, k_lengths=lk).float()
    want = ref.varlen_attention(q.float(), kv[:, 0].float(), kv[:, 1].float(), lq, D ** -0.5, k_lengths=lk)
    assert (got - want).abs().max().item() < 2e-2
    assert got[64 + 0 + 5:64 + 5 + 129].abs().max().item() > 0 and got[64:69].abs().max().item() == 0


@pytest.mark.parametrize("kind", ["bert", "xlmr_cls"])
def test_encoder_on_gpu(tmp_path, kind):
    from ome_amd.runtime.engine import Engine, EngineArgs
    from tests.test_encoder_cpu import PROMPTS, _hf, _scores, _want

    hf = _hf(kind)
    hf.save_pretrained(tmp_path, safe_serialization=True)
    want = torch.stack([_want(kind, hf, p) for p in PROMPTS]).float()
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cuda", max_running_requests=4, context_length=256))
    assert not eng.runner.use_graph
    got = _scores(eng, PROMPTS)
    if kind == "bert":
        cos = torch.nn.functional.cosine_similarity(got, want, dim=-1)
        assert cos.min().item() > 0.999, cos
    else:
        assert torch.allclose(got, want, atol=2e-2, rtol=2e-2), (got, want)

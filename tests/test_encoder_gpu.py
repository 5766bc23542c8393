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

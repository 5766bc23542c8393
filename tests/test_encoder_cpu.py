"""BERT / XLM-RoBERTa encoders (``models/bert.py``): embeddings (CLS pooling + L2 norm) and
cross-encoder reranker scores against transformers on tiny random checkpoints, through the
engine's embedding path (varlen bidirectional attention, no KV cache); the ``/v1/rerank`` and
``/v1/embeddings`` endpoints; the varlen-attention reference against SDPA."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from ome_amd.ops import reference as ref  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

V = 300
# ids never equal the XLM-R pad id (0 here): transformers gives pad tokens the padding position
PROMPTS = [[1] + [(7 * i + 3) % 290 + 5 for i in range(37)] + [2], [1, 17, 33, 2], [1] + list(range(40, 140)) + [2]]


def _rand(m):
    torch.manual_seed(0)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "LayerNorm" in n or "norm" in n.lower():
                p.copy_(1 + 0.1 * torch.randn_like(p)) if n.endswith("weight") else p.normal_(0, 0.1)
            else:
                p.normal_(0, 0.05)
    return m.eval()


def _hf(kind: str):
    T = transformers
    common = dict(vocab_size=V, hidden_size=128, num_hidden_layers=2, num_attention_heads=4, intermediate_size=256,
                  max_position_embeddings=256)
    if kind == "bert":
        m = T.BertModel(T.BertConfig(**common), add_pooling_layer=True)
        m.config.architectures = ["BertModel"]
    elif kind == "bert_cls":
        m = T.BertForSequenceClassification(T.BertConfig(num_labels=2, **common))
    elif kind == "xlmr":
        m = T.XLMRobertaModel(T.XLMRobertaConfig(pad_token_id=0, **{**common, "max_position_embeddings": 258}))
        m.config.architectures = ["XLMRobertaModel"]
    else:
        m = T.XLMRobertaForSequenceClassification(T.XLMRobertaConfig(
            pad_token_id=0, num_labels=1, **{**common, "max_position_embeddings": 258}))
    return _rand(m)


def _want(kind, hf, p):
    x = torch.tensor([p])
    with torch.no_grad():
        if kind in ("bert", "xlmr"):
            return torch.nn.functional.normalize(hf(x).last_hidden_state[0, 0], dim=-1)
        return hf(x).logits[0]


def _scores(eng, prompts):
    reqs = [eng.make_request(p, SamplingParams(max_new_tokens=0)) for p in prompts]
    for r in reqs:
        r.is_embedding = True
        eng.add_request(r)
    while not all(r.finished for r in reqs):
        eng.step()
    return torch.tensor([r.embedding for r in reqs])


@pytest.mark.parametrize("kind", ["bert", "bert_cls", "xlmr", "xlmr_cls"])
def test_encoder_matches_hf(tmp_path, kind):
    hf = _hf(kind)
    hf.save_pretrained(tmp_path, safe_serialization=True)
    want = torch.stack([_want(kind, hf, p) for p in PROMPTS])
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    assert type(eng.runner.model).__name__ == "EncoderModel" and eng.cfg.is_embedding
    assert eng.runner.kv.local_layers == [] and eng.scheduler is not None
    got = _scores(eng, PROMPTS)
    assert got.shape == want.shape, (got.shape, want.shape)
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()


def test_varlen_attention_reference_matches_sdpa():
    torch.manual_seed(1)
    lens = [5, 33, 1, 70]
    q, k, v = (torch.randn(sum(lens), 4, 32) for _ in range(3))
    for causal in (False, True):
        got = ref.varlen_attention(q, k, v, lens, 0.2, causal)
        t0 = 0
        for n in lens:
            s = slice(t0, t0 + n)
            w = torch.nn.functional.scaled_dot_product_attention(
                q[s].transpose(0, 1), k[s].transpose(0, 1), v[s].transpose(0, 1), scale=0.2, is_causal=causal)
            assert torch.allclose(got[s], w.transpose(0, 1), atol=1e-5)
            t0 += n


def test_rerank_and_embeddings_endpoints(tmp_path):
    from fastapi.testclient import TestClient

    from ome_amd.runtime.server import create_app

    hf = _hf("xlmr_cls")
    hf.save_pretrained(tmp_path, safe_serialization=True)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=256))
    eng.start()
    try:
        c = TestClient(create_app(eng))
        docs = ["paris is the capital", "bananas", "the eiffel tower"]
        r = c.post("/v1/rerank", json={"query": "capital of france", "documents": docs, "top_n": 2}).json()
        assert len(r["results"]) == 2
        tok = eng.tokenizer
        want = [_want("xlmr_cls", hf, tok.encode_special("capital of france", d))[0].item() for d in docs]
        best = sorted(range(3), key=lambda i: -want[i])[:2]
        assert [x["index"] for x in r["results"]] == best
        assert abs(r["results"][0]["relevance_score"] - want[best[0]]) < 1e-4
        assert r["results"][0]["document"]["text"] == docs[best[0]]
        e = c.post("/v1/embeddings", json={"input": ["hello", "world"]}).json()
        assert len(e["data"]) == 2 and len(e["data"][0]["embedding"]) == 1   # the head's one logit
    finally:
        eng.shutdown()

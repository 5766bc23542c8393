"""Incremental detokenisation (runtime/detok.py) and the server's tool / reasoning parsing with
real special-token ids.

A small byte-level BPE tokenizer is trained here (the ``tokenizers`` library; no download) with
the harmony markers and ``[TOOL_CALLS]`` as special tokens, so the server path sees exactly what a
gpt-oss / Mistral checkpoint would produce: special tokens that a default (skip_special) decode
would erase before the parsers run."""
import json

import pytest

tokenizers = pytest.importorskip("tokenizers")

SPECIALS = ["<|start|>", "<|end|>", "<|message|>", "<|channel|>", "<|call|>", "<|return|>", "[TOOL_CALLS]",
            "<|eos|>"]
CORPUS = ["the weather in Paris is sunny today", "get_weather city Paris Tokyo München 東京 façade",
          "analysis commentary final functions assistant", "{\"city\": \"Paris\"} to=functions.get_weather",
          "naïve café 😀 emoji 🚀 mixed 混合 text", "I should call the weather tool for the user"] * 20


@pytest.fixture(scope="module")
def hf_tok(tmp_path_factory):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    from ome_amd.runtime.tokenizer import HFTokenizer

    t = Tokenizer(models.BPE())
    t.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    t.decoder = decoders.ByteLevel()
    t.train_from_iterator(CORPUS, trainers.BpeTrainer(vocab_size=700, special_tokens=SPECIALS,
                                                       initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    d = tmp_path_factory.mktemp("tok")
    t.save(str(d / "tokenizer.json"))
    (d / "tokenizer_config.json").write_text(json.dumps({"eos_token": "<|eos|>"}))
    return HFTokenizer(d)


@pytest.mark.parametrize("skip", [True, False])
def test_incremental_matches_full_decode(hf_tok, skip):
    from ome_amd.runtime.detok import IncrementalDetokenizer

    text = "naïve café 😀 in München <|channel|>final<|message|>東京 is sunny 🚀 today, façade!"
    ids = hf_tok.encode(text)
    for step in (1, 2, 3, 7):
        det = IncrementalDetokenizer(hf_tok, skip_special=skip)
        out = ""
        for k in range(0, len(ids), step):
            out += det.push(ids[k:k + step])
            assert "�" not in out    # partial UTF-8 never leaks
        out += det.flush()
        assert out == hf_tok.decode(ids, skip_special=skip) == det.text


def test_stop_matcher_tail_only():
    from ome_amd.runtime.detok import StopMatcher

    m = StopMatcher(["STOP", "\n\n"])
    text = "abc" * 100 + "ST"
    assert m.find(text, 2) is None
    text += "OP and more"
    assert m.find(text, len("OP and more")) == 300
    assert StopMatcher([]).find("anything", 3) is None


def _scripted_engine(hf_tok, script):
    """tiny-llama engine whose sampled tokens follow ``script`` (the model computes as usual)."""
    from ome_amd.runtime.engine import Engine, EngineArgs

    eng = Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=4, context_length=512,
                            served_model_name="oss"))
    eng.tokenizer = hf_tok
    eng.eos_ids = {hf_tok.eos_token_id}
    orig = eng.runner.launch

    class _H:
        def __init__(self, ids, lps):
            self.ids, self.lps = ids, lps

        def result(self):
            return self.ids, self.lps

    def launch(batch, prev=None):
        ids, lps = orig(batch, prev).result()
        return _H([script[min(len(c.req.output_ids), len(script) - 1)] for c in batch.chunks], lps)

    eng.runner.launch = launch
    return eng


HARMONY = ("<|channel|>analysis<|message|>I should call the weather tool<|end|><|start|>assistant"
           "<|channel|>commentary to=functions.get_weather<|message|>{\"city\": \"Paris\"}<|call|>")


@pytest.mark.parametrize("stream", [False, True])
def test_gpt_oss_tool_call_through_server(hf_tok, stream):
    from fastapi.testclient import TestClient

    from ome_amd.runtime.server import build_parser, create_app

    script = hf_tok.encode(HARMONY) + [hf_tok.eos_token_id]
    assert all(t < 1024 for t in script)
    eng = _scripted_engine(hf_tok, script)
    ns = build_parser().parse_args(["--tool-call-parser", "gpt-oss", "--reasoning-parser", "gpt-oss"])
    eng.start()
    body = {"model": "oss", "messages": [{"role": "user", "content": "weather in Paris?"}], "max_tokens": 64,
            "temperature": 0, "stream": stream,
            "tools": [{"type": "function", "function": {"name": "get_weather", "parameters": {}}}]}
    try:
        with TestClient(create_app(eng, ns)) as c:
            if not stream:
                r = c.post("/v1/chat/completions", json=body).json()
                msg, finish = r["choices"][0]["message"], r["choices"][0]["finish_reason"]
                calls, reasoning, content = msg.get("tool_calls"), msg.get("reasoning_content"), msg.get("content")
            else:
                with c.stream("POST", "/v1/chat/completions", json=body) as r:
                    evs = [json.loads(ln[6:]) for ln in r.iter_lines() if ln.startswith("data: {")]
                calls, reasoning, content, finish = None, "", "", None
                for e in evs:
                    d = e["choices"][0]["delta"]
                    reasoning += d.get("reasoning_content") or ""
                    content += d.get("content") or ""
                    calls = d.get("tool_calls") or calls
                    finish = e["choices"][0]["finish_reason"] or finish
    finally:
        eng.shutdown()
    assert finish == "tool_calls"
    assert calls and calls[0]["function"]["name"] == "get_weather"
    assert json.loads(calls[0]["function"]["arguments"]) == {"city": "Paris"}
    assert "weather tool" in (reasoning or "")
    assert "<|" not in (content or "") and "<|" not in (reasoning or "")


def test_mistral_tool_calls_marker_survives(hf_tok):
    from fastapi.testclient import TestClient

    from ome_amd.runtime.server import build_parser, create_app

    text = '[TOOL_CALLS][{"name": "get_weather", "arguments": {"city": "Tokyo"}}]'
    script = hf_tok.encode(text) + [hf_tok.eos_token_id]
    eng = _scripted_engine(hf_tok, script)
    ns = build_parser().parse_args(["--tool-call-parser", "mistral"])
    eng.start()
    try:
        with TestClient(create_app(eng, ns)) as c:
            r = c.post("/v1/chat/completions", json={
                "model": "oss", "messages": [{"role": "user", "content": "x"}], "max_tokens": 64, "temperature": 0,
                "tools": [{"type": "function", "function": {"name": "get_weather"}}]}).json()
    finally:
        eng.shutdown()
    msg = r["choices"][0]["message"]
    assert r["choices"][0]["finish_reason"] == "tool_calls"
    assert json.loads(msg["tool_calls"][0]["function"]["arguments"]) == {"city": "Tokyo"}

"""OpenAI-compatible server on CPU (tiny random Llama)."""
import json

import pytest
from fastapi.testclient import TestClient

from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.server import build_parser, create_app, engine_args_from


@pytest.fixture(scope="module")
def client():
    eng = Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=8, context_length=512,
                            served_model_name="tiny"))
    eng.start()
    with TestClient(create_app(eng)) as c:
        yield c
    eng.shutdown()


def test_health_and_models(client):
    assert client.get("/health").json()["status"] == "ok"
    assert client.get("/health_generate").status_code == 200
    m = client.get("/v1/models").json()
    assert m["data"][0]["id"] == "tiny"


def test_completion_and_usage(client):
    r = client.post("/v1/completions", json={"model": "tiny", "prompt": "hello world", "max_tokens": 5,
                                             "temperature": 0, "ignore_eos": True}).json()
    assert r["usage"]["completion_tokens"] == 5
    assert r["choices"][0]["finish_reason"] == "length"


def test_chat_stream(client):
    with client.stream("POST", "/v1/chat/completions", json={
            "model": "tiny", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 4, "stream": True,
            "ignore_eos": True, "temperature": 0}) as r:
        lines = [ln for ln in r.iter_lines() if ln.startswith("data: ")]
    assert lines[-1] == "data: [DONE]"
    chunks = [json.loads(ln[6:]) for ln in lines[:-1]]
    assert chunks[0]["choices"][0]["delta"].get("role") == "assistant"
    assert chunks[-1]["choices"][0]["finish_reason"] == "length"
    assert chunks[-1]["usage"]["completion_tokens"] == 4


def test_completion_stream_chunks(client):
    """Streamed text completions are formatted from a template (server fast path): every chunk
    must still be the OpenAI text_completion object, texts concatenating to the non-streamed
    completion, usage on every chunk with continuous_usage_stats and on the last one otherwise."""
    body = {"model": "tiny", "prompt": "hello there", "max_tokens": 5, "temperature": 0, "ignore_eos": True}
    full = client.post("/v1/completions", json=body).json()
    for cont in (True, False):
        with client.stream("POST", "/v1/completions", json={**body, "stream": True, "stream_options": {
                "include_usage": True, "continuous_usage_stats": cont}}) as r:
            lines = [ln for ln in r.iter_lines() if ln.startswith("data: ")]
        assert lines[-1] == "data: [DONE]"
        chunks = [json.loads(ln[6:]) for ln in lines[:-1]]
        assert all(c["object"] == "text_completion" and c["id"].startswith("cmpl-") and c["model"]
                   and isinstance(c["created"], int) for c in chunks)
        assert "".join(c["choices"][0]["text"] for c in chunks) == full["choices"][0]["text"]
        assert [c["choices"][0]["finish_reason"] for c in chunks][-1] == "length"
        assert all(c["choices"][0]["finish_reason"] is None for c in chunks[:-1])
        assert chunks[-1]["usage"] == {"prompt_tokens": full["usage"]["prompt_tokens"], "completion_tokens": 5,
                                       "total_tokens": full["usage"]["prompt_tokens"] + 5}
        assert all(("usage" in c) == (cont or c is chunks[-1]) for c in chunks)


def test_metrics_names(client):
    txt = client.get("/metrics").text
    for name in ("vllm:request_success_total", "vllm:avg_generation_throughput_toks_per_s",
                 "sglang:time_to_first_token_seconds_bucket", "sglang:num_running_reqs",
                 'ome:host_phase_seconds_total{model_name="tiny",phase="launch"}'):
        assert name in txt


def test_bad_request(client):
    assert client.post("/v1/chat/completions", json={"messages": []}).status_code == 400


def test_sglang_style_flags_parse():
    ns, unknown = build_parser().parse_known_args(
        ["--model-path", "/raid/models/x", "--tp-size", "4", "--mem-frac", "0.9", "--enable-metrics",
         "--trust-remote-code", "--port", "8080", "--log-requests"])
    # --trust-remote-code is on the reference-flag no-op list (runtime/flags.py): accepted, not unknown
    assert ns.tp_size == 4 and ns.mem_frac == 0.9 and "--trust-remote-code" not in unknown
    ea = engine_args_from(ns)
    assert ea.tp_size == 4 and ea.model == "llama-3-8b"  # no config.json -> random-init preset


def test_chat_with_image_data_url():
    """OpenAI ``image_url`` content (data URL) on a vision-language model: the image is decoded,
    expanded into one placeholder per merged patch and served; usage counts the expanded prompt."""
    import base64
    import io

    import numpy as np
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(np.random.default_rng(0).integers(0, 255, (60, 90, 3), dtype=np.uint8)).save(buf, "PNG")
    url = "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()
    eng = Engine(EngineArgs(model="tiny-qwen2-vl", device="cpu", max_running_requests=4, context_length=512,
                            served_model_name="vl"))
    eng.start()
    with TestClient(create_app(eng)) as c:
        msg = [{"role": "user", "content": [{"type": "text", "text": "what is this?"},
                                            {"type": "image_url", "image_url": {"url": url}}]}]
        r = c.post("/v1/chat/completions", json={"model": "vl", "messages": msg, "max_tokens": 4})
        assert r.status_code == 200, r.text
        body = r.json()
        assert body["usage"]["completion_tokens"] == 4
        assert body["usage"]["prompt_tokens"] > 6  # 56x84 resize -> 4x6 patches -> 6 image tokens + text
        bad = [{"role": "user", "content": [{"type": "image_url", "image_url": {"url": "data:image/png;base64,AAAA"}}]}]
        assert c.post("/v1/chat/completions", json={"model": "vl", "messages": bad}).status_code == 400
    eng.shutdown()
    eng2 = Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=4, context_length=256))
    with TestClient(create_app(eng2)) as c:
        assert c.post("/v1/chat/completions", json={"messages": msg}).status_code == 400


def test_n_choices_and_logprobs_format(client):
    r = client.post("/v1/chat/completions", json={
        "model": "tiny", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 3, "n": 3, "seed": 7,
        "temperature": 1.0, "ignore_eos": True, "logprobs": True}).json()
    assert [c["index"] for c in r["choices"]] == [0, 1, 2] and r["usage"]["completion_tokens"] == 9
    lp = r["choices"][0]["logprobs"]["content"]
    assert len(lp) == 3 and all(isinstance(x["logprob"], float) and x["logprob"] <= 0 for x in lp)
    c = client.post("/v1/completions", json={"model": "tiny", "prompt": "abc", "max_tokens": 2, "logprobs": 1,
                                             "temperature": 0, "ignore_eos": True}).json()
    lp = c["choices"][0]["logprobs"]
    assert len(lp["tokens"]) == 2 and len(lp["token_logprobs"]) == 2 and lp["text_offset"][0] == 0

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


def test_metrics_names(client):
    txt = client.get("/metrics").text
    for name in ("vllm:request_success_total", "vllm:avg_generation_throughput_toks_per_s",
                 "sglang:time_to_first_token_seconds_bucket", "sglang:num_running_reqs"):
        assert name in txt


def test_bad_request(client):
    assert client.post("/v1/chat/completions", json={"messages": []}).status_code == 400


def test_sglang_style_flags_parse():
    ns, unknown = build_parser().parse_known_args(
        ["--model-path", "/raid/models/x", "--tp-size", "4", "--mem-frac", "0.9", "--enable-metrics",
         "--trust-remote-code", "--port", "8080", "--log-requests"])
    assert ns.tp_size == 4 and ns.mem_frac == 0.9 and "--trust-remote-code" in unknown
    ea = engine_args_from(ns)
    assert ea.tp_size == 4 and ea.model == "llama-3-8b"  # no config.json -> random-init preset

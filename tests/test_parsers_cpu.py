"""Tool-call and reasoning parsers (``runtime/parsers.py``) and their wiring into
``/v1/chat/completions`` (``--tool-call-parser`` / ``--reasoning-parser``, streaming and not):
the parser families the reference runtimes enable (llama3_json, pythonic, qwen3_coder, nano_v3,
gpt-oss; deepseek-r1 / qwen3 reasoning) on scripted model outputs."""
import json
import threading

import pytest

from ome_amd.runtime.parsers import ReasoningParser, ToolParser


def _args(c):
    return c["function"]["name"], json.loads(c["function"]["arguments"])


def test_llama3_json():
    content, calls = ToolParser("llama3_json").parse(
        '<|python_tag|>{"name": "get_weather", "parameters": {"city": "Paris"}}; {"name": "now", "parameters": {}}')
    assert content == "" and [_args(c) for c in calls] == [("get_weather", {"city": "Paris"}), ("now", {})]
    assert ToolParser("llama3_json").parse("Hello there") == ("Hello there", [])


def test_pythonic():
    content, calls = ToolParser("pythonic").parse('[get_weather(city="Paris", days=3), search(q="x y")]')
    assert [_args(c) for c in calls] == [("get_weather", {"city": "Paris", "days": 3}), ("search", {"q": "x y"})]
    assert ToolParser("pythonic").parse("[not a call") == ("[not a call", [])


def test_qwen3_coder_and_hermes():
    txt = ("Let me check.\n<tool_call>\n<function=get_weather>\n<parameter=city>\nParis\n</parameter>\n"
           "<parameter=days>\n3\n</parameter>\n</function>\n</tool_call>")
    content, calls = ToolParser("qwen3_coder").parse(txt)
    assert content == "Let me check." and _args(calls[0]) == ("get_weather", {"city": "Paris", "days": 3})
    content, calls = ToolParser("hermes").parse('ok <tool_call>{"name": "f", "arguments": {"a": 1}}</tool_call>')
    assert content == "ok" and _args(calls[0]) == ("f", {"a": 1})


def test_nano_v3_and_gpt_oss():
    content, calls = ToolParser("nano_v3").parse('<TOOLCALL>[{"name": "f", "arguments": {"x": [1, 2]}}]</TOOLCALL>')
    assert _args(calls[0]) == ("f", {"x": [1, 2]})
    harmony = ("<|channel|>analysis<|message|>Need weather.<|end|><|start|>assistant<|channel|>commentary "
               "to=functions.get_weather <|constrain|>json<|message|>{\"city\": \"Paris\"}<|call|>")
    content, calls = ToolParser("gpt-oss").parse(harmony)
    assert _args(calls[0]) == ("get_weather", {"city": "Paris"})
    assert ReasoningParser("gpt-oss").split("<|channel|>analysis<|message|>think<|end|><|start|>assistant"
                                            "<|channel|>final<|message|>Answer.<|return|>") == ("think", "Answer.")


@pytest.mark.parametrize("kind,text,want", [
    ("deepseek-r1", "I should add.\n</think>\n\nThe answer is 4.", ("I should add.", "The answer is 4.")),
    ("deepseek-r1", "<think>\nhmm</think>4", ("hmm", "4")),
    ("deepseek-r1", "still thinking", ("still thinking", "")),
    ("qwen3", "<think>\nplan\n</think>\n\nDone.", ("plan", "Done.")),
    ("qwen3", "No thinking here.", (None, "No thinking here.")),
])
def test_reasoning_split_and_stream(kind, text, want):
    assert ReasoningParser(kind).split(text) == want
    p, r, c = ReasoningParser(kind), "", ""
    for k in range(0, len(text), 3):   # 3-char deltas split the markers
        dr, dc = p.feed(text[k:k + 3])
        r, c = r + dr, c + dc
    fr, fc = p.flush()
    r, c = (r + fr).strip(), (c + fc)
    assert (r or None, c.lstrip("\n")) == want


# ------------------------------------------------------------------ through the server
@pytest.fixture()
def scripted(tmp_path):
    from fastapi.testclient import TestClient

    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import ReqState
    from ome_amd.runtime.server import build_parser, create_app

    eng = Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=4, context_length=512))

    def make(output: str, tool="llama3_json", reasoning="deepseek-r1"):
        ids = eng.tokenizer.encode(output)

        def add(req):
            def run():
                for k in range(0, len(ids), 3):
                    req.output_ids.extend(ids[k:k + 3])
                    fin = k + 3 >= len(ids)
                    if fin:
                        req.finish_reason, req.state = "stop", ReqState.FINISHED
                    req.on_token(req, ids[k:k + 3], fin)
            threading.Thread(target=run, daemon=True).start()

        eng.add_request = add
        ns = build_parser().parse_args(["--tool-call-parser", tool, "--reasoning-parser", reasoning])
        return TestClient(create_app(eng, ns))

    return make


TOOLS = [{"type": "function", "function": {"name": "get_weather", "parameters": {"type": "object"}}}]


def test_chat_tool_call_and_reasoning(scripted):
    c = scripted('Paris weather needed.</think>{"name": "get_weather", "parameters": {"city": "Paris"}}')
    r = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "weather?"}],
                                             "tools": TOOLS}).json()
    ch = r["choices"][0]
    assert ch["finish_reason"] == "tool_calls" and ch["message"]["content"] is None
    assert ch["message"]["reasoning_content"] == "Paris weather needed."
    assert _args(ch["message"]["tool_calls"][0]) == ("get_weather", {"city": "Paris"})
    # tool_choice=none: the text is left alone
    r = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "weather?"}],
                                             "tools": TOOLS, "tool_choice": "none"}).json()
    assert "tool_calls" not in r["choices"][0]["message"]


def test_chat_stream_tool_call_and_reasoning(scripted):
    c = scripted('think</think>Sure. <|python_tag|>{"name": "get_weather", "parameters": {"city": "Rome"}}')
    with c.stream("POST", "/v1/chat/completions", json={
            "messages": [{"role": "user", "content": "weather?"}], "tools": TOOLS, "stream": True}) as r:
        chunks = [json.loads(ln[6:]) for ln in r.iter_lines() if ln.startswith("data: ") and ln != "data: [DONE]"]
    deltas = [ch["choices"][0]["delta"] for ch in chunks]
    assert "".join(d.get("reasoning_content", "") for d in deltas) == "think"
    assert "".join(d.get("content", "") for d in deltas).strip() == "Sure."
    calls = [tc for d in deltas for tc in d.get("tool_calls", [])]
    assert len(calls) == 1 and calls[0]["index"] == 0 and _args(calls[0]) == ("get_weather", {"city": "Rome"})
    assert chunks[-1]["choices"][0]["finish_reason"] == "tool_calls"


def test_chat_plain_text_with_parsers(scripted):
    c = scripted("Just an answer.", reasoning="qwen3")
    r = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "hi"}], "tools": TOOLS}).json()
    m = r["choices"][0]["message"]
    assert m["content"] == "Just an answer." and "tool_calls" not in m and m["reasoning_content"] is None


def test_responses_api(scripted):
    c = scripted('weigh it</think>Final. <|python_tag|>{"name": "get_weather", "parameters": {"city": "Oslo"}}')
    r = c.post("/v1/responses", json={"input": "weather in Oslo?", "instructions": "be brief",
                                      "tools": [{"type": "function", "name": "get_weather",
                                                 "parameters": {"type": "object"}}]}).json()
    kinds = [o["type"] for o in r["output"]]
    assert r["object"] == "response" and r["status"] == "completed"
    assert kinds == ["reasoning", "function_call", "message"], kinds
    fc = r["output"][1]
    assert fc["name"] == "get_weather" and json.loads(fc["arguments"]) == {"city": "Oslo"}
    assert r["output_text"] == "Final." and r["usage"]["output_tokens"] > 0

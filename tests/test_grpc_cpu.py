"""gRPC serving mode (verdict r05, missing item 2): the engine with ``--grpc-mode`` serves
``sglang.grpc.scheduler.SglangScheduler`` + ``grpc.health.v1`` on its port; the router reaches
gRPC workers (``grpc://``, or discovered through a container port named ``grpc*``); the node
executor's gRPC probe is a real Health/Check.  Wire-format parity with SGLang's (unpublished)
proto is unpinned; service / method names and grpc.health.v1 are the contract
(``config/runtimes/srt/gpt-oss-120b-rt.yaml:61-130``)."""
import asyncio
import json
import os
import socket
import threading
import time
import urllib.request

import pytest

grpc = pytest.importorskip("grpc")

from ome_amd.runtime import grpc_server as G  # noqa: E402


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_health_protobuf_encoding():
    """Byte-exact grpc.health.v1 messages (the protobuf encoding any kubelet / grpcurl sends)."""
    assert G.encode_health_request("") == b""
    assert G.encode_health_request("sglang.grpc.scheduler.SglangScheduler") == \
        b"\x0a\x25sglang.grpc.scheduler.SglangScheduler"
    assert G.decode_health_request(b"\x0a\x03abc") == "abc" and G.decode_health_request(b"") == ""
    assert G.encode_health_response(G.SERVING) == b"\x08\x01"
    assert G.decode_health_response(b"\x08\x02") == G.NOT_SERVING
    assert G.decode_health_response(b"") == 0


@pytest.fixture(scope="module")
def grpc_engine():
    from ome_amd.runtime.engine import Engine
    from ome_amd.runtime.server import build_parser, create_app, engine_args_from, validate_args

    ns = build_parser().parse_args(["--model-path", "random://tiny-llama", "--device", "cpu", "--context-length",
                                    "256", "--max-running-requests", "8", "--served-model-name", "tiny",
                                    "--grpc-mode", "--watchdog-timeout", "0"])
    validate_args(ns)
    eng = Engine(engine_args_from(ns))
    eng.start()
    app = create_app(eng, ns)
    port = _port()
    loop = asyncio.new_event_loop()

    def run():
        asyncio.set_event_loop(loop)
        try:
            loop.run_until_complete(G.serve(app, eng, "127.0.0.1", port))
        except BaseException:   # noqa: BLE001 -- loop stopped at teardown
            pass

    t = threading.Thread(target=run, daemon=True)
    t.start()
    for _ in range(200):
        try:
            if G.health_check_sync(f"127.0.0.1:{port}", "", timeout=1) == G.SERVING:
                break
        except grpc.RpcError:
            time.sleep(0.05)
    yield eng, port
    eng.shutdown()
    loop.call_soon_threadsafe(loop.stop)


def test_grpc_health_and_scheduler_methods(grpc_engine):
    eng, port = grpc_engine
    tgt = f"127.0.0.1:{port}"
    assert G.health_check_sync(tgt, "") == G.SERVING
    assert G.health_check_sync(tgt, G.SERVICE) == G.SERVING
    with pytest.raises(grpc.RpcError) as e:
        G.health_check_sync(tgt, "no.such.Service")
    assert e.value.code() == grpc.StatusCode.NOT_FOUND

    async def go():
        c = G.SchedulerClient(tgt)
        try:
            info = await c.call("GetModelInfo")
            assert info["served_model_name"] == "tiny" and info["architecture"] == "LlamaForCausalLM"
            hc = await c.call("HealthCheck", timeout=120)
            assert hc["healthy"] is True
            # non-streaming completion: one header frame + the JSON body
            frames = [f async for f in c.generate("/v1/completions", {"prompt": "hello", "max_tokens": 5,
                                                                       "temperature": 0, "ignore_eos": True})]
            assert frames[0][0] == "start" and frames[0][1][0] == 200
            out = json.loads(b"".join(v for k, v in frames if k == "data"))
            assert out["usage"]["completion_tokens"] == 5
            # streaming chat: SSE chunks arrive as separate frames, [DONE] last
            chunks = []
            async for kind, val in c.generate("/v1/chat/completions", {
                    "messages": [{"role": "user", "content": "hi"}], "max_tokens": 6, "stream": True,
                    "temperature": 0, "ignore_eos": True}):
                if kind == "start":
                    assert val[0] == 200 and val[1].startswith("text/event-stream")
                else:
                    chunks.append(val)
            sse = b"".join(chunks).decode()
            assert sse.rstrip().endswith("data: [DONE]") and sse.count("data: ") >= 3
            # a bad request keeps its HTTP status
            frames = [f async for f in c.generate("/v1/chat/completions", {"messages": []})]
            assert frames[0][1][0] == 400
            # Abort: cancels the in-flight stream with that rid; the engine request is aborted
            got = []

            async def long_stream():
                async for kind, val in c.generate("/v1/completions", {"prompt": "x", "max_tokens": 200,
                                                                       "stream": True, "ignore_eos": True},
                                                  rid="abort-me"):
                    got.append(kind)

            task = asyncio.ensure_future(long_stream())
            for _ in range(200):
                if len(got) >= 3:
                    break
                await asyncio.sleep(0.02)
            res = await c.call("Abort", {"rid": "abort-me"})
            await asyncio.wait_for(task, timeout=60)
            assert res["aborted"] is True
        finally:
            await c.close()

    asyncio.run(go())
    time.sleep(0.5)
    assert eng.scheduler.num_running == 0


def test_router_streams_through_grpc_worker(grpc_engine):
    """Router -> gRPC worker (grpc://): the client sees the same OpenAI SSE stream as over HTTP."""
    from aiohttp import web

    from ome_amd.router.server import Router, create_app

    _, port = grpc_engine
    rport = _port()
    r = Router("round_robin", health_interval=0.2, health_path="/HealthCheck")
    r.add_worker(f"grpc://127.0.0.1:{port}")
    loop = asyncio.new_event_loop()
    runner = web.AppRunner(create_app(r))

    def run():
        asyncio.set_event_loop(loop)
        loop.run_until_complete(runner.setup())
        loop.run_until_complete(web.TCPSite(runner, "127.0.0.1", rport).start())
        loop.run_forever()

    threading.Thread(target=run, daemon=True).start()
    base = f"http://127.0.0.1:{rport}"
    for _ in range(300):
        try:
            with urllib.request.urlopen(base + "/readiness", timeout=2) as resp:
                if resp.status == 200:
                    break
        except Exception:  # noqa: BLE001
            time.sleep(0.1)
    req = urllib.request.Request(base + "/v1/chat/completions", data=json.dumps(
        {"model": "tiny", "messages": [{"role": "user", "content": "hello"}], "max_tokens": 4, "stream": True,
         "temperature": 0, "ignore_eos": True}).encode(), headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=60) as resp:
        assert resp.headers["Content-Type"].startswith("text/event-stream")
        body = resp.read().decode()
    assert body.rstrip().endswith("data: [DONE]")
    deltas = [json.loads(x[6:]) for x in body.split("\n\n") if x.startswith("data: {")]
    assert deltas and deltas[0]["object"] == "chat.completion.chunk"
    with urllib.request.urlopen(base + "/v1/models", timeout=10) as resp:
        assert json.loads(resp.read())["data"][0]["id"] == "tiny"
    loop.call_soon_threadsafe(loop.stop)


def test_executor_grpc_probe_is_a_health_check(grpc_engine):
    from ome_amd.executor.kubelet import Kubelet

    _, port = grpc_engine

    class _CR:
        spec = {"ports": [{"containerPort": 8080, "name": "grpc1"}]}

    class _Run:
        ports = {8080: port}

    k = Kubelet.__new__(Kubelet)
    k.probe_scale = 1.0
    assert k._probe_once({"grpc": {"port": 8080, "service": ""}, "timeoutSeconds": 5}, _Run(), _CR())
    assert k._probe_once({"grpc": {"port": "grpc1", "service": G.SERVICE}, "timeoutSeconds": 5}, _Run(), _CR())
    assert not k._probe_once({"grpc": {"port": 8080, "service": "bogus"}, "timeoutSeconds": 5}, _Run(), _CR())
    # a port with no gRPC server behind it fails (a TCP connect alone used to pass)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        s.listen(1)

        class _Run2:
            ports = {8080: s.getsockname()[1]}

        assert not k._probe_once({"grpc": {"port": 8080}, "timeoutSeconds": 1}, _Run2(), _CR())


def test_catalog_has_grpc_counterparts_of_the_reference_grpc_runtimes():
    """The reference's gRPC runtimes (gpt-oss-20b / -120b, Llama-3.1-8B, Llama-4-Maverick FP8 and its
    PD variant) each have a generated counterpart: engine --grpc-mode on port grpc1 with
    grpc.health.v1 probes, router with --health-check-endpoint /HealthCheck; every one of them
    passes the runtime admission webhook."""
    from ome_amd import catalog

    rts, _ = catalog.generate()
    docs = {d["metadata"]["name"]: d for ds in rts.values() for d in ds}
    want = {"gpt-oss-20b": False, "gpt-oss-120b": False, "llama-3-1-8b-instruct": False,
            "llama-4-maverick-17b-128e-instruct-fp8": True}
    for fam, pd in want.items():
        names = [n for n in docs if n.startswith(f"ome-amd-{fam}-grpc-") or
                 (pd and n.startswith(f"ome-amd-{fam}-pd-grpc-"))]
        assert len(names) == (2 if pd else 1), (fam, names)
        for n in names:
            spec = docs[n]["spec"]
            for comp in ("engineConfig", "decoderConfig"):
                r = (spec.get(comp) or {}).get("runner")
                if r is None:
                    continue
                assert "--grpc-mode" in r["args"] and r["ports"][0]["name"] == "grpc1"
                assert r["readinessProbe"]["grpc"]["service"] == G.SERVICE
                assert r["livenessProbe"]["grpc"]["service"] == ""
            cmd = spec["routerConfig"]["runner"]["command"]
            assert cmd[cmd.index("--health-check-endpoint") + 1] == "/HealthCheck"
            assert not spec["supportedModelFormats"][0]["autoSelect"]   # opt-in by runtime name

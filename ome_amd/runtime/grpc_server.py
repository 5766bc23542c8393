"""gRPC serving mode (``--grpc-mode``) for the engine, and the matching client used by the router
and the node executor's probes.

The reference runs three runtimes with the engine behind gRPC instead of HTTP
(``config/runtimes/srt/gpt-oss-120b-rt.yaml:64-130``, ``srt/meta/llama-4-maverick-17b-128e-instruct-
fp8-grpc-rt.yaml:42-109``, ``...-pd-grpc-rt.yaml:70``): the container port is named ``grpc1``, the
kubelet probes it with ``grpc.health.v1.Health/Check`` (service ``""`` for liveness / startup and
``sglang.grpc.scheduler.SglangScheduler`` for readiness), and the router reaches it over gRPC with
``--health-check-endpoint /HealthCheck``.

Contract implemented here (the SGLang proto is not in the reference, so the message encoding of the
scheduler service is this framework's own -- parity of the wire format is **unpinned**; the
service / method names and ``grpc.health.v1`` are the contract):

* ``grpc.health.v1.Health`` -- ``Check`` / ``Watch`` with the real protobuf encoding (hand-coded:
  ``HealthCheckRequest{string service = 1}`` -> ``HealthCheckResponse{ServingStatus status = 1}``);
* ``sglang.grpc.scheduler.SglangScheduler`` --
  ``Generate`` (server streaming): request ``{"path": "/v1/chat/completions" | "/v1/completions" |
  "/generate" | "/v1/embeddings" | ..., "body": {...}, "rid": optional, "headers": {...}}`` (JSON);
  responses are frames ``b"H" + JSON{"status", "content_type"}`` once, then ``b"D" + bytes`` chunks
  of the same body the HTTP server would send (SSE for streams) -- the request is served by the
  engine's own OpenAI / SGLang handlers (called in-process over ASGI), so every feature of the HTTP
  API (chat templates, tools, reasoning, logprobs, embeddings) is available over gRPC;
  ``Abort`` ``{"rid"}`` cancels an in-flight ``Generate`` (its engine request is aborted);
  ``GetModelInfo`` / ``GetServerInfo`` return the HTTP handlers' JSON;
  ``HealthCheck`` runs a one-token generation (``/health_generate``).
"""
from __future__ import annotations

import asyncio
import json
import logging
from typing import AsyncIterator

log = logging.getLogger("ome_amd.grpc")

SERVICE = "sglang.grpc.scheduler.SglangScheduler"
HEALTH_SERVICE = "grpc.health.v1.Health"
SERVING, NOT_SERVING, SERVICE_UNKNOWN = 1, 2, 3


# ---------------------------------------------------------------------- protobuf (grpc.health.v1)
def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _read_varint(buf: bytes, i: int) -> tuple[int, int]:
    shift = val = 0
    while True:
        b = buf[i]
        i += 1
        val |= (b & 0x7F) << shift
        if not b & 0x80:
            return val, i
        shift += 7


def _fields(buf: bytes):
    """Minimal protobuf wire parser: yields (field number, wire type, value)."""
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 2:
            n, i = _read_varint(buf, i)
            v, i = buf[i:i + n], i + n
        elif wt == 1:
            v, i = buf[i:i + 8], i + 8
        elif wt == 5:
            v, i = buf[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield num, wt, v


def encode_health_request(service: str) -> bytes:
    b = service.encode()
    return b"\x0a" + _varint(len(b)) + b if b else b""


def decode_health_request(buf: bytes) -> str:
    for num, wt, v in _fields(buf):
        if num == 1 and wt == 2:
            return bytes(v).decode()
    return ""


def encode_health_response(status: int) -> bytes:
    return b"\x08" + _varint(status)


def decode_health_response(buf: bytes) -> int:
    for num, wt, v in _fields(buf):
        if num == 1 and wt == 0:
            return int(v)
    return 0   # UNKNOWN


def _json_in(b: bytes) -> dict:
    return json.loads(b.decode() or "{}")


def _json_out(d) -> bytes:
    return json.dumps(d).encode()


def _ident(b: bytes) -> bytes:
    return b


# ---------------------------------------------------------------------- in-process ASGI call
async def asgi_call(app, method: str, path: str, body: bytes = b"", headers: dict | None = None,
                    cancelled: asyncio.Event | None = None) -> AsyncIterator[tuple[str, object]]:
    """Drive an ASGI app directly: yields ("start", (status, content_type)) then ("data", bytes)
    chunks as the app sends them (true streaming; a set ``cancelled`` event delivers
    ``http.disconnect``, which ends a FastAPI streaming response and aborts its engine request)."""
    q: asyncio.Queue = asyncio.Queue()
    cancelled = cancelled or asyncio.Event()
    sent = False

    async def receive():
        nonlocal sent
        if not sent:
            sent = True
            return {"type": "http.request", "body": body, "more_body": False}
        await cancelled.wait()
        return {"type": "http.disconnect"}

    async def send(msg):
        await q.put(msg)

    hdrs = [(k.lower().encode(), str(v).encode()) for k, v in (headers or {}).items()]
    if body:
        hdrs.append((b"content-type", b"application/json"))
        hdrs.append((b"content-length", str(len(body)).encode()))
    scope = {"type": "http", "asgi": {"version": "3.0", "spec_version": "2.3"}, "http_version": "1.1",
             "method": method, "scheme": "http", "path": path, "raw_path": path.encode(), "query_string": b"",
             "headers": hdrs, "client": ("127.0.0.1", 0), "server": ("127.0.0.1", 0), "root_path": ""}

    async def run():
        try:
            await app(scope, receive, send)
        finally:
            await q.put(None)

    task = asyncio.create_task(run())
    try:
        while True:
            msg = await q.get()
            if msg is None:
                break
            if msg["type"] == "http.response.start":
                ctype = ""
                for k, v in msg.get("headers") or []:
                    if k.lower() == b"content-type":
                        ctype = v.decode()
                yield "start", (int(msg["status"]), ctype)
            elif msg["type"] == "http.response.body":
                if msg.get("body"):
                    yield "data", msg["body"]
                if not msg.get("more_body"):
                    break
    finally:
        cancelled.set()
        if not task.done():
            try:
                await asyncio.wait_for(task, timeout=30)
            except (asyncio.TimeoutError, asyncio.CancelledError):
                task.cancel()


# ---------------------------------------------------------------------- server
class SchedulerService:
    """The engine behind gRPC: every call is served by the engine's HTTP handlers in-process."""

    def __init__(self, app, engine):
        self.app, self.engine = app, engine
        self.inflight: dict[str, asyncio.Event] = {}

    def healthy(self) -> bool:
        wd = getattr(self.engine, "watchdog", None)
        return not (wd is not None and wd.fired)

    async def Generate(self, request: dict, context):
        path = request.get("path") or "/generate"
        body = request.get("body") or {}
        rid = str(request.get("rid") or "")
        stop = asyncio.Event()
        if rid:
            self.inflight[rid] = stop
        try:
            async for kind, val in asgi_call(self.app, "POST", path, _json_out(body), request.get("headers"), stop):
                if kind == "start":
                    yield b"H" + _json_out({"status": val[0], "content_type": val[1]})
                else:
                    yield b"D" + bytes(val)
        except asyncio.CancelledError:   # client cancelled the call
            stop.set()
            raise
        finally:
            if rid:
                self.inflight.pop(rid, None)

    async def _get_json(self, path: str) -> tuple[int, dict]:
        status, chunks = 500, []
        async for kind, val in asgi_call(self.app, "GET", path):
            if kind == "start":
                status = val[0]
            else:
                chunks.append(val)
        try:
            return status, json.loads(b"".join(chunks) or b"{}")
        except json.JSONDecodeError:
            return status, {}

    async def Abort(self, request: dict, context):
        ev = self.inflight.get(str(request.get("rid") or ""))
        if ev is not None:
            ev.set()
        return _json_out({"aborted": ev is not None})

    async def GetModelInfo(self, request: dict, context):
        return _json_out((await self._get_json("/get_model_info"))[1])

    async def GetServerInfo(self, request: dict, context):
        return _json_out((await self._get_json("/get_server_info"))[1])

    async def HealthCheck(self, request: dict, context):
        status, body = await self._get_json("/health_generate")
        return _json_out({"healthy": status == 200 and self.healthy(), "status": status, **body})

    # grpc.health.v1 ---------------------------------------------------
    def _status(self, service: str) -> int | None:
        if service not in ("", SERVICE):
            return None
        return SERVING if self.healthy() else NOT_SERVING

    async def Check(self, service: str, context):
        import grpc

        st = self._status(service)
        if st is None:
            await context.abort(grpc.StatusCode.NOT_FOUND, f"unknown service {service!r}")
        return st

    async def Watch(self, service: str, context):
        last = None
        while True:
            st = self._status(service)
            st = SERVICE_UNKNOWN if st is None else st
            if st != last:
                yield st
                last = st
            await asyncio.sleep(1.0)

    def handlers(self):
        import grpc

        sched = grpc.method_handlers_generic_handler(SERVICE, {
            "Generate": grpc.unary_stream_rpc_method_handler(self.Generate, request_deserializer=_json_in,
                                                             response_serializer=_ident),
            "Abort": grpc.unary_unary_rpc_method_handler(self.Abort, request_deserializer=_json_in,
                                                         response_serializer=_ident),
            "GetModelInfo": grpc.unary_unary_rpc_method_handler(self.GetModelInfo, request_deserializer=_json_in,
                                                                response_serializer=_ident),
            "GetServerInfo": grpc.unary_unary_rpc_method_handler(self.GetServerInfo, request_deserializer=_json_in,
                                                                 response_serializer=_ident),
            "HealthCheck": grpc.unary_unary_rpc_method_handler(self.HealthCheck, request_deserializer=_json_in,
                                                               response_serializer=_ident),
        })
        health = grpc.method_handlers_generic_handler(HEALTH_SERVICE, {
            "Check": grpc.unary_unary_rpc_method_handler(self.Check, request_deserializer=decode_health_request,
                                                         response_serializer=encode_health_response),
            "Watch": grpc.unary_stream_rpc_method_handler(self.Watch, request_deserializer=decode_health_request,
                                                          response_serializer=encode_health_response),
        })
        return [sched, health]


async def serve(app, engine, host: str, port: int, ready: asyncio.Event | None = None) -> None:
    """Run the gRPC server until cancelled (``--grpc-mode``)."""
    import grpc

    svc = SchedulerService(app, engine)
    server = grpc.aio.server(options=[("grpc.max_receive_message_length", 256 << 20),
                                      ("grpc.max_send_message_length", 256 << 20)])
    server.add_generic_rpc_handlers(svc.handlers())
    bound = server.add_insecure_port(f"{'[::]' if host in ('0.0.0.0', '::') else host}:{port}")
    if not bound:
        raise OSError(f"gRPC server could not bind {host}:{port}")
    await server.start()
    log.info("gRPC %s + %s on %s:%d", SERVICE, HEALTH_SERVICE, host, port)
    if ready is not None:
        ready.set()
    try:
        await server.wait_for_termination()
    finally:
        await server.stop(grace=2)


# ---------------------------------------------------------------------- client
def target_of(url: str) -> str:
    """``grpc://host:port`` (or ``host:port``) -> ``host:port``."""
    return url.split("://", 1)[1].rstrip("/") if "://" in url else url


class SchedulerClient:
    """Async client of :class:`SchedulerService` (the router's gRPC worker transport)."""

    def __init__(self, target: str):
        import grpc

        self.target = target_of(target)
        self.channel = grpc.aio.insecure_channel(self.target, options=[("grpc.max_receive_message_length", 256 << 20),
                                                                       ("grpc.max_send_message_length", 256 << 20)])
        self._gen = self.channel.unary_stream(f"/{SERVICE}/Generate", request_serializer=_json_out,
                                              response_deserializer=_ident)
        self._unary = {m: self.channel.unary_unary(f"/{SERVICE}/{m}", request_serializer=_json_out,
                                                   response_deserializer=_json_in)
                       for m in ("Abort", "GetModelInfo", "GetServerInfo", "HealthCheck")}
        self._check = self.channel.unary_unary(f"/{HEALTH_SERVICE}/Check", request_serializer=encode_health_request,
                                               response_deserializer=decode_health_response)

    async def generate(self, path: str, body: dict, rid: str | None = None, headers: dict | None = None,
                       timeout: float | None = None):
        """-> async iterator of ("start", (status, content_type)) / ("data", bytes)."""
        call = self._gen({"path": path, "body": body, "rid": rid, "headers": headers or {}}, timeout=timeout)
        async for frame in call:
            if frame[:1] == b"H":
                h = json.loads(frame[1:])
                yield "start", (int(h.get("status", 200)), h.get("content_type") or "application/json")
            else:
                yield "data", frame[1:]

    async def call(self, method: str, req: dict | None = None, timeout: float = 30.0) -> dict:
        return await self._unary[method](req or {}, timeout=timeout)

    async def health(self, service: str = SERVICE, timeout: float = 5.0) -> int:
        return await self._check(service, timeout=timeout)

    async def close(self) -> None:
        await self.channel.close()


def health_check_sync(target: str, service: str = "", timeout: float = 5.0) -> int:
    """Blocking ``grpc.health.v1.Health/Check`` (the node executor's gRPC probe): the serving
    status, or raises ``grpc.RpcError``."""
    import grpc

    with grpc.insecure_channel(target_of(target)) as ch:
        fn = ch.unary_unary(f"/{HEALTH_SERVICE}/Check", request_serializer=encode_health_request,
                            response_deserializer=decode_health_response)
        return fn(service, timeout=timeout)


__all__ = ["HEALTH_SERVICE", "SERVICE", "SERVING", "NOT_SERVING", "SERVICE_UNKNOWN", "SchedulerClient",
           "SchedulerService", "asgi_call", "decode_health_request", "decode_health_response",
           "encode_health_request", "encode_health_response", "health_check_sync", "serve", "target_of"]

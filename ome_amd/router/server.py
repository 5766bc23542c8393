"""Router HTTP server (aiohttp): proxying, streaming passthrough, health checking, service
discovery, PD-disaggregated dispatch and Prometheus metrics."""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import random
import time
from dataclasses import dataclass, field
from urllib.parse import urlsplit

from aiohttp import ClientSession, ClientTimeout, TCPConnector, web

from ome_amd.executor.dns import resolve_url
from ome_amd.router.policy import Policy, make_policy

log = logging.getLogger("ome_amd.router")

PROXIED = ("/v1/chat/completions", "/v1/completions", "/generate", "/v1/embeddings", "/v1/rerank", "/v1/score",
           "/encode")


@dataclass
class Worker:
    url: str
    role: str = "regular"          # regular | prefill | decode
    healthy: bool = True
    inflight: int = 0
    fails: int = 0
    served: int = 0
    errors: int = 0
    bootstrap_port: int | None = None
    info: dict = field(default_factory=dict)
    added_at: float = field(default_factory=time.monotonic)
    ever_ok: bool = False          # has any health probe succeeded (--worker-startup-timeout-secs)

    @property
    def host(self) -> str:
        return urlsplit(self.url).hostname or "127.0.0.1"

    @property
    def grpc(self) -> bool:
        """A gRPC-mode engine (``--grpc-mode``: runtime/grpc_server.py), reached as grpc://host:port."""
        return self.url.startswith("grpc://")


def _selector_arg(parts: list[str] | None) -> str | None:
    """``--selector a=b c=d`` (nargs) or ``"a=b c=d"`` -> ``a=b,c=d``."""
    if not parts:
        return None
    toks = []
    for p in parts:
        toks += [t for t in p.replace(",", " ").split() if t]
    return ",".join(toks)


class Router:
    def __init__(self, policy: str = "cache_aware", pd: bool = False, health_interval: float = 5.0,
                 health_failures: int = 3, retries: int = 2, request_timeout: float = 3600.0,
                 discovery: dict | None = None, pd_policy: str | None = None, health_path: str = "/health",
                 startup_timeout: float = 0.0, model_path: str | None = None):
        self.workers: dict[str, Worker] = {}
        self.health_path = health_path if health_path.startswith("/") else "/" + health_path
        self.startup_timeout = float(startup_timeout or 0.0)   # 0: never drop a slow-starting worker
        self.model_path = model_path
        self._grpc: dict = {}   # worker url -> grpc_server.SchedulerClient
        self.policy: Policy = make_policy(policy)
        self.prefill_policy: Policy = make_policy(pd_policy or policy)
        self.decode_policy: Policy = make_policy(pd_policy or policy)
        self.pd = pd
        self.health_interval = health_interval
        self.health_failures = health_failures
        self.retries = retries
        self.timeout = ClientTimeout(total=request_timeout, sock_connect=10)
        self.discovery = discovery
        self.session: ClientSession | None = None
        self.metrics = {"requests": 0, "errors": 0, "retries": 0, "latency_sum": 0.0}
        self._tasks: list[asyncio.Task] = []

    # ------------------------------------------------------------------ workers
    def add_worker(self, url: str, role: str = "regular") -> Worker:
        url = url.rstrip("/")
        w = self.workers.get(url)
        if w is None:
            w = self.workers[url] = Worker(url, role)
            log.info("added %s worker %s", role, url)
        return w

    def _client(self, w: Worker):
        c = self._grpc.get(w.url)
        if c is None:
            from ome_amd.runtime.grpc_server import SchedulerClient

            c = self._grpc[w.url] = SchedulerClient(resolve_url(w.url.replace("grpc://", "http://")).split("://", 1)[1])
        return c

    def remove_worker(self, url: str) -> None:
        url = url.rstrip("/")
        c = self._grpc.pop(url, None)
        if c is not None:
            try:
                asyncio.get_running_loop().create_task(c.close())
            except RuntimeError:   # no loop (admin call from a plain thread): the channel is dropped
                pass
        if self.workers.pop(url, None) is not None:
            for p in (self.policy, self.prefill_policy, self.decode_policy):
                tree = getattr(p, "tree", None)
                if tree is not None:
                    tree.remove_worker(url)
            log.info("removed worker %s", url)

    def healthy(self, role: str) -> list[Worker]:
        # a decode worker is routable only once its KV bootstrap port is known (first probe)
        return [w for w in self.workers.values()
                if w.healthy and w.role == role and (role != "decode" or w.bootstrap_port is not None)]

    async def _probe(self, w: Worker) -> None:
        try:
            if w.grpc:
                from ome_amd.runtime.grpc_server import SERVING

                c = self._client(w)
                if self.health_path.strip("/") == "HealthCheck":   # a one-token generation
                    ok = bool((await c.call("HealthCheck", timeout=60)).get("healthy"))
                else:
                    ok = await c.health(timeout=5) == SERVING
                if ok and w.role == "decode" and w.bootstrap_port is None:
                    w.info = await c.call("GetServerInfo", timeout=5)
                    w.bootstrap_port = int(w.info.get("disaggregation_bootstrap_port") or 0) or None
            else:
                async with self.session.get(resolve_url(w.url) + self.health_path, timeout=ClientTimeout(total=5)) as r:
                    ok = r.status == 200
                if ok and w.role == "decode" and w.bootstrap_port is None:
                    async with self.session.get(resolve_url(w.url) + "/server_info",
                                                timeout=ClientTimeout(total=5)) as r:
                        w.info = await r.json()
                        w.bootstrap_port = int(w.info.get("disaggregation_bootstrap_port") or 0) or None
        except Exception:  # noqa: BLE001
            ok = False
        if ok:
            w.fails, w.healthy, w.ever_ok = 0, True, True
        else:
            w.fails += 1
            if w.fails >= self.health_failures:
                w.healthy = False
            if not w.ever_ok and self.startup_timeout > 0 and \
                    time.monotonic() - w.added_at > self.startup_timeout:
                log.warning("worker %s not healthy %.0f s after it was added (--worker-startup-timeout-secs): "
                            "dropped", w.url, self.startup_timeout)
                self.remove_worker(w.url)

    async def _health_loop(self) -> None:
        while True:
            await asyncio.gather(*(self._probe(w) for w in list(self.workers.values())), return_exceptions=True)
            await asyncio.sleep(self.health_interval)

    async def _discover_once(self) -> None:
        d = self.discovery
        api = os.environ.get("OME_API_SERVER")
        if not d or not api:
            return
        seen = set()
        for role, sel in d["selectors"].items():
            if not sel:
                continue
            url = f"{api.rstrip('/')}/api/v1/namespaces/{d['namespace']}/pods"
            try:
                async with self.session.get(url, params={"labelSelector": sel}, timeout=ClientTimeout(total=5)) as r:
                    pods = (await r.json()).get("items") or []
            except Exception as e:  # noqa: BLE001
                log.warning("service discovery failed: %s", e)
                return
            for p in pods:
                st = p.get("status") or {}
                if not any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or []):
                    continue
                port = d["port"]
                # a container port named grpc* serves the gRPC-mode engine (the reference's grpc1)
                scheme = "http"
                for c in (p.get("spec") or {}).get("containers") or []:
                    for cp in c.get("ports") or []:
                        if int(cp.get("containerPort", -1)) == int(port) and str(cp.get("name", "")).startswith("grpc"):
                            scheme = "grpc"
                hp = json.loads((p["metadata"].get("annotations") or {}).get("ome.io/host-ports") or "{}")
                port = hp.get(str(port), port)
                u = f"{scheme}://{st.get('podIP') or '127.0.0.1'}:{port}"
                seen.add(u)
                self.add_worker(u, role)
        for u in [u for u in self.workers if u not in seen]:
            self.remove_worker(u)

    async def _discovery_loop(self) -> None:
        while True:
            await self._discover_once()
            await asyncio.sleep(self.discovery.get("interval", 5.0))

    async def start(self, app=None) -> None:
        # no pool cap: aiohttp's default (100 connections) would park PD prefill calls behind
        # >= 100 long-lived decode streams, and those streams wait for that very prefill's KV
        self.session = ClientSession(timeout=self.timeout, connector=TCPConnector(limit=0, limit_per_host=0))
        self._tasks.append(asyncio.create_task(self._health_loop()))
        if self.discovery:
            await self._discover_once()
            self._tasks.append(asyncio.create_task(self._discovery_loop()))

    async def stop(self, app=None) -> None:
        for t in self._tasks:
            t.cancel()
        for c in list(self._grpc.values()):
            await c.close()
        self._grpc.clear()
        if self.session:
            await self.session.close()

    # ------------------------------------------------------------------ dispatch
    @staticmethod
    def _text_of(body: dict) -> str:
        if "messages" in body:
            return "\n".join(str(m.get("content", "")) for m in body.get("messages") or [])
        p = body.get("prompt", body.get("text", body.get("input", "")))
        return p if isinstance(p, str) else json.dumps(p)[:4096]

    async def _forward_grpc(self, request: web.Request, w: Worker, body: dict, stream: bool) -> web.StreamResponse:
        """Same response as the HTTP path, carried over the worker's gRPC Generate stream."""
        auth = {k: v for k, v in request.headers.items() if k.lower() == "authorization"}
        resp = None
        status, ctype, buf = 200, "application/json", []
        async for kind, val in self._client(w).generate(request.path, body, headers=auth):
            if kind == "start":
                status, ctype = val
                if stream and status == 200:
                    resp = web.StreamResponse(status=200, headers={"Content-Type": ctype or "text/event-stream",
                                                                   "Cache-Control": "no-cache"})
                    await resp.prepare(request)
            elif resp is not None:
                await resp.write(val)
            else:
                buf.append(val)
        if resp is not None:
            await resp.write_eof()
            return resp
        return web.Response(body=b"".join(buf), status=status, content_type=(ctype or "application/json").split(";")[0])

    async def _forward(self, request: web.Request, w: Worker, body: dict, stream: bool) -> web.StreamResponse:
        if w.grpc:
            import grpc

            w.inflight += 1
            try:
                return await self._forward_grpc(request, w, body, stream)
            except grpc.aio.AioRpcError as e:   # transport failure: retried on another worker
                raise ConnectionError(f"gRPC worker {w.url}: {e.code()}") from e
            finally:
                w.inflight -= 1
                w.served += 1
        url = resolve_url(w.url) + request.path
        w.inflight += 1
        try:
            async with self.session.post(url, json=body, headers={k: v for k, v in request.headers.items()
                                                                  if k.lower() == "authorization"}) as up:
                if not stream or up.status != 200:
                    data = await up.read()
                    return web.Response(body=data, status=up.status, content_type=up.content_type)
                resp = web.StreamResponse(status=200, headers={"Content-Type": up.headers.get(
                    "Content-Type", "text/event-stream"), "Cache-Control": "no-cache"})
                await resp.prepare(request)
                async for chunk in up.content.iter_any():
                    await resp.write(chunk)
                await resp.write_eof()
                return resp
        finally:
            w.inflight -= 1
            w.served += 1

    async def handle(self, request: web.Request) -> web.StreamResponse:
        t0 = time.perf_counter()
        self.metrics["requests"] += 1
        try:
            body = await request.json()
        except json.JSONDecodeError:
            return web.json_response({"error": {"message": "invalid JSON body"}}, status=400)
        stream = bool(body.get("stream"))
        try:
            if self.pd:
                return await self._handle_pd(request, body, stream)
            text = self._text_of(body)
            tried: set[str] = set()
            last_err = None
            for attempt in range(self.retries + 1):
                cands = [w for w in self.healthy("regular") if w.url not in tried]
                if not cands:
                    break
                w = self.policy.pick(cands, text)
                tried.add(w.url)
                try:
                    return await self._forward(request, w, body, stream)
                except (OSError, asyncio.TimeoutError) as e:  # connection-level failure -> retry elsewhere
                    last_err = e
                    w.errors += 1
                    w.fails += 1
                    if w.fails >= self.health_failures:
                        w.healthy = False
                    self.metrics["retries"] += 1
            self.metrics["errors"] += 1
            return web.json_response({"error": {"message": f"no healthy worker available ({last_err})"}}, status=503)
        finally:
            self.metrics["latency_sum"] += time.perf_counter() - t0

    async def _handle_pd(self, request: web.Request, body: dict, stream: bool) -> web.StreamResponse:
        pre, dec = self.healthy("prefill"), self.healthy("decode")
        if not pre or not dec:
            self.metrics["errors"] += 1
            return web.json_response({"error": {"message": "no healthy prefill/decode pair"}}, status=503)
        text = self._text_of(body)
        p = self.prefill_policy.pick(pre, text)
        d = self.decode_policy.pick(dec, text)
        room = random.getrandbits(63)
        common = {"bootstrap_room": room, "bootstrap_host": d.host, "bootstrap_port": d.bootstrap_port}
        pbody = {**body, **common, "stream": False, "disagg_role": "prefill"}
        dbody = {**body, **common, "disagg_role": "decode", "bootstrap_prefill": p.url}

        async def run_prefill():
            p.inflight += 1
            try:
                if p.grpc:
                    async for kind, val in self._client(p).generate(request.path, pbody):
                        if kind == "start" and val[0] != 200:
                            log.warning("prefill worker %s returned %d", p.url, val[0])
                    return
                async with self.session.post(resolve_url(p.url) + request.path, json=pbody) as r:
                    await r.read()
                    if r.status != 200:
                        log.warning("prefill worker %s returned %d", p.url, r.status)
            except Exception as e:  # noqa: BLE001
                log.warning("prefill worker %s failed: %s", p.url, e)
                p.errors += 1
            finally:
                p.inflight -= 1

        ptask = asyncio.create_task(run_prefill())
        try:
            return await self._forward(request, d, dbody, stream)
        finally:
            await ptask

    # ------------------------------------------------------------------ admin / info
    async def models(self, request):
        for w in self.workers.values():
            if w.healthy and w.role in ("regular", "decode") and w.grpc:
                try:
                    info = await self._client(w).call("GetModelInfo", timeout=10)
                    return web.json_response({"object": "list", "data": [
                        {"id": info.get("served_model_name"), "object": "model", "owned_by": "ome_amd",
                         "max_model_len": info.get("context_length")}]})
                except Exception:  # noqa: BLE001
                    continue
            if w.healthy and w.role in ("regular", "decode"):
                try:
                    async with self.session.get(resolve_url(w.url) + "/v1/models") as r:
                        return web.json_response(await r.json(), status=r.status)
                except Exception:  # noqa: BLE001
                    continue
        data = [{"id": self.model_path, "object": "model", "owned_by": "ome_amd"}] if self.model_path else []
        return web.json_response({"object": "list", "data": data})

    async def readiness(self, request):
        ok = (self.healthy("prefill") and self.healthy("decode")) if self.pd else bool(self.healthy("regular"))
        return web.json_response({"status": "ready" if ok else "not ready"}, status=200 if ok else 503)

    async def liveness(self, request):
        return web.json_response({"status": "ok"})

    async def list_workers(self, request):
        return web.json_response({"workers": [{"url": w.url, "role": w.role, "healthy": w.healthy,
                                               "inflight": w.inflight, "served": w.served, "errors": w.errors}
                                              for w in self.workers.values()]})

    async def add_worker_ep(self, request):
        url = request.query.get("url")
        if not url:
            return web.json_response({"error": "url required"}, status=400)
        self.add_worker(url, request.query.get("role", "regular"))
        return web.json_response({"status": "ok"})

    async def remove_worker_ep(self, request):
        self.remove_worker(request.query.get("url", ""))
        return web.json_response({"status": "ok"})

    async def prom(self, request):
        m = self.metrics
        lines = [f"router_requests_total {m['requests']}", f"router_errors_total {m['errors']}",
                 f"router_retries_total {m['retries']}", f"router_request_seconds_sum {m['latency_sum']:.6f}"]
        for w in self.workers.values():
            lab = f'worker="{w.url}",role="{w.role}"'
            lines += [f"router_worker_inflight{{{lab}}} {w.inflight}", f"router_worker_served_total{{{lab}}} {w.served}",
                      f"router_worker_healthy{{{lab}}} {int(w.healthy)}"]
        return web.Response(text="\n".join(lines) + "\n", content_type="text/plain")


def create_app(router: Router, max_payload: int = 256 << 20) -> web.Application:
    # --max-payload-size: larger request bodies are refused with HTTP 413
    app = web.Application(client_max_size=max_payload)
    for p in PROXIED:
        app.router.add_post(p, router.handle)
    app.router.add_get("/v1/models", router.models)
    app.router.add_get("/health", router.liveness)
    app.router.add_get("/liveness", router.liveness)
    app.router.add_get("/readiness", router.readiness)
    app.router.add_get("/list_workers", router.list_workers)
    app.router.add_post("/add_worker", router.add_worker_ep)
    app.router.add_post("/remove_worker", router.remove_worker_ep)
    app.router.add_get("/metrics", router.prom)
    app.on_startup.append(router.start)
    app.on_cleanup.append(router.stop)
    return app


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser("ome_amd.router")
    a = ap.add_argument
    a("--host", default="0.0.0.0")
    a("--port", type=int, default=8080)
    a("--policy", default="cache_aware", choices=["round_robin", "random", "power_of_two", "cache_aware"])
    a("--worker-urls", nargs="*", default=[])
    a("--pd-disaggregation", action="store_true")
    a("--prefill", nargs="+", action="append", default=[], help="prefill URL [bootstrap port]")
    a("--decode", action="append", default=[])
    a("--service-discovery", action="store_true")
    a("--service-discovery-namespace", default=os.environ.get("NAMESPACE", "default"))
    a("--service-discovery-port", type=int, default=8080)
    a("--selector", nargs="*", default=None)
    a("--prefill-selector", nargs="*", default=None)
    a("--decode-selector", nargs="*", default=None)
    a("--health-check-interval-secs", type=float, default=5.0)
    a("--request-timeout-secs", type=float, default=3600.0)
    a("--cache-threshold", type=float, default=0.5)
    a("--model-path", default=None, help="model id reported when no worker answers /v1/models")
    a("--log-level", default="info")
    a("--health-check-endpoint", default="/health", help="worker health path (HTTP) / gRPC method")
    a("--max-payload-size", type=int, default=256 << 20, help="largest request body in bytes (413 above)")
    a("--worker-startup-timeout-secs", type=float, default=0.0,
      help="drop a worker that is not healthy this long after it was added (0: never)")
    return ap


def main(argv=None) -> int:
    ap = build_parser()
    args, unknown = ap.parse_known_args(argv)
    logging.basicConfig(level=getattr(logging, str(args.log_level).upper(), logging.INFO),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    if unknown:   # every reference router flag is handled (ome_amd/runtime/flags.py)
        if os.environ.get("OME_ALLOW_UNKNOWN_FLAGS", "0") == "1":
            log.warning("ignoring unsupported router flags: %s", unknown)
        else:
            ap.error(f"unsupported router flags: {' '.join(unknown)} (OME_ALLOW_UNKNOWN_FLAGS=1 to ignore)")
    disc = None
    if args.service_discovery:
        sels = ({"prefill": _selector_arg(args.prefill_selector), "decode": _selector_arg(args.decode_selector)}
                if args.pd_disaggregation else {"regular": _selector_arg(args.selector)})
        disc = {"namespace": args.service_discovery_namespace, "port": args.service_discovery_port,
                "selectors": sels, "interval": 5.0}
    r = Router(args.policy, pd=args.pd_disaggregation, health_interval=args.health_check_interval_secs,
               request_timeout=args.request_timeout_secs, discovery=disc, health_path=args.health_check_endpoint,
               startup_timeout=args.worker_startup_timeout_secs, model_path=args.model_path)
    for u in args.worker_urls:
        r.add_worker(u)
    for p in args.prefill:
        r.add_worker(p[0], "prefill")
    for d in args.decode:
        r.add_worker(d, "decode")
    web.run_app(create_app(r, args.max_payload_size), host=args.host, port=args.port, print=None)
    return 0

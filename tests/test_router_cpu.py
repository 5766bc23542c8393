"""Router: policies, streaming passthrough, failover, PD dispatch (fake aiohttp workers)."""
import asyncio
import json

from aiohttp import ClientSession, web

from ome_amd.router import Router, create_app
from ome_amd.router.policy import CacheAwarePolicy, PrefixTree


def _worker_app(name, log, role="regular"):
    app = web.Application()

    async def chat(req):
        body = await req.json()
        log.append((name, body))
        if body.get("stream"):
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream"})
            await resp.prepare(req)
            for i in range(3):
                await resp.write(f'data: {json.dumps({"w": name, "i": i})}\n\n'.encode())
            await resp.write(b"data: [DONE]\n\n")
            return resp
        return web.json_response({"worker": name, "role": role})

    async def health(req):
        return web.json_response({"status": "ok"})

    async def info(req):
        return web.json_response({"disaggregation_bootstrap_port": 9999})

    app.router.add_post("/v1/chat/completions", chat)
    app.router.add_get("/health", health)
    app.router.add_get("/server_info", info)
    return app


async def _serve(app):
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    port = site._server.sockets[0].getsockname()[1]
    return runner, f"http://127.0.0.1:{port}"


def test_round_robin_stream_and_failover():
    async def main():
        log = []
        r1, u1 = await _serve(_worker_app("a", log))
        r2, u2 = await _serve(_worker_app("b", log))
        router = Router("round_robin", health_interval=0.2)
        router.add_worker(u1)
        router.add_worker(u2)
        router.add_worker("http://127.0.0.1:1")  # dead worker: connection refused -> retried elsewhere
        rr, ur = await _serve(create_app(router))
        async with ClientSession() as s:
            names = []
            for _ in range(6):
                async with s.post(ur + "/v1/chat/completions", json={"messages": [{"content": "x"}]}) as r:
                    assert r.status == 200
                    names.append((await r.json())["worker"])
            assert set(names) == {"a", "b"}
            async with s.post(ur + "/v1/chat/completions", json={"stream": True, "messages": []}) as r:
                text = (await r.read()).decode()
            assert text.count("data: ") == 4 and text.strip().endswith("[DONE]")
            await asyncio.sleep(0.8)
            async with s.get(ur + "/list_workers") as r:
                ws = {w["url"]: w for w in (await r.json())["workers"]}
            assert not ws["http://127.0.0.1:1"]["healthy"]
            async with s.get(ur + "/metrics") as r:
                assert "router_requests_total 7" in await r.text()
        for x in (rr, r1, r2):
            await x.cleanup()

    asyncio.run(main())


def test_pd_dispatch_sends_room_to_both():
    async def main():
        log = []
        rp, up = await _serve(_worker_app("p", log, "prefill"))
        rd, ud = await _serve(_worker_app("d", log, "decode"))
        router = Router("power_of_two", pd=True, health_interval=0.1)
        router.add_worker(up, "prefill")
        router.add_worker(ud, "decode")
        rr, ur = await _serve(create_app(router))
        await asyncio.sleep(0.3)  # health loop fetches the decode bootstrap port
        async with ClientSession() as s:
            async with s.post(ur + "/v1/chat/completions", json={"messages": [{"content": "hi"}]}) as r:
                assert (await r.json())["worker"] == "d"
            async with s.get(ur + "/readiness") as r:
                assert r.status == 200
        rooms = {n: b["bootstrap_room"] for n, b in log}
        assert rooms["p"] == rooms["d"]
        pbody = next(b for n, b in log if n == "p")
        assert pbody["disagg_role"] == "prefill" and pbody["bootstrap_port"] == 9999 and pbody["stream"] is False
        for x in (rr, rp, rd):
            await x.cleanup()

    asyncio.run(main())


def test_cache_aware_prefers_prefix_owner():
    class W:
        def __init__(self, url):
            self.url, self.inflight = url, 0

    ws = [W("a"), W("b")]
    pol = CacheAwarePolicy(cache_threshold=0.5)
    long = "system prompt " * 40
    first = pol.pick(ws, long + "question one")
    ws[[w.url for w in ws].index(first.url) ^ 1].inflight = 0
    assert pol.pick(ws, long + "question two").url == first.url
    t = PrefixTree(chunk=4, max_chars=64)
    t.insert("a" * 200, "w")
    assert t.chars["w"] <= 64

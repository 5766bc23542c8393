"""multinode-prober: health façade for multi-node (Ray / LWS) inference deployments
(``cmd/multinode-prober/multinode_prober.go``).

    python -m ome_amd.prober --addr :8080 --vllm-endpoint http://<head-svc>:8080

``/healthz`` and ``/readyz`` pass when ``<endpoint>/health`` answers 200; ``/startupz`` passes
once a real chat completion succeeds end-to-end (the engine has loaded weights and can run a
forward across all nodes); ``/metrics`` exposes Prometheus counters of the probe outcomes.
Unlike the reference, which hardcodes the model name ``vllm-model``, the startup probe asks
``/v1/models`` for the served name first.
"""
from __future__ import annotations

import argparse
import json
import logging
import urllib.request

from ome_amd.executor.dns import resolve_url

log = logging.getLogger("ome_amd.prober")


class Prober:
    def __init__(self, endpoint: str, timeout: float = 10.0, inference_timeout: float = 100.0):
        self.endpoint = endpoint.rstrip("/")
        if self.endpoint.endswith("/health"):  # reference default passes the /health URL itself
            self.endpoint = self.endpoint[: -len("/health")]
        self.timeout, self.inference_timeout = timeout, inference_timeout
        self.counts = {"healthz_ok": 0, "healthz_fail": 0, "readyz_ok": 0, "readyz_fail": 0, "startupz_ok": 0,
                       "startupz_fail": 0}
        self._model = None

    def _url(self, path: str) -> str:
        return resolve_url(self.endpoint) + path

    def check_endpoint(self) -> bool:
        try:
            with urllib.request.urlopen(self._url("/health"), timeout=self.timeout) as r:
                return r.status == 200
        except Exception as e:  # noqa: BLE001
            log.info("endpoint %s not healthy: %s", self.endpoint, e)
            return False

    def model_name(self) -> str:
        if self._model is None:
            try:
                with urllib.request.urlopen(self._url("/v1/models"), timeout=self.timeout) as r:
                    data = json.loads(r.read()).get("data") or []
                    self._model = data[0]["id"] if data else "vllm-model"
            except Exception:  # noqa: BLE001
                return "vllm-model"
        return self._model

    def send_inference(self) -> bool:
        body = {"model": self.model_name(), "max_tokens": 8,
                "messages": [{"role": "system", "content": "You are a helpful assistant."},
                             {"role": "user", "content": "Hello, how are you?"}]}
        req = urllib.request.Request(self._url("/v1/chat/completions"), data=json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.inference_timeout) as r:
                return r.status == 200
        except Exception as e:  # noqa: BLE001
            log.info("inference request to %s failed: %s", self.endpoint, e)
            return False

    def probe(self, kind: str) -> bool:
        ok = self.send_inference() if kind == "startupz" else self.check_endpoint()
        self.counts[f"{kind}_{'ok' if ok else 'fail'}"] += 1
        return ok

    def metrics(self) -> str:
        lines = ["# TYPE multinode_prober_checks_total counter"]
        for k, v in self.counts.items():
            kind, res = k.split("_")
            lines.append(f'multinode_prober_checks_total{{probe="{kind}",result="{res}"}} {v}')
        return "\n".join(lines) + "\n"


def create_app(prober: Prober):
    from fastapi import FastAPI
    from fastapi.responses import PlainTextResponse

    app = FastAPI(title="multinode-prober")

    def handler(kind: str):
        def h():
            ok = prober.probe(kind)
            return PlainTextResponse("OK" if ok else "Service Unavailable", status_code=200 if ok else 503)

        return h

    for kind in ("healthz", "readyz", "startupz"):
        app.add_api_route(f"/{kind}", handler(kind), methods=["GET"])
    app.add_api_route("/metrics", lambda: PlainTextResponse(prober.metrics()), methods=["GET"])
    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("ome_amd.prober")
    ap.add_argument("--vllm-endpoint", default="http://localhost:8081/health")
    ap.add_argument("--addr", default=":8081")
    ap.add_argument("--read-timeout", type=float, default=10.0)
    ap.add_argument("--inference-timeout", type=float, default=100.0)
    args, _ = ap.parse_known_args(argv)
    logging.basicConfig(level=logging.INFO)
    host, _, port = args.addr.rpartition(":")
    import uvicorn

    uvicorn.run(create_app(Prober(args.vllm_endpoint, args.read_timeout, args.inference_timeout)),
                host=host or "0.0.0.0", port=int(port), log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

"""Metrics aggregator sidecar (``cmd/qpext``): one ``/metrics`` endpoint that merges the
serving sidecar's (queue-proxy) metrics with the engine container's, so a single Prometheus
scrape target covers both.

Env contract (same keys as the reference):
  AGGREGATE_PROMETHEUS_METRICS_PORT   port this server listens on (default 9088)
  CONTAINER_PROMETHEUS_METRICS_PORT   engine container metrics port (default 8080)
  CONTAINER_PROMETHEUS_METRICS_PATH   engine metrics path (default /metrics)
  QUEUE_PROXY_METRICS_PORT            queue-proxy metrics port (default 9091; empty disables)
  SERVING_SERVICE / SERVING_CONFIGURATION / SERVING_REVISION
                                      appended to every app sample as service_name /
                                      configuration_name / revision_name labels

Untyped app families are sanitised like the reference: ``*_created`` -> counter,
``*_total`` -> gauge (``sanitizeMetrics``).
"""
from __future__ import annotations

import os
import re
import urllib.request

LABEL_ENV = (("service_name", "SERVING_SERVICE"), ("configuration_name", "SERVING_CONFIGURATION"),
             ("revision_name", "SERVING_REVISION"))
_SAMPLE = re.compile(r"^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{([^}]*)\})?(\s+.*)$")


def _scrape(url: str, timeout: float) -> str | None:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.read().decode(errors="replace")
    except Exception:  # noqa: BLE001 — a missing source contributes nothing
        return None


def add_labels(text: str, labels: dict[str, str]) -> str:
    """Append ``labels`` to every sample line; sanitise untyped families."""
    extra = ",".join(f'{k}="{v}"' for k, v in labels.items())
    typed: dict[str, str] = {}
    out = []
    for line in text.splitlines():
        if line.startswith("# TYPE "):
            parts = line.split()
            if len(parts) >= 4:
                name, kind = parts[2], parts[3]
                if kind == "untyped":
                    kind = "counter" if name.endswith("_created") else "gauge" if name.endswith("_total") else kind
                    line = f"# TYPE {name} {kind}"
                typed[name] = kind
            out.append(line)
            continue
        if not line or line.startswith("#"):
            out.append(line)
            continue
        m = _SAMPLE.match(line)
        if not m or not extra:
            out.append(line)
            continue
        name, _, lab, rest = m.groups()
        lab = f"{lab},{extra}" if lab else extra
        out.append(f"{name}{{{lab}}}{rest}")
    return "\n".join(out) + "\n"


def aggregate(app_port: str, app_path: str, qp_port: str | None, timeout: float = 5.0) -> str:
    parts = []
    if qp_port:
        qp = _scrape(f"http://127.0.0.1:{qp_port}/metrics", timeout)
        if qp:
            parts.append(qp if qp.endswith("\n") else qp + "\n")
    if app_port:
        app = _scrape(f"http://127.0.0.1:{app_port}{app_path}", timeout)
        if app:
            labels = {k: os.environ.get(e, "") for k, e in LABEL_ENV if os.environ.get(e)}
            parts.append(add_labels(app, labels))
    return "".join(parts)


def create_app():
    from fastapi import FastAPI, Request
    from fastapi.responses import PlainTextResponse

    app = FastAPI(title="ome-amd metrics aggregator")
    app_port = os.environ.get("CONTAINER_PROMETHEUS_METRICS_PORT", "8080")
    app_path = os.environ.get("CONTAINER_PROMETHEUS_METRICS_PATH", "/metrics")
    qp_port = os.environ.get("QUEUE_PROXY_METRICS_PORT", "9091") or None

    @app.get("/metrics")
    def metrics(request: Request):
        t = request.headers.get("X-Prometheus-Scrape-Timeout-Seconds")
        timeout = float(t) if t else 5.0
        return PlainTextResponse(aggregate(app_port, app_path, qp_port, timeout),
                                 media_type="text/plain; version=0.0.4")

    return app


def main() -> int:
    import uvicorn

    uvicorn.run(create_app(), host="0.0.0.0", port=int(os.environ.get("AGGREGATE_PROMETHEUS_METRICS_PORT", "9088")),
                log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

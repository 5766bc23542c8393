"""Model-agent Prometheus metrics (``pkg/modelagent/metrics.go``), on a private registry so
several agents (tests) can coexist in one process."""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

REGISTRY = CollectorRegistry()
DOWNLOADS = Counter("model_agent_downloads_success_total", "Successful model downloads", ["model"], registry=REGISTRY)
DOWNLOAD_FAILURES = Counter("model_agent_download_failures_total", "Failed download attempts", ["model"],
                            registry=REGISTRY)
DELETES = Counter("model_agent_deletes_total", "Model artifacts removed", ["model"], registry=REGISTRY)
DOWNLOAD_SECONDS = Histogram("model_agent_download_duration_seconds", "Download wall time",
                             buckets=(1, 5, 15, 60, 300, 900, 1800, 3600, 7200), registry=REGISTRY)
DOWNLOAD_BYTES = Counter("model_agent_download_bytes_total", "Bytes materialised on this node", registry=REGISTRY)


def render() -> bytes:
    return generate_latest(REGISTRY)

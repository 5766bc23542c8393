"""Model-agent Prometheus metrics with the reference's series names and labels
(``pkg/modelagent/metrics.go:142-201``): every per-model series is labelled
``model_type`` (BaseModel / ClusterBaseModel), ``namespace`` ("" for cluster-scoped) and ``name``,
so dashboards written against the reference's agent keep working.  A private registry lets
several agents (tests) coexist in one process."""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

REGISTRY = CollectorRegistry()
_L = ["model_type", "namespace", "name"]


def _exp(start: float, factor: float, n: int) -> tuple:
    return tuple(start * factor ** i for i in range(n))


DOWNLOADS = Counter("model_agent_downloads_success_total", "The total number of successful model downloads", _L,
                    registry=REGISTRY)
DOWNLOADS_FAILED = Counter("model_agent_downloads_failed_total", "The total number of failed model downloads", _L,
                           registry=REGISTRY)
VERIFICATIONS = Counter("model_agent_verifications_total", "The total number of model verification attempts",
                        _L + ["result"], registry=REGISTRY)
MD5_FAILED = Counter("model_agent_md5_checksum_failed_total", "The total number of MD5 checksum failures", _L,
                     registry=REGISTRY)
RATE_LIMITS = Counter("model_agent_rate_limit_total", "The total number of rate limit (429) responses encountered",
                      _L, registry=REGISTRY)
DOWNLOAD_SECONDS = Histogram("model_agent_download_duration_seconds", "The duration of model downloads in seconds",
                             _L, buckets=_exp(0.1, 2, 10), registry=REGISTRY)
VERIFICATION_SECONDS = Histogram("model_agent_verification_duration_seconds",
                                 "The duration of model verifications in seconds", buckets=_exp(0.1, 2, 10),
                                 registry=REGISTRY)
DOWNLOAD_BYTES = Counter("model_agent_download_bytes_total", "The total bytes transferred while downloading models",
                         _L, registry=REGISTRY)
RATE_LIMIT_WAIT = Histogram("model_agent_rate_limit_wait_seconds", "The duration waited due to rate limits in seconds",
                            _L, buckets=_exp(1, 2, 10), registry=REGISTRY)
# ome_amd addition (no reference series): artifacts removed from the node
DELETES = Counter("model_agent_deletes_total", "Model artifacts removed", _L, registry=REGISTRY)


def model_labels(obj: dict) -> tuple[str, str, str]:
    """(model_type, namespace, name) of a BaseModel / ClusterBaseModel (GetModelTypeNamespaceAndName)."""
    kind = obj.get("kind") or ""
    md = obj.get("metadata") or {}
    if kind == "ClusterBaseModel":
        return "ClusterBaseModel", "", md.get("name", "")
    if kind == "BaseModel":
        return "BaseModel", md.get("namespace", ""), md.get("name", "")
    return "unknown", "unknown", "unknown"


def record_success(obj: dict) -> None:
    DOWNLOADS.labels(*model_labels(obj)).inc()


def record_failed(obj: dict, error_type: str = "") -> None:   # error_type: logged by the caller, not a label
    DOWNLOADS_FAILED.labels(*model_labels(obj)).inc()


def record_verification(obj: dict, ok: bool) -> None:
    t, ns, n = model_labels(obj)
    if not ok:
        MD5_FAILED.labels(t, ns, n).inc()
    VERIFICATIONS.labels(t, ns, n, "success" if ok else "failure").inc()


def observe_download(obj: dict, seconds: float) -> None:
    DOWNLOAD_SECONDS.labels(*model_labels(obj)).observe(seconds)


def observe_verification(seconds: float) -> None:
    VERIFICATION_SECONDS.observe(seconds)


def record_bytes(obj: dict, n: int) -> None:
    DOWNLOAD_BYTES.labels(*model_labels(obj)).inc(n)


def record_rate_limit(obj: dict, wait_s: float) -> None:
    RATE_LIMITS.labels(*model_labels(obj)).inc()
    RATE_LIMIT_WAIT.labels(*model_labels(obj)).observe(wait_s)


def record_delete(obj: dict) -> None:
    DELETES.labels(*model_labels(obj)).inc()


def render() -> bytes:
    return generate_latest(REGISTRY)

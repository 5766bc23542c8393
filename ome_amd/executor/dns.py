"""Cluster-DNS stand-in: resolve ``<svc>.<ns>.svc.cluster.local[:port]`` (and ingress hosts) to
the executor's local service proxies.  The executor writes the table to ``$OME_LOCAL_DNS``;
clients inside pods (loadgen, router, prober) call :func:`resolve_url` before connecting.
"""
from __future__ import annotations

import json
import os
from urllib.parse import urlsplit, urlunsplit


def _table(path: str | None = None) -> dict:
    path = path or os.environ.get("OME_LOCAL_DNS")
    if not path or not os.path.exists(path):
        return {}
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def resolve_host_port(host: str, port: int | None, path: str | None = None) -> tuple[str, int | None]:
    ent = _table(path).get(host)
    if ent is None:
        return host, port
    if port is None:
        port = 80
    p = ent.get(str(port))
    if p is None and len(ent) == 1:
        p = next(iter(ent.values()))
    return ("127.0.0.1", int(p)) if p is not None else (host, port)


def resolve_url(url: str, path: str | None = None) -> str:
    u = urlsplit(url)
    if not u.hostname:
        return url
    default = 443 if u.scheme == "https" else 80
    host, port = resolve_host_port(u.hostname, u.port or default, path)
    if host == u.hostname:
        return url
    scheme = "http" if u.scheme == "https" else u.scheme  # local proxies speak plain HTTP
    return urlunsplit((scheme, f"{host}:{port}", u.path, u.query, u.fragment))

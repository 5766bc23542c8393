"""Python SDK for the ``ome.io/v1beta1`` API (the reference generates one with openapi-codegen
from ``pkg/openapi/swagger.json``: ``hack/python-sdk/client-gen.sh``, package ``ome``).

Here the client is written against the same document (:mod:`ome_amd.api.openapi`, served by
the manager at ``/openapi/v2``): typed models come from :mod:`ome_amd.sdk.models`
(``V1beta1InferenceService`` ... -- the generated SDK's names), and :class:`OmeClient` wraps the
manager's Kubernetes-style REST routes with per-kind accessors, dry-run admission, merge
patches, status updates, multi-document apply and readiness waits::

    from ome_amd.sdk import OmeClient, models as m
    c = OmeClient("http://127.0.0.1:8080")
    c.cluster_base_models.create(m.V1beta1ClusterBaseModel(metadata={"name": "llama-3-8b"}, spec={...}))
    isvc = c.inference_services.create({"metadata": {"name": "llama", "namespace": "default"},
                                        "spec": {"model": {"name": "llama-3-8b"}}})
    c.inference_services.wait_ready("llama", "default", timeout=900)
"""
from __future__ import annotations

import time
from typing import Any, Iterable

import httpx
import yaml

from ome_amd.api import constants as C
from ome_amd.api import objects as O
from ome_amd.api import v1beta1 as V
from ome_amd.sdk import models  # noqa: F401  (re-export)


class ApiError(RuntimeError):
    def __init__(self, status: int, message: str, body: Any = None):
        super().__init__(f"HTTP {status}: {message}")
        self.status, self.body = status, body


class NotFound(ApiError):
    pass


class Conflict(ApiError):
    pass


class Invalid(ApiError):
    pass


_ERRORS = {404: NotFound, 409: Conflict, 422: Invalid}


def _as_dict(obj) -> dict:
    if isinstance(obj, V.Model):
        return obj.dump()
    if isinstance(obj, dict):
        return obj
    raise TypeError(f"expected a dict or an ome_amd model, got {type(obj).__name__}")


def is_ready(obj) -> bool:
    """Ready condition True (InferenceService) or state Ready / Completed (models, benchmarks)."""
    d = _as_dict(obj)
    st = d.get("status") or {}
    if st.get("state") in ("Ready", "Completed"):
        return True
    return any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or [])


def is_failed(obj) -> bool:
    d = _as_dict(obj)
    st = d.get("status") or {}
    if st.get("state") == "Failed":
        return True
    return any(c.get("type") == "Ready" and c.get("status") == "False" and c.get("reason") in
               ("ModelLoadFailed", "RuntimeNotRecognized", "NoSupportingRuntime", "Failed")
               for c in st.get("conditions") or [])


class OmeClient:
    def __init__(self, base_url: str = "http://127.0.0.1:8080", token: str | None = None, timeout: float = 30.0,
                 typed: bool = True, transport: httpx.BaseTransport | None = None):
        headers = {"Authorization": f"Bearer {token}"} if token else {}
        self.base = base_url.rstrip("/")
        self.http = httpx.Client(base_url=self.base, headers=headers, timeout=timeout, transport=transport)
        self.typed = typed
        for kind, (plural, _ns, _spec) in V.KINDS.items():
            setattr(self, _attr(plural), Resource(self, kind))

    # ------------------------------------------------------------------ plumbing
    def close(self):
        self.http.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def path(self, kind: str, namespace: str | None = None, name: str | None = None, sub: str | None = None) -> str:
        plural, namespaced, _ = V.KINDS[kind]
        if namespaced and not namespace:
            namespace = "default"
        p = f"/apis/{C.API_VERSION}/" + (f"namespaces/{namespace}/" if namespaced else "") + plural
        if name:
            p += f"/{name}"
        if sub:
            p += f"/{sub}"
        return p

    def _call(self, method: str, path: str, **kw) -> Any:
        r = self.http.request(method, path, **kw)
        body = r.json() if r.content and r.headers.get("content-type", "").startswith("application/json") else r.text
        if r.status_code >= 400 or (isinstance(body, dict) and body.get("status") == "Failure"):
            code = body.get("code", r.status_code) if isinstance(body, dict) else r.status_code
            msg = body.get("message") or body.get("detail") if isinstance(body, dict) else str(body)
            raise _ERRORS.get(code, ApiError)(code, str(msg), body)
        return body

    def _out(self, d: dict, typed: bool | None):
        return O.parse(d) if (self.typed if typed is None else typed) and d.get("kind") in O.OBJECTS else d

    # ------------------------------------------------------------------ CRUD
    def create(self, obj, dry_run: bool = False, typed: bool | None = None):
        d = _as_dict(obj)
        kind = d.get("kind")
        if kind not in V.KINDS:
            raise ValueError(f"unknown kind {kind!r}; expected one of {sorted(V.KINDS)}")
        d.setdefault("apiVersion", C.API_VERSION)
        ns = (d.get("metadata") or {}).get("namespace")
        out = self._call("POST", self.path(kind, ns), json=d, params={"dryRun": "All"} if dry_run else None)
        return self._out(out, typed)

    def get(self, kind: str, name: str, namespace: str | None = None, typed: bool | None = None):
        return self._out(self._call("GET", self.path(kind, namespace, name)), typed)

    def list(self, kind: str, namespace: str | None = None, label_selector: str | None = None, typed: bool | None = None):
        plural, namespaced, _ = V.KINDS[kind]
        path = self.path(kind, namespace) if (namespace or not namespaced) else f"/apis/{C.API_VERSION}/{plural}"
        body = self._call("GET", path, params={"labelSelector": label_selector} if label_selector else None)
        if self.typed if typed is None else typed:
            return O.parse_list(kind, body)
        return body

    def replace(self, obj, typed: bool | None = None):
        d = _as_dict(obj)
        m = d.get("metadata") or {}
        return self._out(self._call("PUT", self.path(d["kind"], m.get("namespace"), m["name"]), json=d), typed)

    def replace_status(self, obj, typed: bool | None = None):
        d = _as_dict(obj)
        m = d.get("metadata") or {}
        return self._out(self._call("PUT", self.path(d["kind"], m.get("namespace"), m["name"], "status"), json=d), typed)

    def patch(self, kind: str, name: str, patch: dict, namespace: str | None = None, typed: bool | None = None):
        out = self._call("PATCH", self.path(kind, namespace, name), json=patch,
                         headers={"Content-Type": "application/merge-patch+json"})
        return self._out(out, typed)

    def delete(self, kind: str, name: str, namespace: str | None = None) -> dict:
        return self._call("DELETE", self.path(kind, namespace, name))

    def apply(self, manifests: str | Iterable[dict]) -> list[dict]:
        """Create-or-update every document (the manager's ``/apply``: same admission chain)."""
        text = manifests if isinstance(manifests, str) else yaml.safe_dump_all([_as_dict(x) for x in manifests])
        return self._call("POST", "/apply", content=text.encode(), headers={"Content-Type": "application/yaml"})["items"]

    def wait(self, kind: str, name: str, namespace: str | None = None, predicate=is_ready, timeout: float = 600.0,
             poll: float = 1.0, fail=is_failed, typed: bool | None = None):
        """Poll until ``predicate(obj)``; raise on ``fail(obj)`` or after ``timeout`` seconds."""
        deadline = time.monotonic() + timeout
        last = None
        while True:
            try:
                last = self.get(kind, name, namespace, typed=False)
                if predicate(last):
                    return self._out(last, typed)
                if fail is not None and fail(last):
                    raise ApiError(500, f"{kind} {name} failed: {(last.get('status') or {})}", last)
            except NotFound:
                last = None
            if time.monotonic() > deadline:
                raise TimeoutError(f"{kind} {namespace + '/' if namespace else ''}{name} not ready after {timeout}s"
                                   f" (status: {(last or {}).get('status')})")
            time.sleep(poll)

    def logs(self, pod: str, namespace: str = "default", container: str | None = None) -> str:
        r = self.http.get(f"/api/v1/namespaces/{namespace}/pods/{pod}/log", params={"container": container} if container else None)
        if r.status_code >= 400:
            raise _ERRORS.get(r.status_code, ApiError)(r.status_code, r.text)
        return r.text

    def openapi(self) -> dict:
        return self._call("GET", "/openapi/v2")


def _attr(plural: str) -> str:
    """``inferenceservices`` -> ``inference_services`` (accessor names)."""
    words = {"inferenceservices": "inference_services", "basemodels": "base_models",
             "clusterbasemodels": "cluster_base_models", "finetunedweights": "fine_tuned_weights",
             "servingruntimes": "serving_runtimes", "clusterservingruntimes": "cluster_serving_runtimes",
             "acceleratorclasses": "accelerator_classes", "benchmarkjobs": "benchmark_jobs"}
    return words.get(plural, plural)


class Resource:
    """Per-kind accessor: ``client.inference_services.get("llama", "default")``."""

    def __init__(self, client: OmeClient, kind: str):
        self.client, self.kind = client, kind
        self.namespaced = V.KINDS[kind][1]

    def _obj(self, obj) -> dict:
        d = dict(_as_dict(obj))
        d.setdefault("kind", self.kind)
        if d["kind"] != self.kind:
            raise ValueError(f"{self.kind} accessor given a {d['kind']}")
        return d

    def create(self, obj, dry_run: bool = False, **kw):
        return self.client.create(self._obj(obj), dry_run=dry_run, **kw)

    def get(self, name: str, namespace: str | None = None, **kw):
        return self.client.get(self.kind, name, namespace, **kw)

    def list(self, namespace: str | None = None, label_selector: str | None = None, **kw):
        return self.client.list(self.kind, namespace, label_selector, **kw)

    def replace(self, obj, **kw):
        return self.client.replace(self._obj(obj), **kw)

    def replace_status(self, obj, **kw):
        return self.client.replace_status(self._obj(obj), **kw)

    def patch(self, name: str, patch: dict, namespace: str | None = None, **kw):
        return self.client.patch(self.kind, name, patch, namespace, **kw)

    def delete(self, name: str, namespace: str | None = None):
        return self.client.delete(self.kind, name, namespace)

    def wait_ready(self, name: str, namespace: str | None = None, timeout: float = 600.0, poll: float = 1.0, **kw):
        return self.client.wait(self.kind, name, namespace, timeout=timeout, poll=poll, **kw)


__all__ = ["OmeClient", "Resource", "ApiError", "NotFound", "Conflict", "Invalid", "is_ready", "is_failed", "models"]

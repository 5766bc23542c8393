"""Web-console REST backend.

Same route table as the reference console backend (``web-console/backend/internal/api/
server.go:56-156``): ClusterBaseModel CRUD + status / events / download progress, namespaced
BaseModel CRUD, ClusterServingRuntime CRUD + fetch-yaml / compatible / recommend / validate /
compatibility / clone, InferenceService CRUD + status, AcceleratorClasses, namespaces, YAML /
model / runtime validation, Hugging Face model search / info / config, and a Server-Sent-Events
stream of resource changes.

Design differences (MI355X node, no Kubernetes): the backend talks to an ``ome_amd`` object
store — in-process (mounted into ``python -m ome_amd.manager``) or a remote manager over its
k8s-style REST API (:class:`ome_amd.console.remote.RemoteStore`); writes go through the store's
admission chain, so the console gets the same defaulting/validation as ``omectl apply``; runtime
recommendations come from the controller's own RuntimeSelector; Hugging Face lookups are answered
offline from the local hub cache and the model catalog (no egress on the serving node).
"""
from __future__ import annotations

import asyncio
import json
import os
import queue
import re
import threading
import time
from pathlib import Path

import yaml
from fastapi import Request  # module level: FastAPI resolves the string annotations against it

from ome_amd.api import v1beta1 as V
from ome_amd.console import hf as HF
from ome_amd.console import intelligence as RI

API = "ome.io/v1beta1"
STATIC = Path(__file__).resolve().parent / "static"

RESOURCE_OF_KIND = {"ClusterBaseModel": "models", "BaseModel": "basemodels", "ClusterServingRuntime": "runtimes",
                    "ServingRuntime": "runtimes", "InferenceService": "services", "AcceleratorClass": "accelerators",
                    "Namespace": "namespaces", "BenchmarkJob": "benchmarks"}
_EVENT_TYPE = {"ADDED": "add", "MODIFIED": "update", "DELETED": "delete"}


class EventBroadcaster:
    """Fan-out of store watch events to SSE subscribers (reference k8s/client.go:104-142)."""

    def __init__(self, store):
        self.subs: list[queue.Queue] = []
        self.lock = threading.Lock()
        self.store = store
        self._entry = store.watch(self._on_event, kinds=list(RESOURCE_OF_KIND))

    def _on_event(self, ev) -> None:
        kind = ev.obj.get("kind")
        msg = {"type": _EVENT_TYPE.get(ev.type, ev.type.lower()), "resource": RESOURCE_OF_KIND.get(kind, kind),
               "name": ev.obj.get("metadata", {}).get("name"), "namespace": ev.obj.get("metadata", {}).get("namespace"),
               "data": ev.obj}
        with self.lock:
            subs = list(self.subs)
        for q in subs:
            try:
                q.put_nowait(msg)
            except queue.Full:  # a stalled client drops events rather than blocking the store
                pass

    def subscribe(self) -> queue.Queue:
        q: queue.Queue = queue.Queue(maxsize=1000)
        with self.lock:
            self.subs.append(q)
        return q

    def unsubscribe(self, q: queue.Queue) -> None:
        with self.lock:
            if q in self.subs:
                self.subs.remove(q)

    def close(self) -> None:
        self.store.unwatch(self._entry)


_GITHUB = re.compile(r"^https?://(?:github\.com/[^/]+/[^/]+/(?:blob|raw)/[^/]+|raw\.githubusercontent\.com/[^/]+/[^/]+/[^/]+)/(.*)$")


def _candidates(p: str, roots: list[Path]):
    """Where a fetch-yaml argument may live: an absolute path, or -- for a catalog-relative path
    or a GitHub blob URL of a repository laid out like the catalog (``config/runtimes/...``) --
    that path under each root, with and without a leading ``config/``."""
    m = _GITHUB.match(p.strip())
    rel = m.group(1) if m else p.strip()
    if not m and Path(rel).is_absolute():
        yield Path(rel)
        return
    parts = Path(rel).parts
    tails = [Path(*parts)] + ([Path(*parts[1:])] if len(parts) > 1 and parts[0] == "config" else [])
    for r in roots:
        for t in tails:
            yield r / t
            yield r / "runtimes" / t


def _sanitize_yaml_path(p: str, roots: list[Path]) -> Path | None:
    """fetch-yaml only reads YAML files under the configured catalog roots (the reference
    restricts the URL host to github.com, runtimes.go:222-326; here there is no egress, so a
    GitHub URL is mapped onto the local catalog and anything outside the roots is refused)."""
    for cand in _candidates(p, roots):
        try:
            rp = cand.resolve()
        except (OSError, RuntimeError):
            continue
        if rp.suffix not in (".yaml", ".yml") or not rp.is_file():
            continue
        for r in roots:
            try:
                rp.relative_to(r.resolve())
                return rp
            except ValueError:
                continue
    return None


def _catalog(roots: list[Path], installed: set[str]) -> list[dict]:
    """Runtime YAMLs under the catalog roots (the import page's picker)."""
    out = []
    for r in roots:
        base = r / "runtimes" if (r / "runtimes").is_dir() else r
        for f in sorted(base.rglob("*.yaml")):
            try:
                docs = [d for d in yaml.safe_load_all(f.read_text()) if isinstance(d, dict)]
            except (OSError, yaml.YAMLError):
                continue
            rts = [d for d in docs if d.get("kind") in ("ClusterServingRuntime", "ServingRuntime")]
            if rts:
                name = (rts[0].get("metadata") or {}).get("name")
                out.append({"path": str(f.relative_to(r)), "name": name, "kind": rts[0]["kind"],
                            "installed": name in installed})
    return out


def create_router(store, catalog_roots: list[str] | None = None, models_root: str | None = None):
    """FastAPI router with the console API (mount under ``/api/v1`` standalone, or under a prefix
    next to the manager's own ``/api`` routes)."""
    from fastapi import APIRouter, HTTPException
    from fastapi.responses import StreamingResponse

    from ome_amd.store import store as S

    r = APIRouter()
    roots = [Path(p) for p in (catalog_roots or [str(Path(__file__).resolve().parents[2] / "config")])]
    bcast = EventBroadcaster(store)
    r.broadcaster = bcast  # type: ignore[attr-defined]

    def fail(e: Exception, what: str):
        code = {S.NotFound: 404, S.AlreadyExists: 409, S.Conflict: 409, S.Invalid: 422}.get(type(e), 400)
        raise HTTPException(code, {"error": what, "details": str(e)})

    def items(kind: str, ns: str | None = None, selector: str | None = None) -> dict:
        objs = store.list(API, kind, ns, selector=selector)
        return {"items": objs, "total": len(objs)}

    async def body(req: Request) -> dict:
        raw = await req.body()
        ctype = req.headers.get("content-type", "")
        data = yaml.safe_load(raw) if "yaml" in ctype else json.loads(raw or b"{}")
        if not isinstance(data, dict):
            raise HTTPException(400, {"error": "body must be an object"})
        return data

    def put_obj(kind: str, name: str, data: dict, ns: str | None = None) -> dict:
        try:
            cur = store.get(API, kind, name, ns)
        except Exception as e:  # noqa: BLE001
            fail(e, f"{kind} not found")
        data.setdefault("apiVersion", API)
        data["kind"] = kind
        meta = data.setdefault("metadata", {})
        meta["name"] = name
        if ns:
            meta["namespace"] = ns
        meta.setdefault("resourceVersion", cur["metadata"].get("resourceVersion"))
        try:
            return store.update(data)
        except Exception as e:  # noqa: BLE001
            fail(e, f"failed to update {kind}")

    def post_obj(kind: str, data: dict, ns: str | None = None) -> dict:
        data.setdefault("apiVersion", API)
        data["kind"] = kind
        if ns:
            data.setdefault("metadata", {})["namespace"] = ns
        try:
            return store.create(data)
        except Exception as e:  # noqa: BLE001
            fail(e, f"failed to create {kind}")

    def get_obj(kind: str, name: str, ns: str | None = None) -> dict:
        try:
            return store.get(API, kind, name, ns)
        except Exception as e:  # noqa: BLE001
            fail(e, f"{kind} not found")

    def del_obj(kind: str, name: str, ns: str | None = None) -> dict:
        try:
            store.delete(API, kind, name, ns)
        except Exception as e:  # noqa: BLE001
            fail(e, f"failed to delete {kind}")
        return {"message": f"{kind} {name} deleted"}

    # ------------------------------------------------------------------ ClusterBaseModel
    @r.get("/models")
    def list_models():
        return items("ClusterBaseModel")

    @r.post("/models", status_code=201)
    async def create_model(req: Request):
        data = await body(req)
        token = data.pop("huggingFaceToken", None)
        if token:  # reference k8s/secrets.go: the token becomes a Secret the model-agent reads
            sec = f"{data.get('metadata', {}).get('name', 'model')}-hf-token"
            store.apply({"apiVersion": "v1", "kind": "Secret",
                         "metadata": {"name": sec, "namespace": os.environ.get("POD_NAMESPACE", "ome")},
                         "stringData": {"token": token}})
            data.setdefault("spec", {}).setdefault("storage", {}).setdefault("key", sec)
        return post_obj("ClusterBaseModel", data)

    @r.get("/models/{name}")
    def get_model(name: str):
        return get_obj("ClusterBaseModel", name)

    @r.put("/models/{name}")
    async def update_model(name: str, req: Request):
        return put_obj("ClusterBaseModel", name, await body(req))

    @r.delete("/models/{name}")
    def delete_model(name: str):
        return del_obj("ClusterBaseModel", name)

    @r.get("/models/{name}/status")
    def model_status(name: str):
        return {"status": get_obj("ClusterBaseModel", name).get("status") or {}}

    @r.get("/models/{name}/events")
    def model_events(name: str):
        obj = get_obj("ClusterBaseModel", name)
        evs = sorted(store.events_for(obj) if hasattr(store, "events_for") else [],
                     key=lambda e: e.get("lastTimestamp") or "", reverse=True)
        return {"events": evs, "total": len(evs)}

    @r.get("/models/{name}/progress")
    def model_progress(name: str):
        """Per-node download progress from the model-agent's node ConfigMaps
        (reference handlers/models.go:515-600)."""
        out = []
        want = {f"clusterbasemodel.{name}", f"default.basemodel.{name}"}
        for cm in store.list("v1", "ConfigMap", None, selector="models.ome/basemodel-status=true"):
            node = (cm["metadata"].get("annotations") or {}).get("models.ome.io/node-name", cm["metadata"]["name"])
            for key, raw in (cm.get("data") or {}).items():
                if key not in want:
                    continue
                try:
                    info = json.loads(raw)
                except ValueError:
                    continue
                p = info.get("progress")
                if not p:
                    continue
                total, done = int(p.get("totalBytes") or 0), int(p.get("completedBytes") or 0)
                speed = float(p.get("speedBytesPerSec") or p.get("bytesPerSecond") or 0.0)
                out.append({"node": node, "phase": p.get("phase"), "totalBytes": total, "completedBytes": done,
                            "bytesPerSecond": speed, "remainingTime": (total - done) / speed if speed > 0 else 0.0,
                            "percentage": 100.0 * done / total if total > 0 else 0.0,
                            "totalFiles": p.get("totalFiles"), "completedFiles": p.get("completedFiles")})
        return {"progress": out, "total": len(out)}

    # ------------------------------------------------------------------ namespaces + BaseModel
    @r.get("/namespaces")
    def namespaces():
        names = {o["metadata"]["name"] for o in store.list("v1", "Namespace")}
        for kind in ("BaseModel", "InferenceService", "ServingRuntime"):
            names.update(o["metadata"].get("namespace") for o in store.list(API, kind))
        names.discard(None)
        names.add("default")
        return {"namespaces": sorted(names), "total": len(names)}

    @r.get("/namespaces/{ns}/models")
    def list_basemodels(ns: str):
        return items("BaseModel", ns)

    @r.get("/namespaces/{ns}/models/{name}")
    def get_basemodel(ns: str, name: str):
        return get_obj("BaseModel", name, ns)

    @r.post("/namespaces/{ns}/models", status_code=201)
    async def create_basemodel(ns: str, req: Request):
        return post_obj("BaseModel", await body(req), ns)

    @r.put("/namespaces/{ns}/models/{name}")
    async def update_basemodel(ns: str, name: str, req: Request):
        return put_obj("BaseModel", name, await body(req), ns)

    @r.delete("/namespaces/{ns}/models/{name}")
    def delete_basemodel(ns: str, name: str):
        return del_obj("BaseModel", name, ns)

    # ------------------------------------------------------------------ runtimes
    @r.get("/runtimes")
    def list_runtimes():
        return items("ClusterServingRuntime")

    @r.get("/runtimes/catalog")
    def runtime_catalog():
        have = {o["metadata"]["name"] for o in store.list(API, "ClusterServingRuntime")}
        files = _catalog(roots, have)
        return {"files": files, "total": len(files)}

    @r.get("/runtimes/fetch-yaml")
    def fetch_yaml(path: str):
        p = _sanitize_yaml_path(path, roots)
        if p is None:
            raise HTTPException(400, {"error": "path must be a .yaml file under a catalog root",
                                      "roots": [str(x) for x in roots]})
        docs = [d for d in yaml.safe_load_all(p.read_text()) if isinstance(d, dict)]
        rts = [d for d in docs if d.get("kind") in ("ClusterServingRuntime", "ServingRuntime")]
        if not rts:
            raise HTTPException(422, {"error": "no ServingRuntime in file"})
        return {"runtime": rts[0], "yaml": yaml.safe_dump(rts[0], sort_keys=False)}

    def _model_from_query(req: Request) -> V.BaseModelSpec:
        q = req.query_params
        if q.get("model"):
            try:
                return RI.model_spec_of(store, q["model"], q.get("namespace"))
            except Exception as e:  # noqa: BLE001
                fail(e, "model not found")
        fmt = q.get("modelFormat") or q.get("format")
        if not fmt:
            raise HTTPException(400, {"error": "modelFormat (or model) query parameter is required"})
        return RI.model_spec_from_query(fmt, q.get("modelFramework"), q.get("modelArchitecture"),
                                        q.get("modelSize"), q.get("quantization"), q.get("formatVersion"))

    @r.get("/runtimes/compatible")
    def compatible(req: Request):
        model = _model_from_query(req)
        res = RI.find_compatible(store, model, req.query_params.get("namespace", "default"))
        return {"runtimes": res, "total": len(res)}

    @r.get("/runtimes/recommend")
    def recommend(req: Request):
        model = _model_from_query(req)
        res = RI.recommend(store, model, req.query_params.get("namespace", "default"))
        if res.get("runtime") is None:
            raise HTTPException(404, {"error": "no compatible runtime", "details": res.get("error")})
        return res

    @r.post("/runtimes/validate")
    async def validate_runtime_cfg(req: Request):
        errs, warns = RI.validate_runtime(await body(req))
        return {"valid": not errs, "errors": errs, "warnings": warns}

    @r.get("/runtimes/{name}")
    def get_runtime(name: str):
        return get_obj("ClusterServingRuntime", name)

    @r.get("/runtimes/{name}/compatibility")
    def runtime_compat(name: str, req: Request):
        rt = get_obj("ClusterServingRuntime", name)
        res = RI.evaluate(store, name, V.spec_of(rt), _model_from_query(req))
        return res

    @r.post("/runtimes/{name}/clone", status_code=201)
    async def clone_runtime(name: str, req: Request):
        data = await body(req)
        new = data.get("newName") or data.get("name")
        if not new:
            raise HTTPException(400, {"error": "newName is required"})
        src = get_obj("ClusterServingRuntime", name)
        obj = {"apiVersion": API, "kind": "ClusterServingRuntime",
               "metadata": {"name": new, "labels": dict(src["metadata"].get("labels") or {}),
                            "annotations": {**(src["metadata"].get("annotations") or {}),
                                            "ome.io/cloned-from": name}},
               "spec": json.loads(json.dumps(src.get("spec") or {}))}
        # an exact copy would tie its source on (format, priority) and the ServingRuntime
        # admission webhook rejects that; the clone is staged disabled until it is edited
        obj["spec"]["disabled"] = bool(data.get("disabled", True))
        return post_obj("ClusterServingRuntime", obj)

    @r.post("/runtimes", status_code=201)
    async def create_runtime(req: Request):
        data = await body(req)
        errs, _ = RI.validate_runtime(data)
        if errs:
            raise HTTPException(422, {"error": "invalid runtime", "details": errs})
        return post_obj("ClusterServingRuntime", data)

    @r.put("/runtimes/{name}")
    async def update_runtime(name: str, req: Request):
        return put_obj("ClusterServingRuntime", name, await body(req))

    @r.delete("/runtimes/{name}")
    def delete_runtime(name: str):
        return del_obj("ClusterServingRuntime", name)

    # ------------------------------------------------------------------ InferenceServices
    @r.get("/services")
    def list_services(namespace: str | None = None):
        return items("InferenceService", namespace)

    @r.get("/services/{name}")
    def get_service(name: str, namespace: str = "default"):
        return get_obj("InferenceService", name, namespace)

    @r.post("/services", status_code=201)
    async def create_service(req: Request, namespace: str = "default"):
        data = await body(req)
        ns = data.get("metadata", {}).get("namespace") or namespace
        return post_obj("InferenceService", data, ns)

    @r.put("/services/{name}")
    async def update_service(name: str, req: Request, namespace: str = "default"):
        return put_obj("InferenceService", name, await body(req), namespace)

    @r.delete("/services/{name}")
    def delete_service(name: str, namespace: str = "default"):
        return del_obj("InferenceService", name, namespace)

    @r.get("/services/{name}/status")
    def service_status(name: str, namespace: str = "default"):
        obj = get_obj("InferenceService", name, namespace)
        st = obj.get("status") or {}
        conds = {c.get("type"): c.get("status") for c in st.get("conditions") or []}
        return {"status": st, "ready": conds.get("Ready") == "True", "url": st.get("url")}

    # ------------------------------------------------------------------ accelerators
    @r.get("/accelerators")
    def list_accelerators():
        return items("AcceleratorClass")

    @r.get("/accelerators/{name}")
    def get_accelerator(name: str):
        return get_obj("AcceleratorClass", name)

    # ------------------------------------------------------------------ benchmarks
    @r.get("/benchmarks")
    def list_benchmarks(namespace: str | None = None):
        return items("BenchmarkJob", namespace)

    @r.get("/benchmarks/{name}")
    def get_benchmark(name: str, namespace: str = "default"):
        return get_obj("BenchmarkJob", name, namespace)

    @r.post("/benchmarks", status_code=201)
    async def create_benchmark(req: Request, namespace: str = "default"):
        data = await body(req)
        return post_obj("BenchmarkJob", data, data.get("metadata", {}).get("namespace") or namespace)

    @r.delete("/benchmarks/{name}")
    def delete_benchmark(name: str, namespace: str = "default"):
        return del_obj("BenchmarkJob", name, namespace)

    @r.get("/summary")
    def summary():
        """Dashboard counters: objects per kind and how many are ready."""
        def ready(o):
            st = o.get("status") or {}
            if st.get("state"):
                return st["state"] == "Ready"
            return any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or [])

        out = {}
        for key, kind in (("models", "ClusterBaseModel"), ("namespacedModels", "BaseModel"),
                          ("runtimes", "ClusterServingRuntime"), ("services", "InferenceService"),
                          ("accelerators", "AcceleratorClass"), ("benchmarks", "BenchmarkJob")):
            objs = store.list(API, kind)
            out[key] = {"total": len(objs), "ready": sum(1 for o in objs if ready(o))}
        out["nodes"] = len(store.list("v1", "Node"))
        return out

    # ------------------------------------------------------------------ validation
    @r.post("/validate/yaml")
    async def validate_yaml(req: Request):
        raw = (await req.body()).decode()
        results = []
        try:
            docs = [d for d in yaml.safe_load_all(raw) if d]
        except yaml.YAMLError as e:
            return {"valid": False, "errors": [f"YAML parse error: {e}"], "results": []}
        for d in docs:
            res = {"kind": d.get("kind"), "name": (d.get("metadata") or {}).get("name"), "errors": []}
            if not d.get("kind") or not d.get("apiVersion"):
                res["errors"].append("apiVersion and kind are required")
            else:
                try:  # the admission chain (defaulting + validating webhooks) without persisting
                    store.create(d, dry_run=True)
                except Exception as e:  # noqa: BLE001
                    res["errors"].append(str(e))
            results.append(res)
        return {"valid": all(not x["errors"] for x in results) and bool(results), "results": results,
                "errors": [f"{x['kind']}/{x['name']}: {e}" for x in results for e in x["errors"]]}

    @r.post("/validate/model")
    async def validate_model(req: Request):
        data = await body(req)
        errs = []
        spec = data.get("spec", data)
        try:
            m = V.BaseModelSpec.model_validate(spec)
            if not (m.storage and m.storage.storage_uri):
                errs.append("spec.storage.storageUri is required")
            if m.model_format is None or not m.model_format.name:
                errs.append("spec.modelFormat.name is required")
        except Exception as e:  # noqa: BLE001
            errs.append(str(e))
        return {"valid": not errs, "errors": errs}

    @r.post("/validate/runtime")
    async def validate_runtime(req: Request):
        errs, warns = RI.validate_runtime(await body(req))
        return {"valid": not errs, "errors": errs, "warnings": warns}

    # ------------------------------------------------------------------ Hugging Face (offline)
    @r.get("/huggingface/models/search")
    def hf_search(q: str = "", limit: int = 20, author: str | None = None):
        res = HF.search(q, limit=limit, author=author, store=store, models_root=models_root)
        return {"models": res, "total": len(res)}

    @r.get("/huggingface/models/{org}/{name}/info")
    def hf_info2(org: str, name: str):
        return _hf_info(f"{org}/{name}")

    @r.get("/huggingface/models/{model_id}/info")
    def hf_info(model_id: str):
        return _hf_info(model_id)

    def _hf_info(model_id: str):
        info = HF.info(model_id, models_root=models_root)
        if info is None:
            raise HTTPException(404, {"error": f"model {model_id} not in the local hub cache / models root"})
        return info

    @r.get("/huggingface/models/{org}/{name}/config")
    def hf_config2(org: str, name: str):
        return _hf_config(f"{org}/{name}")

    @r.get("/huggingface/models/{model_id}/config")
    def hf_config(model_id: str):
        return _hf_config(model_id)

    def _hf_config(model_id: str):
        cfg = HF.config(model_id, models_root=models_root)
        if cfg is None:
            raise HTTPException(404, {"error": f"config.json of {model_id} not available offline"})
        return cfg

    # ------------------------------------------------------------------ SSE
    @r.get("/events")
    async def events(req: Request, keepalive: float = 30.0):
        q = bcast.subscribe()

        async def gen():
            try:
                yield 'event: connected\ndata: {"message": "Connected to event stream"}\n\n'
                last = time.monotonic()
                while True:
                    if await req.is_disconnected():
                        break
                    try:
                        msg = q.get_nowait()
                    except queue.Empty:
                        if time.monotonic() - last > keepalive:
                            last = time.monotonic()
                            ts = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
                            yield f'event: ping\ndata: {{"timestamp": "{ts}"}}\n\n'
                        await asyncio.sleep(0.05)
                        continue
                    yield f"event: {msg['type']}\ndata: {json.dumps(msg)}\n\n"
            finally:
                bcast.unsubscribe(q)

        return StreamingResponse(gen(), media_type="text/event-stream",
                                 headers={"Cache-Control": "no-cache", "Connection": "keep-alive"})

    return r


def mount(app, store, prefix: str = "/console", catalog_roots: list[str] | None = None,
          models_root: str | None = None) -> None:
    """Mount the console (API at ``{prefix}/api/v1``, dashboard at ``{prefix}/``) into a FastAPI app."""
    from fastapi.responses import FileResponse, RedirectResponse

    app.include_router(create_router(store, catalog_roots, models_root), prefix=f"{prefix}/api/v1")

    @app.get(f"{prefix}/health")
    def console_health():
        return {"status": "ok", "service": "ome-amd-web-console-api"}

    @app.get(prefix or "/", include_in_schema=False)
    def console_root_redirect():
        return RedirectResponse(f"{prefix}/")

    @app.get(f"{prefix}/", include_in_schema=False)
    def console_index():
        return FileResponse(STATIC / "index.html")

    @app.get(f"{prefix}/static/{{fname}}", include_in_schema=False)
    def console_static(fname: str):
        p = (STATIC / fname).resolve()
        if p.parent != STATIC.resolve() or not p.is_file():
            from fastapi import HTTPException

            raise HTTPException(404)
        return FileResponse(p)


def create_app(store, catalog_roots: list[str] | None = None, models_root: str | None = None, cors: list[str] | None = None):
    """Standalone console server: API at ``/api/v1`` (the reference's paths), dashboard at ``/``."""
    from fastapi import FastAPI
    from fastapi.middleware.cors import CORSMiddleware
    from fastapi.responses import FileResponse

    app = FastAPI(title="ome-amd web console")
    app.add_middleware(CORSMiddleware, allow_origins=cors or ["http://localhost:3000"], allow_credentials=True,
                       allow_methods=["GET", "POST", "PUT", "DELETE", "OPTIONS"],
                       allow_headers=["Origin", "Content-Type", "Authorization"])
    app.include_router(create_router(store, catalog_roots, models_root), prefix="/api/v1")

    @app.get("/health")
    def health():
        return {"status": "ok", "service": "ome-amd-web-console-api"}

    @app.get("/", include_in_schema=False)
    def index():
        return FileResponse(STATIC / "index.html")

    @app.get("/static/{fname}", include_in_schema=False)
    def static(fname: str):
        from fastapi import HTTPException

        p = (STATIC / fname).resolve()
        if p.parent != STATIC.resolve() or not p.is_file():
            raise HTTPException(404)
        return FileResponse(p)

    return app

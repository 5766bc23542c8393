"""Store adapter over a remote ``ome_amd.manager`` REST API, so the console can run as its own
process (the reference console is a separate Deployment talking to the kube-apiserver,
``web-console/backend/internal/k8s/client.go:45-103``).  Implements the subset of
:class:`ome_amd.store.store.Store` the console uses; watches are emulated by polling list
results (resourceVersion diff) on a background thread."""
from __future__ import annotations

import threading

import httpx

from ome_amd.manager import PLURALS
from ome_amd.store import store as S
from ome_amd.store.store import CLUSTER_SCOPED, WatchEvent, group_of

_ERR = {404: S.NotFound, 409: S.Conflict, 422: S.Invalid}


class RemoteStore:
    def __init__(self, base_url: str, poll_s: float = 1.0, timeout: float = 30.0):
        self.base = base_url.rstrip("/")
        self.http = httpx.Client(timeout=timeout)
        self.poll_s = poll_s
        self._watchers: list = []
        self._lock = threading.Lock()
        self._thread: threading.Thread | None = None
        self._stop = threading.Event()

    # ------------------------------------------------------------------ paths
    def _path(self, api_version: str, kind: str, namespace: str | None, name: str | None = None) -> str:
        g, v = (api_version.split("/", 1) if "/" in api_version else ("", api_version))
        plural = PLURALS.get(kind) or kind.lower() + "s"
        root = f"/apis/{g}/{v}" if g else f"/api/{v}"
        scoped = namespace and (g, kind) not in CLUSTER_SCOPED
        p = f"{root}/namespaces/{namespace}/{plural}" if scoped else f"{root}/{plural}"
        return f"{self.base}{p}/{name}" if name else f"{self.base}{p}"

    def _check(self, r: httpx.Response) -> dict:
        body = r.json() if r.content else {}
        if r.status_code >= 400 or (isinstance(body, dict) and body.get("status") == "Failure"):
            code = body.get("code", r.status_code) if isinstance(body, dict) else r.status_code
            raise _ERR.get(code, S.Invalid)(body.get("message", r.text) if isinstance(body, dict) else r.text)
        return body

    # ------------------------------------------------------------------ CRUD
    def list(self, api_version: str, kind: str, namespace: str | None = None, selector=None, **_) -> list[dict]:
        params = {"labelSelector": selector} if isinstance(selector, str) else None
        return self._check(self.http.get(self._path(api_version, kind, namespace), params=params)).get("items", [])

    def get(self, api_version: str, kind: str, name: str, namespace: str | None = None) -> dict:
        return self._check(self.http.get(self._path(api_version, kind, namespace, name)))

    def try_get(self, api_version: str, kind: str, name: str, namespace: str | None = None) -> dict | None:
        try:
            return self.get(api_version, kind, name, namespace)
        except S.NotFound:
            return None

    def create(self, obj: dict, dry_run: bool = False) -> dict:
        m = obj.get("metadata", {})
        params = {"dryRun": "All"} if dry_run else None
        return self._check(self.http.post(self._path(obj["apiVersion"], obj["kind"], m.get("namespace")), json=obj,
                                          params=params))

    def update(self, obj: dict, status_only: bool = False) -> dict:
        m = obj["metadata"]
        url = self._path(obj["apiVersion"], obj["kind"], m.get("namespace"), m["name"])
        return self._check(self.http.put(url + ("/status" if status_only else ""), json=obj))

    def apply(self, obj: dict) -> dict:
        cur = self.try_get(obj["apiVersion"], obj["kind"], obj["metadata"]["name"], obj["metadata"].get("namespace"))
        if cur is None:
            return self.create(obj)
        obj = {**obj, "metadata": {**obj["metadata"], "resourceVersion": cur["metadata"].get("resourceVersion")}}
        return self.update(obj)

    def delete(self, api_version: str, kind: str, name: str, namespace: str | None = None, **_) -> None:
        self._check(self.http.delete(self._path(api_version, kind, namespace, name)))

    def events_for(self, obj: dict) -> list[dict]:
        uid = obj["metadata"].get("uid")
        return [e for e in self.list("v1", "Event") if e.get("involvedObject", {}).get("uid") == uid]

    # ------------------------------------------------------------------ watch (polling)
    def watch(self, callback, kinds=None):
        entry = (set(kinds) if kinds else None, callback)
        with self._lock:
            self._watchers.append(entry)
            if self._thread is None:
                self._thread = threading.Thread(target=self._poll, daemon=True, name="console-remote-watch")
                self._thread.start()
        return entry

    def unwatch(self, entry) -> None:
        with self._lock:
            if entry in self._watchers:
                self._watchers.remove(entry)

    def close(self) -> None:
        self._stop.set()

    def _poll(self) -> None:
        seen: dict[tuple, str] = {}
        first = True
        while not self._stop.is_set():
            with self._lock:
                kinds = set()
                for k, _ in self._watchers:
                    kinds |= k or set()
            now: dict[tuple, dict] = {}
            for kind in sorted(kinds):
                api = "v1" if kind == "Namespace" else "ome.io/v1beta1"
                try:
                    for o in self.list(api, kind):
                        key = (group_of(api), kind, o["metadata"].get("namespace"), o["metadata"]["name"])
                        now[key] = o
                except Exception:  # noqa: BLE001 — manager briefly unreachable: retry next poll
                    continue
            events = []
            if not first:
                for key, o in now.items():
                    rv = o["metadata"].get("resourceVersion", "")
                    if key not in seen:
                        events.append(WatchEvent("ADDED", o))
                    elif seen[key] != rv:
                        events.append(WatchEvent("MODIFIED", o))
                for key in set(seen) - set(now):
                    events.append(WatchEvent("DELETED", {"kind": key[1], "metadata": {"namespace": key[2],
                                                                                       "name": key[3]}}))
            seen = {k: o["metadata"].get("resourceVersion", "") for k, o in now.items()}
            first = False
            with self._lock:
                ws = list(self._watchers)
            for ev in events:
                for ks, cb in ws:
                    if ks is None or ev.obj.get("kind") in ks:
                        try:
                            cb(ev)
                        except Exception:  # noqa: BLE001
                            pass
            self._stop.wait(self.poll_s)

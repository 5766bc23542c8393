"""KubeStore / KubeClient against a local fake API server (list, watch streams with resourceVersion
resume, create / replace / status subresource / merge patch / delete with finalizers, 409s), then
the model agent + BaseModel controller reconciling THROUGH the adapter, and the AdmissionReview
webhook handler."""
import base64
import copy
import json
import os
import sys
import threading
import time
import urllib.parse
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd.api import constants as C  # noqa: E402
from ome_amd.store import kube as K  # noqa: E402
from ome_amd.store.store import Conflict, NotFound, merge_patch  # noqa: E402

API = C.API_VERSION
NODE = "n0"


class FakeAPIServer:
    """Resources keyed by (collection path without namespace, namespace, name)."""

    def __init__(self, token="sekret"):
        self.objs: dict[tuple[str, str, str], dict] = {}
        self.log: list[tuple[int, str, str, str, dict]] = []   # (rv, type, coll, ns, obj)
        self.rv = 100
        self.cv = threading.Condition()
        self.token = token
        fake = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _json(self, code, body):
                raw = json.dumps(body).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(raw)))
                self.end_headers()
                self.wfile.write(raw)

            def _parse(self):
                u = urllib.parse.urlsplit(self.path)
                q = dict(urllib.parse.parse_qsl(u.query))
                seg = [s for s in u.path.split("/") if s]
                # /api/v1/... or /apis/g/v/...
                base = seg[:2] if seg[0] == "api" else seg[:3]
                rest = seg[len(base):]
                ns = ""
                if rest and rest[0] == "namespaces" and len(rest) >= 3:
                    ns, rest = rest[1], rest[2:]
                coll = "/".join(base + rest[:1]) if rest else "/".join(base)
                name = rest[1] if len(rest) > 1 else ""
                sub = rest[2] if len(rest) > 2 else ""
                return coll, ns, name, sub, q, len(rest) == 0

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n)) if n else {}

            def handle_one(self):
                if self.headers.get("Authorization") != f"Bearer {fake.token}":
                    return self._json(401, {"message": "unauthorized"})
                coll, ns, name, sub, q, discovery = self._parse()
                if discovery:
                    return self._json(200, {"resources": [{"name": "widgets", "kind": "Widget", "namespaced": True}]})
                m = self.command
                with fake.cv:
                    if m == "GET" and not name and q.get("watch"):
                        return self._watch(coll, ns, int(q.get("resourceVersion") or 0),
                                           float(q.get("timeoutSeconds", 5)))
                    if m == "GET" and not name:
                        items = [copy.deepcopy(o) for (c, n_, _), o in sorted(fake.objs.items())
                                 if c == coll and (not ns or n_ == ns)]
                        return self._json(200, {"kind": "List", "metadata": {"resourceVersion": str(fake.rv)},
                                                "items": items})
                    key = (coll, ns, name)
                    cur = fake.objs.get(key)
                    if m == "POST":
                        o = self._body()
                        key = (coll, ns, o["metadata"]["name"])
                        if key in fake.objs:
                            return self._json(409, {"message": f"{o['metadata']['name']} already exists"})
                        o["metadata"].update(uid=str(uuid.uuid4()), creationTimestamp="2026-01-01T00:00:00Z")
                        return self._json(201, fake.put(key, o, "ADDED"))
                    if cur is None:
                        return self._json(404, {"message": "not found"})
                    if m == "GET":
                        return self._json(200, cur)
                    if m == "PUT":
                        o = self._body()
                        if o["metadata"].get("resourceVersion") != cur["metadata"]["resourceVersion"]:
                            return self._json(409, {"message": "the object has been modified"})
                        if sub == "status":
                            new = copy.deepcopy(cur)
                            new["status"] = o.get("status")
                        else:
                            new = copy.deepcopy(o)
                            if "status" in cur:
                                new["status"] = cur["status"]
                            new["metadata"]["uid"] = cur["metadata"]["uid"]
                            if cur["metadata"].get("deletionTimestamp"):
                                new["metadata"]["deletionTimestamp"] = cur["metadata"]["deletionTimestamp"]
                        if new["metadata"].get("deletionTimestamp") and not new["metadata"].get("finalizers"):
                            fake.drop(key)
                            return self._json(200, new)
                        return self._json(200, fake.put(key, new, "MODIFIED"))
                    if m == "PATCH":
                        new = merge_patch(cur, self._body())
                        return self._json(200, fake.put(key, new, "MODIFIED"))
                    if m == "DELETE":
                        if cur["metadata"].get("finalizers"):
                            new = copy.deepcopy(cur)
                            new["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:01Z"
                            return self._json(200, fake.put(key, new, "MODIFIED"))
                        fake.drop(key)
                        return self._json(200, {"kind": "Status", "status": "Success"})
                return self._json(405, {"message": "no"})

            def _watch(self, coll, ns, rv, timeout):
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()
                end = time.time() + timeout
                while time.time() < end:
                    evs = [e for e in fake.log if e[0] > rv and e[2] == coll and (not ns or e[3] == ns)]
                    for e in evs:
                        line = (json.dumps({"type": e[1], "object": e[4]}) + "\n").encode()
                        self.wfile.write(f"{len(line):x}\r\n".encode() + line + b"\r\n")
                        rv = e[0]
                    self.wfile.flush()
                    fake.cv.wait(timeout=0.1)
                self.wfile.write(b"0\r\n\r\n")

            do_GET = do_POST = do_PUT = do_PATCH = do_DELETE = handle_one

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def put(self, key, o, typ):
        self.rv += 1
        o["metadata"]["resourceVersion"] = str(self.rv)
        self.objs[key] = o
        self.log.append((self.rv, typ, key[0], key[1], copy.deepcopy(o)))
        self.cv.notify_all()
        return copy.deepcopy(o)

    def drop(self, key):
        o = self.objs.pop(key)
        self.rv += 1
        self.log.append((self.rv, "DELETED", key[0], key[1], copy.deepcopy(o)))
        self.cv.notify_all()

    def external(self, coll, ns, obj):      # kubectl apply from outside
        obj["metadata"].setdefault("uid", str(uuid.uuid4()))
        with self.cv:
            return self.put((coll, ns, obj["metadata"]["name"]), obj, "ADDED")

    def close(self):
        self.srv.shutdown()


@pytest.fixture
def api():
    f = FakeAPIServer()
    yield f
    f.close()


def _wait(pred, t=5.0):
    end = time.time() + t
    while time.time() < end:
        if pred():
            return True
        time.sleep(0.02)
    return False


KINDS = [("v1", "Node"), ("v1", "ConfigMap"), ("v1", "Namespace"), (API, "ClusterBaseModel")]


def _client(api):
    return K.KubeClient(api.url, token="sekret")


def test_list_watch_and_writes(api):
    api.external("api/v1/nodes", "", {"apiVersion": "v1", "kind": "Node", "metadata": {"name": NODE}})
    st = K.KubeStore(_client(api), KINDS)
    try:
        assert st.get("v1", "Node", NODE)["metadata"]["resourceVersion"]
        seen = []
        st.watch(lambda ev: seen.append((ev.type, ev.obj["metadata"]["name"])), ["ConfigMap"])
        cm = st.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c1", "namespace": "ome"},
                        "data": {"a": "1"}})
        assert ("api/v1/configmaps", "ome", "c1") in api.objs and cm["metadata"]["resourceVersion"]
        # an object created outside the manager arrives through the watch stream
        api.external("api/v1/configmaps", "ome", {"apiVersion": "v1", "kind": "ConfigMap",
                                                  "metadata": {"name": "c2", "namespace": "ome"}, "data": {}})
        assert _wait(lambda: st.try_get("v1", "ConfigMap", "c2", "ome") is not None)
        assert ("ADDED", "c1") in seen and _wait(lambda: ("ADDED", "c2") in seen)
        assert seen.count(("ADDED", "c1")) == 1        # our own write is not re-announced by the watch
        # optimistic concurrency: a stale resourceVersion is a Conflict
        stale = copy.deepcopy(cm)
        cm["data"]["a"] = "2"
        st.update(cm)
        stale["data"]["a"] = "3"
        with pytest.raises(Conflict):
            st.update(stale)
        assert api.objs[("api/v1/configmaps", "ome", "c1")]["data"]["a"] == "2"
        st.patch("v1", "ConfigMap", "c1", {"data": {"b": "x"}}, "ome")
        assert st.get("v1", "ConfigMap", "c1", "ome")["data"] == {"a": "2", "b": "x"}
        st.delete("v1", "ConfigMap", "c2", "ome")
        assert st.try_get("v1", "ConfigMap", "c2", "ome") is None and ("api/v1/configmaps", "ome", "c2") not in api.objs
        with pytest.raises(NotFound):
            st.delete("v1", "ConfigMap", "c2", "ome")
    finally:
        st.close()


def test_status_subresource_and_finalizer_delete(api):
    st = K.KubeStore(_client(api), KINDS)
    try:
        o = st.create({"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "m"},
                       "spec": {"storage": {"storageUri": "random://tiny-llama"}}})
        o["status"] = {"state": "Ready"}
        st.update_status(o)
        assert api.objs[("apis/ome.io/v1beta1/clusterbasemodels", "", "m")]["status"] == {"state": "Ready"}
        o = st.add_finalizer(st.get(API, "ClusterBaseModel", "m"), "x/f")
        st.delete(API, "ClusterBaseModel", "m")
        cur = st.get(API, "ClusterBaseModel", "m")
        assert cur["metadata"]["deletionTimestamp"]
        st.remove_finalizer(cur, "x/f")
        assert st.try_get(API, "ClusterBaseModel", "m") is None
        assert ("apis/ome.io/v1beta1/clusterbasemodels", "", "m") not in api.objs
    finally:
        st.close()


def test_agent_and_basemodel_controller_through_the_adapter(api, tmp_path):
    from ome_amd.controllers import basemodel
    from ome_amd.modelagent.agent import DOWNLOAD, ModelAgent, Task

    api.external("api/v1/nodes", "", {"apiVersion": "v1", "kind": "Node", "metadata": {"name": NODE}})
    api.external("apis/ome.io/v1beta1/clusterbasemodels", "",
                 {"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "tiny"},
                  "spec": {"storage": {"storageUri": "random://tiny-llama", "path": str(tmp_path / "tiny")}}})
    st = K.KubeStore(_client(api), KINDS)
    try:
        ctrl = basemodel.setup(st, cluster=True)
        ag = ModelAgent(st, NODE, models_root=str(tmp_path / "models"))
        ag.gopher.process(Task(DOWNLOAD, st.get(API, "ClusterBaseModel", "tiny")))
        cm = api.objs[("api/v1/configmaps", C.OME_NAMESPACE, NODE)]
        assert json.loads(cm["data"][C.model_configmap_key(None, "tiny", True)])["status"] == "Ready"
        ctrl.reconciler.reconcile(("", "tiny"))
        remote = api.objs[("apis/ome.io/v1beta1/clusterbasemodels", "", "tiny")]
        assert remote["status"]["state"] == "Ready" and remote["status"]["nodesReady"] == [NODE]
        assert C.CLUSTERBASEMODEL_FINALIZER in remote["metadata"]["finalizers"]
        assert remote["spec"].get("modelArchitecture") == "LlamaForCausalLM"
        node = api.objs[("api/v1/nodes", "", NODE)]
        assert node["metadata"]["labels"][C.model_label(None, "tiny", True)] == "Ready"
    finally:
        st.close()


def test_discovery_for_unknown_kinds_and_kubeconfig(api, tmp_path):
    c = _client(api)
    assert c.resource("example.com/v1", "Widget") == ("widgets", True)
    assert c.path("example.com/v1", "Widget", "ns1", "w") == "/apis/example.com/v1/namespaces/ns1/widgets/w"
    assert c.path("v1", "Node", None, "n") == "/api/v1/nodes/n"
    kc = tmp_path / "kubeconfig"
    kc.write_text(json.dumps({"current-context": "c", "contexts": [{"name": "c", "context": {"cluster": "k",
                                                                                              "user": "u"}}],
                              "clusters": [{"name": "k", "cluster": {"server": api.url}}],
                              "users": [{"name": "u", "user": {"token": "sekret"}}]}))
    c2 = K.KubeClient.from_kubeconfig(str(kc))
    assert c2.server == api.url and c2.token == "sekret"
    st = K.KubeStore(c2, [("v1", "Node")], start_watches=False)
    assert st.list("v1", "Node") == []


def test_admission_review_mutates_and_denies():
    from ome_amd.admission import webhooks
    from ome_amd.store.store import Store

    s = Store()
    webhooks.install(s)
    s.create({"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "llama"},
              "spec": {"storage": {"storageUri": "random://tiny-llama"}}})
    isvc = {"apiVersion": API, "kind": "InferenceService", "metadata": {"name": "x", "namespace": "default"},
            "spec": {"model": {"name": "llama"}}}
    out = K.admission_review(s, {"request": {"uid": "u1", "operation": "CREATE", "object": isvc}})
    r = out["response"]
    assert r["uid"] == "u1" and r["allowed"]
    if "patch" in r:
        ops = json.loads(base64.b64decode(r["patch"]))
        assert all(op["op"] in ("add", "replace", "remove") for op in ops)
    bad = {"apiVersion": API, "kind": "InferenceService", "metadata": {"name": "y", "namespace": "default"},
           "spec": {"model": {"name": "missing"}}}
    out = K.admission_review(s, {"request": {"uid": "u2", "operation": "CREATE", "object": bad}})
    assert out["response"]["allowed"] is False and out["response"]["status"]["message"]


def test_manager_bootstraps_cluster_objects_and_serves_admission(api, tmp_path):
    from fastapi.testclient import TestClient

    from ome_amd.manager import Cluster, create_api

    st = K.KubeStore(_client(api), KINDS)
    try:
        cl = Cluster(str(tmp_path / "state"), store=st, with_agent=False, with_executor=False)
        assert ("api/v1/namespaces", "", C.OME_NAMESPACE) in api.objs
        assert ("api/v1/configmaps", C.OME_NAMESPACE, C.INFERENCESERVICE_CONFIGMAP) in api.objs
        app = TestClient(create_api(cl))
        review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                  "request": {"uid": "r1", "operation": "CREATE",
                              "object": {"apiVersion": API, "kind": "InferenceService",
                                         "metadata": {"name": "z", "namespace": "default"},
                                         "spec": {"model": {"name": "nope"}}}}}
        r = app.post("/admission", json=review).json()
        assert r["response"]["uid"] == "r1" and r["response"]["allowed"] is False
        # the hooks see the cluster's models through the informer cache
        api.external("apis/ome.io/v1beta1/clusterbasemodels", "",
                     {"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "nope"},
                      "spec": {"storage": {"storageUri": "random://tiny-llama"}}})
        assert _wait(lambda: st.try_get(API, "ClusterBaseModel", "nope") is not None)
        r = app.post("/admission", json=review).json()
        assert r["response"]["allowed"] is True
    finally:
        st.close()

"""Web console backend (H8): the reference console's route table (web-console/backend/internal/
api/server.go:56-156) served over an in-process store; runtime recommendations must agree with
the controller's RuntimeSelector; SSE stream delivers store changes."""
import json
import threading
import time

import pytest
import yaml
from fastapi.testclient import TestClient

from ome_amd.console import create_app
from ome_amd.manager import Cluster, create_api

RT = """
apiVersion: ome.io/v1beta1
kind: ClusterServingRuntime
metadata: {name: ome-amd-llama}
spec:
  supportedModelFormats:
  - {name: safetensors, modelFormat: {name: safetensors, version: "1"}, modelArchitecture: LlamaForCausalLM,
     autoSelect: true, priority: 2}
  modelSizeRange: {min: 1B, max: 80B}
  protocolVersions: [openAI]
  engineConfig:
    runner: {name: ome-container, image: ome-amd:latest}
---
apiVersion: ome.io/v1beta1
kind: ClusterServingRuntime
metadata: {name: ome-amd-qwen}
spec:
  supportedModelFormats:
  - {name: safetensors, modelFormat: {name: safetensors, version: "1"}, modelArchitecture: Qwen2ForCausalLM,
     autoSelect: true, priority: 1}
  protocolVersions: [openAI]
  engineConfig:
    runner: {name: ome-container, image: ome-amd:latest}
---
apiVersion: ome.io/v1beta1
kind: AcceleratorClass
metadata: {name: amd-mi355x}
spec: {vendor: amd, family: cdna4, model: mi355x, capabilities: {memoryGB: 288Gi}}
"""


@pytest.fixture()
def cl(tmp_path):
    c = Cluster(str(tmp_path), with_agent=False, with_executor=False)
    c.apply(RT)
    c.start()
    yield c
    c.shutdown()


@pytest.fixture()
def client(cl):
    return TestClient(create_app(cl.store))


def _model(name="llama-3-8b", arch="LlamaForCausalLM"):
    return {"metadata": {"name": name}, "spec": {"modelFormat": {"name": "safetensors", "version": "1"},
                                                  "modelArchitecture": arch, "modelParameterSize": "8B",
                                                  "storage": {"storageUri": f"hf://meta-llama/{name}"}}}


def test_health_and_static(client):
    assert client.get("/health").json()["status"] == "ok"
    assert "<title>" in client.get("/").text


def test_model_crud_and_status(client, cl):
    r = client.post("/api/v1/models", json=_model())
    assert r.status_code == 201, r.text
    assert client.get("/api/v1/models").json()["total"] == 1
    m = client.get("/api/v1/models/llama-3-8b").json()
    m["spec"]["modelParameterSize"] = "8.03B"
    assert client.put("/api/v1/models/llama-3-8b", json=m).status_code == 200
    assert client.get("/api/v1/models/llama-3-8b").json()["spec"]["modelParameterSize"] == "8.03B"
    assert "status" in client.get("/api/v1/models/llama-3-8b/status").json()
    assert client.get("/api/v1/models/missing").status_code == 404
    assert client.delete("/api/v1/models/llama-3-8b").status_code == 200


def test_progress_from_node_configmap(client, cl):
    client.post("/api/v1/models", json=_model())
    cl.store.create({"apiVersion": "v1", "kind": "ConfigMap",
                     "metadata": {"name": "node-a", "namespace": "ome", "labels": {"models.ome/basemodel-status": "true"}},
                     "data": {"clusterbasemodel.llama-3-8b": json.dumps(
                         {"name": "llama-3-8b", "status": "Updating",
                          "progress": {"phase": "Downloading", "totalBytes": 1000, "completedBytes": 250,
                                       "speedBytesPerSec": 50.0}})}})
    p = client.get("/api/v1/models/llama-3-8b/progress").json()
    assert p["total"] == 1
    e = p["progress"][0]
    assert e["node"] == "node-a" and e["percentage"] == 25.0 and e["remainingTime"] == 15.0


def test_namespaced_basemodels_and_namespaces(client):
    r = client.post("/api/v1/namespaces/team-a/models", json=_model("qwen"))
    assert r.status_code == 201, r.text
    assert client.get("/api/v1/namespaces/team-a/models").json()["total"] == 1
    assert "team-a" in client.get("/api/v1/namespaces").json()["namespaces"]
    assert client.delete("/api/v1/namespaces/team-a/models/qwen").status_code == 200


def test_runtime_intelligence_matches_selector(client, cl):
    from ome_amd.api import v1beta1 as V
    from ome_amd.policy.runtime_selector import RuntimeSelector

    res = client.get("/api/v1/runtimes/compatible",
                     params={"modelFormat": "safetensors", "modelArchitecture": "LlamaForCausalLM",
                             "modelSize": "8B", "formatVersion": "1"}).json()
    names = [m["runtime"] for m in res["runtimes"]]
    # reference semantics: a runtime format pinned to another architecture is not a match
    assert names == ["ome-amd-llama"]
    rec = client.get("/api/v1/runtimes/recommend",
                     params={"modelFormat": "safetensors", "modelArchitecture": "LlamaForCausalLM", "modelSize": "8B",
                             "formatVersion": "1"}).json()
    spec = V.BaseModelSpec.model_validate(_model()["spec"])
    assert rec["runtime"] == RuntimeSelector(cl.store).select(spec, None, "default").name
    # an architecture only the other runtime accepts
    rec2 = client.get("/api/v1/runtimes/recommend", params={"modelFormat": "safetensors", "formatVersion": "1",
                                                            "modelArchitecture": "Qwen2ForCausalLM"}).json()
    assert rec2["runtime"] == "ome-amd-qwen"
    # by stored model name
    client.post("/api/v1/models", json=_model())
    assert client.get("/api/v1/runtimes/recommend", params={"model": "llama-3-8b"}).json()["runtime"] == "ome-amd-llama"
    c = client.get("/api/v1/runtimes/ome-amd-llama/compatibility",
                   params={"modelFormat": "safetensors", "modelArchitecture": "MistralForCausalLM",
                           "formatVersion": "1"}).json()
    assert c["compatible"] is False and c["warnings"]
    assert client.get("/api/v1/runtimes/recommend", params={"modelFormat": "onnx"}).status_code == 404


def test_runtime_validate_clone_create(client):
    v = client.post("/api/v1/runtimes/validate", json={"spec": {"containers": [{"name": "x"}]}}).json()
    assert not v["valid"] and any("image" in e for e in v["errors"])
    assert client.post("/api/v1/runtimes/ome-amd-llama/clone", json={"newName": "copy"}).status_code == 201
    cp = client.get("/api/v1/runtimes/copy").json()
    assert cp["metadata"]["annotations"]["ome.io/cloned-from"] == "ome-amd-llama" and cp["spec"]["disabled"]
    bad = client.post("/api/v1/runtimes", json={"metadata": {"name": "bad"}, "spec": {}})
    assert bad.status_code == 422


def test_fetch_yaml_is_sandboxed(client, tmp_path):
    ok = client.get("/api/v1/runtimes/fetch-yaml", params={"path": "config/runtimes/ome-amd-runtimes.yaml"})
    assert ok.status_code == 200 and ok.json()["runtime"]["kind"] in ("ClusterServingRuntime", "ServingRuntime")
    assert client.get("/api/v1/runtimes/fetch-yaml", params={"path": "/etc/passwd"}).status_code == 400


def test_services_and_accelerators(client):
    client.post("/api/v1/models", json=_model())
    isvc = {"metadata": {"name": "llama", "namespace": "default"}, "spec": {"model": {"name": "llama-3-8b"}}}
    r = client.post("/api/v1/services", json=isvc)
    assert r.status_code == 201, r.text
    assert client.get("/api/v1/services").json()["total"] == 1
    st = client.get("/api/v1/services/llama/status").json()
    assert "ready" in st
    assert client.get("/api/v1/accelerators").json()["total"] == 1
    assert client.get("/api/v1/accelerators/amd-mi355x").json()["spec"]["vendor"] == "amd"
    assert client.delete("/api/v1/services/llama").status_code == 200


def test_validate_yaml_uses_admission(client):
    good = yaml.safe_dump({"apiVersion": "ome.io/v1beta1", "kind": "ClusterBaseModel", "metadata": {"name": "m"},
                           "spec": _model()["spec"]})
    r = client.post("/api/v1/validate/yaml", content=good, headers={"content-type": "application/yaml"}).json()
    assert r["valid"], r
    assert client.get("/api/v1/models").json()["total"] == 0  # dry run: nothing persisted
    bad = client.post("/api/v1/validate/yaml", content="kind: [", headers={"content-type": "application/yaml"}).json()
    assert not bad["valid"]
    m = client.post("/api/v1/validate/model", json={"spec": {"modelFormat": {"name": "safetensors"}}}).json()
    assert not m["valid"] and any("storageUri" in e for e in m["errors"])


def test_hf_offline_lookup(client, tmp_path, monkeypatch):
    snap = tmp_path / "hub" / "models--meta-llama--Llama-3.1-8B" / "snapshots" / "abc"
    snap.mkdir(parents=True)
    (snap / "config.json").write_text(json.dumps({"architectures": ["LlamaForCausalLM"], "model_type": "llama"}))
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "hub"))
    s = client.get("/api/v1/huggingface/models/search", params={"q": "llama"}).json()
    assert s["models"][0]["id"] == "meta-llama/Llama-3.1-8B" and "llama" in s["models"][0]["tags"]
    assert client.get("/api/v1/huggingface/models/meta-llama/Llama-3.1-8B/config").json()["model_type"] == "llama"
    info = client.get("/api/v1/huggingface/models/meta-llama/Llama-3.1-8B/info").json()
    assert {"rfilename": "config.json"} in info["siblings"]
    assert client.get("/api/v1/huggingface/models/nobody/none/info").status_code == 404


def test_sse_broadcast(cl):
    from ome_amd.console.api import EventBroadcaster

    b = EventBroadcaster(cl.store)
    q = b.subscribe()
    cl.store.create({"apiVersion": "ome.io/v1beta1", "kind": "ClusterBaseModel", **_model("sse-model")})
    msg = q.get(timeout=5)
    assert msg["type"] == "add" and msg["resource"] == "models" and msg["name"] == "sse-model"
    b.unsubscribe(q)
    b.close()


def test_console_mounted_in_manager(cl):
    c = TestClient(create_api(cl))
    assert c.get("/console/health").json()["status"] == "ok"
    assert "<title>" in c.get("/console/").text
    assert c.get("/console/api/v1/runtimes").json()["total"] == 2
    # the manager's own k8s-style routes are untouched
    assert c.get("/apis/ome.io/v1beta1/clusterservingruntimes").json()["kind"] == "ClusterServingRuntimeList"


def test_remote_store_console(cl):
    """Standalone console over a manager's REST API (RemoteStore)."""
    import socket

    import uvicorn

    from ome_amd.console.remote import RemoteStore

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = uvicorn.Server(uvicorn.Config(create_api(cl), host="127.0.0.1", port=port, log_level="error"))
    t = threading.Thread(target=srv.run, daemon=True)
    t.start()
    for _ in range(100):
        if srv.started:
            break
        time.sleep(0.05)
    rs = RemoteStore(f"http://127.0.0.1:{port}", poll_s=0.1)
    try:
        c = TestClient(create_app(rs))
        assert c.post("/api/v1/models", json=_model()).status_code == 201
        assert cl.store.try_get("ome.io/v1beta1", "ClusterBaseModel", "llama-3-8b") is not None
        assert c.get("/api/v1/runtimes/recommend", params={"model": "llama-3-8b"}).json()["runtime"] == "ome-amd-llama"
        assert c.get("/api/v1/models/nope").status_code == 404
    finally:
        rs.close()
        srv.should_exit = True
        t.join(timeout=5)


def test_spa_assets_summary_and_benchmarks(client, cl):
    """The multi-page console: shell + app.js + style.css served; dashboard counters and the
    benchmark-job routes the views call."""
    assert 'src="static/app.js"' in client.get("/").text
    js = client.get("/static/app.js")
    assert js.status_code == 200 and "ServiceDeploy" in js.text and "ROUTES" in js.text
    assert client.get("/static/style.css").status_code == 200
    assert client.get("/static/../api.py").status_code == 404
    s = client.get("/api/v1/summary").json()
    assert set(s) >= {"models", "runtimes", "services", "accelerators", "benchmarks", "nodes"}
    bj = """apiVersion: ome.io/v1beta1
kind: BenchmarkJob
metadata: {name: b1, namespace: default}
spec:
  endpoint: {endpoint: {url: "http://127.0.0.1:1/v1", apiFormat: openai, modelName: m}}
  task: text-to-text
  trafficScenarios: ["D(100,100)"]
  numConcurrency: [1]
  maxTimePerIteration: 1
  maxRequestsPerIteration: 1
  outputLocation: {storageUri: "local:///tmp/ome-bench-results"}
"""
    r = client.post("/api/v1/benchmarks", content=bj, headers={"Content-Type": "application/yaml"})
    assert r.status_code == 201, r.text
    assert client.get("/api/v1/benchmarks").json()["total"] == 1
    assert client.get("/api/v1/benchmarks/b1").json()["spec"]["task"] == "text-to-text"
    assert client.delete("/api/v1/benchmarks/b1").status_code == 200

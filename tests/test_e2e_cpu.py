"""Milestone A end-to-end on CPU: ClusterBaseModel + ClusterServingRuntime + InferenceService
reconcile to Ready through the model agent, the controllers and the local node executor, which
runs the real ``ome_amd.runtime.server`` (tiny random Llama, --device cpu) as a supervised
process behind a Service proxy; then a BenchmarkJob drives it with the load generator."""
import json
import os
import time
import urllib.request

import pytest

from ome_amd.api import constants as C
from ome_amd.executor.dns import resolve_url
from ome_amd.manager import Cluster

API = C.API_VERSION


def _runtime(name="tiny-cpu-rt"):
    return {
        "apiVersion": API, "kind": "ClusterServingRuntime", "metadata": {"name": name},
        "spec": {
            "supportedModelFormats": [{"modelFormat": {"name": "safetensors", "version": "1.0.0"},
                                       "modelFramework": {"name": "transformers", "version": "4.46.0"},
                                       "modelArchitecture": "LlamaForCausalLM", "autoSelect": True, "priority": 1}],
            "protocolVersions": ["openAI"], "modelSizeRange": {"min": "100K", "max": "50M"},
            "engineConfig": {"runner": {
                "name": "ome-container", "image": "docker.io/lmsysorg/sglang:v0.5",
                "ports": [{"containerPort": 8080, "name": "http1"}],
                # reference-style sglang command: the executor maps it onto ome_amd.runtime.server
                "command": ["python3", "-m", "sglang.launch_server", "--host", "0.0.0.0", "--port", "8080",
                            "--model-path", "$(MODEL_PATH)", "--served-model-name", "tiny", "--device", "cpu",
                            "--context-length", "512", "--max-running-requests", "8", "--enable-metrics"],
                "readinessProbe": {"httpGet": {"path": "/health", "port": 8080}, "periodSeconds": 1},
                "startupProbe": {"httpGet": {"path": "/health_generate", "port": 8080}, "periodSeconds": 1,
                                 "failureThreshold": 240, "timeoutSeconds": 30},
                "livenessProbe": {"httpGet": {"path": "/health", "port": 8080}, "periodSeconds": 5,
                                  "failureThreshold": 5, "timeoutSeconds": 10},
            }},
        }}


def _model(tmp, name="tiny-llama"):
    return {"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": name},
            "spec": {"vendor": "meta", "storage": {"storageUri": "random://tiny-llama",
                                                   "path": str(tmp / "models" / name)}}}


def _isvc(name="tiny"):
    return {"apiVersion": API, "kind": "InferenceService", "metadata": {"name": name, "namespace": "default"},
            "spec": {"model": {"name": "tiny-llama"}, "engine": {"minReplicas": 1, "maxReplicas": 1}}}


def _ready(obj):
    return any(c.get("type") == "Ready" and c.get("status") == "True"
               for c in (obj.get("status") or {}).get("conditions") or [])


def test_control_plane_simulated(tmp_path):
    """Fake-kubelet mode: the whole object graph converges without launching processes."""
    cl = Cluster(str(tmp_path / "state"), simulate=True, gpus=8)
    try:
        cl.load_catalog(os.path.join(os.path.dirname(__file__), "..", "config", "acceleratorclasses"))
        cl.apply([_runtime(), _model(tmp_path)])
        cl.agent.start()
        cl.step(3)
        cl.apply([_isvc()])  # admission needs the parsed model format to pick a runtime
        cl.step(6)
        bm = cl.store.get(API, "ClusterBaseModel", "tiny-llama")
        assert bm["status"]["state"] == "Ready", bm.get("status")
        assert bm["spec"]["modelArchitecture"] == "LlamaForCausalLM"
        node = cl.store.get("v1", "Node", "mi355x-node-0")
        assert node["metadata"]["labels"][C.model_label(None, "tiny-llama", True)] == "Ready"
        isvc = cl.store.get(API, "InferenceService", "tiny", "default")
        assert _ready(isvc), isvc.get("status")
        dep = cl.store.get("apps/v1", "Deployment", "tiny-engine", "default")
        assert dep["status"]["readyReplicas"] == 1
        pods = cl.store.list("v1", "Pod", "default")
        assert pods and pods[0]["spec"]["nodeName"] == "mi355x-node-0"
        ac = cl.store.get(API, "AcceleratorClass", "amd-mi355x")
        assert "mi355x-node-0" in json.dumps(ac.get("status") or {})
    finally:
        cl.shutdown()


def test_gpu_scheduling_and_lws_env(tmp_path):
    """GPU bookkeeping (HIP_VISIBLE_DEVICES blocks) and LeaderWorkerSet env contract."""
    cl = Cluster(str(tmp_path / "state"), simulate=True, gpus=8, with_agent=False)
    try:
        tmpl = {"metadata": {"labels": {"app": "x"}}, "spec": {"containers": [{
            "name": "c", "image": "i", "resources": {"limits": {"amd.com/gpu": 4}}}]}}
        cl.apply([{"apiVersion": "leaderworkerset.x-k8s.io/v1", "kind": "LeaderWorkerSet",
                   "metadata": {"name": "mn", "namespace": "default"},
                   "spec": {"replicas": 1, "leaderWorkerTemplate": {"size": 2, "leaderTemplate": tmpl,
                                                                   "workerTemplate": tmpl}}}])
        cl.step(4)
        pods = {p["metadata"]["name"]: p for p in cl.store.list("v1", "Pod", "default")}
        assert set(pods) == {"mn-0", "mn-0-1"}
        ids = sorted(pods[n]["metadata"]["annotations"]["ome.io/gpu-ids"] for n in pods)
        assert ids == ["0,1,2,3", "4,5,6,7"]
        env = {e["name"]: e["value"] for e in pods["mn-0-1"]["spec"]["containers"][0]["env"]}
        assert env["LWS_WORKER_INDEX"] == "1" and env["LWS_GROUP_SIZE"] == "2"
        lws = cl.store.get("leaderworkerset.x-k8s.io/v1", "LeaderWorkerSet", "mn", "default")
        assert lws["status"]["readyReplicas"] == 1
        # a third 4-GPU pod cannot be scheduled
        cl.apply([{"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "extra", "namespace": "default"},
                   "spec": tmpl["spec"]}])
        cl.step(2)
        p = cl.store.get("v1", "Pod", "extra", "default")
        assert "Insufficient amd.com/gpu" in p["status"]["conditions"][0]["message"]
    finally:
        cl.shutdown()


@pytest.mark.timeout(600)
def test_isvc_serves_and_benchmarks_on_cpu(tmp_path):
    cl = Cluster(str(tmp_path / "state"), gpus=0, probe_scale=1.0)
    try:
        cl.apply([_runtime(), _model(tmp_path)])
        cl.start()
        assert cl.wait_for(lambda: (cl.store.get(API, "ClusterBaseModel", "tiny-llama").get("status") or {})
                           .get("state") == "Ready", timeout=60)
        cl.apply([_isvc()])
        ok = cl.wait_for(lambda: _ready(cl.store.get(API, "InferenceService", "tiny", "default")), timeout=240)
        if not ok:
            pods = cl.store.list("v1", "Pod", "default")
            logs = {p["metadata"]["name"]: cl.executor.kubelet.logs("default", p["metadata"]["name"])[-3000:]
                    for p in pods}
            pytest.fail(f"ISVC not ready: {cl.store.get(API, 'InferenceService', 'tiny', 'default').get('status')}"
                        f"\npods={[p.get('status') for p in pods]}\nlogs={logs}")
        isvc = cl.store.get(API, "InferenceService", "tiny", "default")
        url = isvc["status"]["url"]
        os.environ["OME_LOCAL_DNS"] = cl.executor.kubelet.proxies.dns_path
        base = resolve_url(url)
        assert base.startswith("http://127.0.0.1:")
        req = urllib.request.Request(base + "/v1/completions", data=json.dumps(
            {"model": "tiny", "prompt": "hello", "max_tokens": 4, "temperature": 0, "ignore_eos": True}).encode(),
            headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=60) as r:
            out = json.loads(r.read())
        assert out["usage"]["completion_tokens"] == 4

        results = tmp_path / "bench"
        cl.apply([{"apiVersion": API, "kind": "BenchmarkJob", "metadata": {"name": "bj", "namespace": "default"},
                   "spec": {"endpoint": {"inferenceService": {"name": "tiny", "namespace": "default"}},
                            "task": "text-to-text", "trafficScenarios": ["D(16,8)"], "numConcurrency": [1, 2],
                            "maxTimePerIteration": 1, "maxRequestsPerIteration": 4,
                            "resultFolderName": "exp1",
                            "outputLocation": {"storageUri": f"local://{results}"}}}])
        done = cl.wait_for(lambda: (cl.store.get(API, "BenchmarkJob", "bj", "default").get("status") or {})
                           .get("state") in ("Completed", "Failed"), timeout=240)
        bj = cl.store.get(API, "BenchmarkJob", "bj", "default")
        logs = cl.executor.kubelet.logs("default", "bj-0")
        assert done and bj["status"]["state"] == "Completed", f"{bj.get('status')}\n{logs[-3000:]}"
        summary = json.loads((results / "exp1" / "summary.json").read_text())
        assert [s["concurrency"] for s in summary] == [1, 2]
        assert all(s["num_completed"] == 4 and s["output_tokens"]["mean"] == 8 for s in summary)
        # deleting the ISVC tears down its pods (ownerRef GC + process termination)
        cl.store.delete(API, "InferenceService", "tiny", "default")
        gone = cl.wait_for(lambda: not [p for p in cl.store.list("v1", "Pod", "default")
                                        if p["metadata"]["name"].startswith("tiny-engine")], timeout=60)
        assert gone
    finally:
        cl.shutdown()


@pytest.mark.timeout(600)
def test_baseline_config1_opt125m_on_cpu_runtime(tmp_path):
    """BASELINE.json config 1: BaseModel + InferenceService reconcile for OPT-125m on the CPU
    runtime.  The ISVC names no runtime: the model agent parses the (random-init) OPT-125m
    config -- architecture, 125M parameters -- and the RuntimeSelector picks the CPU runtime by
    ``modelArchitecture: OPTForCausalLM`` and its size range; the executor runs the real server,
    which serves a completion through the OPT decoder (learned positions, ReLU MLP)."""
    rt = _runtime("opt-cpu-rt")
    fmt = rt["spec"]["supportedModelFormats"][0]
    fmt["modelArchitecture"] = "OPTForCausalLM"
    rt["spec"]["modelSizeRange"] = {"min": "100M", "max": "200M"}
    cmd = rt["spec"]["engineConfig"]["runner"]["command"]
    cmd[cmd.index("tiny")] = "opt"
    bm = {"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "opt-125m"},
          "spec": {"vendor": "facebook", "storage": {"storageUri": "random://opt-125m",
                                                     "path": str(tmp_path / "models" / "opt-125m")}}}
    isvc = {"apiVersion": API, "kind": "InferenceService", "metadata": {"name": "opt", "namespace": "default"},
            "spec": {"model": {"name": "opt-125m"}, "engine": {"minReplicas": 1, "maxReplicas": 1}}}
    cl = Cluster(str(tmp_path / "state"), gpus=0, probe_scale=1.0)
    try:
        cl.apply([_runtime(), rt, bm])
        cl.start()
        assert cl.wait_for(lambda: (cl.store.get(API, "ClusterBaseModel", "opt-125m").get("status") or {})
                           .get("state") == "Ready", timeout=60)
        spec = cl.store.get(API, "ClusterBaseModel", "opt-125m")["spec"]
        assert spec.get("modelArchitecture") == "OPTForCausalLM" and spec.get("modelParameterSize") == "125.24M"
        cl.apply([isvc])
        ok = cl.wait_for(lambda: _ready(cl.store.get(API, "InferenceService", "opt", "default")), timeout=300)
        got = cl.store.get(API, "InferenceService", "opt", "default")
        assert ok, got.get("status")
        dep = cl.store.get("apps/v1", "Deployment", "opt-engine", "default")
        assert dep["metadata"]["labels"].get(C.SERVING_RUNTIME_LABEL, dep["metadata"]["labels"].get(
            "serving-runtime")) == "opt-cpu-rt"
        os.environ["OME_LOCAL_DNS"] = cl.executor.kubelet.proxies.dns_path
        base = resolve_url(got["status"]["url"])
        req = urllib.request.Request(base + "/v1/completions", data=json.dumps(
            {"model": "opt", "prompt": "hello world", "max_tokens": 5, "temperature": 0, "ignore_eos": True}).encode(),
            headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            out = json.loads(r.read())
        assert out["usage"]["completion_tokens"] == 5
    finally:
        cl.shutdown()

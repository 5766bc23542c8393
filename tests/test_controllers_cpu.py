"""InferenceService controller object generation per deployment mode (the reference's
fake-client reconciler tests: ``controller_test.go`` "engine only", "engine and decoder
(PD-disaggregated)", "Multi-node engine deployment" asserting exactly one LWS, components and
reconcilers tests), status propagation, ingress / external service, autoscalers, cleanup, and
the BaseModel / AcceleratorClass / BenchmarkJob controllers.  No executor, no processes."""
import json

import pytest

from ome_amd.api import constants as C
from ome_amd.manager import Cluster

API = C.API_VERSION
RUNNER = {"name": "ome-container", "image": "sglang:v0.5", "command": ["python3", "-m", "sglang.launch_server"],
          "args": ["--port=8080", "--tp-size=1", "--model-path=$(MODEL_PATH)"],
          "ports": [{"containerPort": 8080, "name": "http1"}], "resources": {"limits": {"amd.com/gpu": "1"}}}


def _rt(name="rt", **extra):
    return {"apiVersion": API, "kind": "ClusterServingRuntime", "metadata": {"name": name},
            "spec": {"protocolVersions": ["openAI"], "modelSizeRange": {"min": "1B", "max": "10B"},
                     "supportedModelFormats": [{"name": "safetensors",
                                                "modelFormat": {"name": "safetensors", "version": "1.0.0"},
                                                "modelFramework": {"name": "transformers", "version": "4.46.0"},
                                                "modelArchitecture": "LlamaForCausalLM", "autoSelect": True,
                                                "priority": 1}], **extra}}


def _isvc(name="svc", ann=None, **spec):
    return {"apiVersion": API, "kind": "InferenceService",
            "metadata": {"name": name, "namespace": "default", "annotations": dict(ann or {})},
            "spec": {"model": {"name": "llama"}, **spec}}


@pytest.fixture
def cl(tmp_path):
    c = Cluster(str(tmp_path), with_agent=False, with_executor=False)
    c.apply([{"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "llama"},
              "spec": {"modelFormat": {"name": "safetensors", "version": "1.0.0"},
                       "modelFramework": {"name": "transformers", "version": "4.46.0"},
                       "modelArchitecture": "LlamaForCausalLM", "modelParameterSize": "8B",
                       "storage": {"storageUri": "hf://meta-llama/Meta-Llama-3-8B-Instruct",
                                   "path": "/raid/models/llama"}}}])
    yield c
    c.shutdown()


def _kinds(cl, ns="default"):
    return sorted((o["kind"], o["metadata"]["name"]) for o in cl.store.all()
                  if o["metadata"].get("namespace") == ns and o["kind"] not in ("Event", "InferenceService"))


def _cond(obj, t):
    return next((c for c in (obj.get("status") or {}).get("conditions") or [] if c["type"] == t), None)


def _mark_available(cl, api, kind, name):
    o = cl.store.get(api, kind, name, "default")
    o["status"] = {"replicas": 1, "readyReplicas": 1, "availableReplicas": 1, "updatedReplicas": 1,
                   "observedGeneration": o["metadata"].get("generation", 1),
                   "conditions": [{"type": "Available", "status": "True", "reason": "MinimumReplicasAvailable"}]}
    cl.store.update_status(o)


def test_raw_engine_only(cl):
    cl.apply([_rt(engineConfig={"runner": RUNNER})])
    cl.apply([_isvc(engine={"minReplicas": 1, "maxReplicas": 2})])
    cl.step(3)
    assert _kinds(cl) == [("ConfigMap", "modelconfig-svc"), ("Deployment", "svc-engine"),
                          ("HorizontalPodAutoscaler", "svc-engine"), ("Service", "svc"), ("Service", "svc-engine")]
    d = cl.store.get("apps/v1", "Deployment", "svc-engine", "default")
    assert d["metadata"]["ownerReferences"][0]["kind"] == "InferenceService"
    sp = d["spec"]
    assert sp["strategy"]["rollingUpdate"] == {"maxUnavailable": 0, "maxSurge": 1}
    assert sp["revisionHistoryLimit"] == 10 and sp["progressDeadlineSeconds"] == 600
    pod = sp["template"]["spec"]
    c = pod["containers"][0]
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["MODEL_PATH"] == "/raid/models/llama" and env["PARALLELISM_SIZE"] == "1"
    assert c["readinessProbe"]["tcpSocket"]["port"] == 8080  # default TCP readiness probe
    assert pod["nodeSelector"] == {"models.ome.io/clusterbasemodel.llama": "Ready"}
    assert {"name": "llama", "hostPath": {"path": "/raid/models/llama"}} in pod["volumes"]
    labels = sp["template"]["metadata"]["labels"]
    assert labels[C.ISVC_LABEL] == "svc" and labels["component"] == "engine"
    hpa = cl.store.get("autoscaling/v2", "HorizontalPodAutoscaler", "svc-engine", "default")["spec"]
    assert (hpa["minReplicas"], hpa["maxReplicas"]) == (1, 2)
    models = json.loads(cl.store.get("v1", "ConfigMap", "modelconfig-svc", "default")["data"]["models.json"])
    assert models[0]["modelName"] == "llama"
    isvc = cl.store.get(API, "InferenceService", "svc", "default")
    assert isvc["status"]["url"] == "http://svc.default.svc.cluster.local:8080"
    assert _cond(isvc, "Ready")["status"] == "Unknown"
    # the Deployment becomes Available -> EngineReady / Ready
    _mark_available(cl, "apps/v1", "Deployment", "svc-engine")
    cl.step(2)
    isvc = cl.store.get(API, "InferenceService", "svc", "default")
    assert _cond(isvc, "EngineReady")["status"] == "True" and _cond(isvc, "Ready")["status"] == "True"


def test_isvc_runner_args_replace_runtime_args(cl):
    """Strategic merge of the engine spec replaces list fields (reference ``MergeEngineSpec``)."""
    cl.apply([_rt(engineConfig={"runner": RUNNER})])
    cl.apply([_isvc(engine={"runner": {"args": ["--tp-size=8", "--enable-metrics"]}})])
    cl.step(3)
    c = cl.store.get("apps/v1", "Deployment", "svc-engine", "default")["spec"]["template"]["spec"]["containers"][0]
    assert c["args"] == ["--tp-size=8", "--enable-metrics"]
    assert c["image"] == "sglang:v0.5" and c["command"] == RUNNER["command"]


def test_accelerator_config_args_and_tp_override(cl):
    """``acceleratorConfig[<class>]``: runtimeArgsOverride merged by key, TP/PP rewritten in place,
    resources from the AcceleratorClass (reference ``components/base.go:258-306``)."""
    cl.load_catalog(__file__.rsplit("/tests/", 1)[0] + "/config/acceleratorclasses")
    rt = _rt(engineConfig={"runner": RUNNER}, acceleratorRequirements={"acceleratorClasses": ["amd-mi355x"]})
    rt["spec"]["supportedModelFormats"][0]["acceleratorConfig"] = {
        "amd-mi355x": {"runtimeArgsOverride": ["--mem-frac=0.85", "--port=8080"],
                       "tensorParallelismOverride": {"tensorParallelSize": 8}}}
    cl.apply([rt])
    cl.apply([_isvc(engine={}, acceleratorSelector={"acceleratorClass": "amd-mi355x"})])
    cl.step(3)
    c = cl.store.get("apps/v1", "Deployment", "svc-engine", "default")["spec"]["template"]["spec"]["containers"][0]
    assert c["args"] == ["--port=8080", "--tp-size=8", "--model-path=$(MODEL_PATH)", "--mem-frac=0.85"]
    isvc = cl.store.get(API, "InferenceService", "svc", "default")
    sa = isvc["status"]["components"]["engine"]["selectedAccelerator"]
    assert sa["acceleratorClass"] == "amd-mi355x" and sa["reason"] == "explicit"


def test_pd_disaggregated(cl):
    cl.apply([_rt(engineConfig={"runner": RUNNER}, decoderConfig={"runner": RUNNER},
                  routerConfig={"runner": {**RUNNER, "name": "router"}})])
    cl.apply([_isvc(engine={}, decoder={}, router={})])
    cl.step(3)
    kinds = _kinds(cl)
    for k in [("Deployment", "svc-engine"), ("Deployment", "svc-decoder"), ("Deployment", "svc-router"),
              ("ServiceAccount", "svc-router"), ("Role", "svc-router"), ("RoleBinding", "svc-router"),
              ("Service", "svc")]:
        assert k in kinds, k
    role = cl.store.get("rbac.authorization.k8s.io/v1", "Role", "svc-router", "default")
    assert set(role["rules"][0]["verbs"]) >= {"get", "list", "watch"}
    ext = cl.store.get("v1", "Service", "svc", "default")
    assert ext["spec"]["selector"] == {"app": "svc-router"}  # router is the entrypoint
    isvc = cl.store.get(API, "InferenceService", "svc", "default")
    assert isvc["metadata"]["annotations"][C.DEPLOYMENT_MODE] == C.DeploymentMode.PD


def test_multinode_single_lws(cl):
    cl.apply([_rt(engineConfig={"leader": {"runner": RUNNER}, "worker": {"size": 1, "runner": RUNNER}})])
    cl.apply([_isvc(engine={"leader": {}, "worker": {"size": 1}})])
    cl.step(3)
    lws = [o for o in cl.store.all() if o["kind"] == "LeaderWorkerSet"]
    assert len(lws) == 1 and lws[0]["metadata"]["name"] == "lws-svc-engine"
    t = lws[0]["spec"]["leaderWorkerTemplate"]
    assert t["size"] == 2 and t["restartPolicy"] == "RecreateGroupOnPodRestart"
    assert lws[0]["spec"]["networkConfig"]["subdomainPolicy"] == "Shared"
    assert not [o for o in cl.store.all() if o["kind"] == "Deployment"]


def test_serverless_knative(cl):
    cl.apply([_rt(engineConfig={"runner": RUNNER})])
    cl.apply([_isvc(ann={C.DEPLOYMENT_MODE: C.DeploymentMode.SERVERLESS}, engine={"minReplicas": 0})])
    cl.step(3)
    ks = [o for o in cl.store.all() if o["kind"] == "Service" and o["apiVersion"].startswith("serving.knative.dev")]
    assert len(ks) == 1
    ann = ks[0]["spec"]["template"]["metadata"]["annotations"]
    assert ann.get("autoscaling.knative.dev/min-scale") == "0"


def test_keda_scaled_object(cl):
    cl.apply([_rt(engineConfig={"runner": RUNNER})])
    cl.apply([_isvc(ann={C.AUTOSCALER_CLASS: C.AUTOSCALER_KEDA}, engine={"minReplicas": 1, "maxReplicas": 4},
                    kedaConfig={"promServerAddress": "http://prom:9090", "customPromQuery": "sum(rate(x[1m]))",
                                "scalingThreshold": "10", "scalingOperator": "GreaterThan"})])
    cl.step(3)
    so = [o for o in cl.store.all() if o["kind"] == "ScaledObject"]
    assert len(so) == 1
    trig = so[0]["spec"]["triggers"][0]
    assert trig["type"] == "prometheus" and trig["metadata"]["serverAddress"] == "http://prom:9090"
    assert trig["metadata"]["query"] == "sum(rate(x[1m]))" and trig["metadata"]["threshold"] == "10"
    assert not [o for o in cl.store.all() if o["kind"] == "HorizontalPodAutoscaler"]


def test_ingress_when_enabled(cl):
    cm = cl.store.get("v1", "ConfigMap", C.INFERENCESERVICE_CONFIGMAP, C.OME_NAMESPACE)
    cm["data"]["ingress"] = json.dumps({"disableIngressCreation": False, "ingressDomain": "example.com"})
    cl.store.update(cm)
    cl.apply([_rt(engineConfig={"runner": RUNNER})])
    cl.apply([_isvc(engine={})])
    cl.step(3)
    ing = cl.store.get("networking.k8s.io/v1", "Ingress", "svc", "default")
    rule = ing["spec"]["rules"][0]
    assert rule["host"] == "svc.default.example.com"
    assert rule["http"]["paths"][0]["backend"]["service"]["name"] == "svc-engine"
    assert cl.store.try_get("v1", "Service", "svc", "default") is None  # no external service with ingress


def test_delete_cleans_up(cl):
    cl.apply([_rt(engineConfig={"runner": RUNNER})])
    cl.apply([_isvc(engine={})])
    cl.step(3)
    assert _kinds(cl)
    cl.store.delete(API, "InferenceService", "svc", "default")
    cl.step(3)
    assert _kinds(cl) == []


def test_ray_vllm_mode(cl):
    cl.apply([_rt(engineConfig={"leader": {"runner": RUNNER}, "worker": {"size": 1, "runner": RUNNER}})])
    cl.apply([_isvc(ann={C.DEPLOYMENT_MODE: C.DeploymentMode.MULTINODE_RAY_VLLM},
                    engine={"minReplicas": 2, "leader": {}, "worker": {"size": 1}})])
    cl.step(3)
    rcs = sorted(o["metadata"]["name"] for o in cl.store.all() if o["kind"] == "RayCluster")
    assert len(rcs) == 2
    probers = [o for o in cl.store.all() if o["kind"] == "Deployment" and o["metadata"]["name"].endswith("-mnp")]
    assert len(probers) == 2


def test_accelerator_class_status(cl):
    cl.apply([{"apiVersion": "v1", "kind": "Node",
               "metadata": {"name": "n0", "labels": {"amd.com/gpu.product-name": "AMD_Instinct_MI355X"}},
               "status": {"capacity": {"amd.com/gpu": "8"}, "allocatable": {"amd.com/gpu": "6"},
                          "conditions": [{"type": "Ready", "status": "True"}]}},
              {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n1", "labels": {"other": "gpu"}},
               "status": {"capacity": {"nvidia.com/gpu": "8"}, "conditions": [{"type": "Ready", "status": "True"}]}}])
    cl.load_catalog(__file__.rsplit("/tests/", 1)[0] + "/config/acceleratorclasses")
    cl.step(2)
    st = cl.store.get(API, "AcceleratorClass", "amd-mi355x")["status"]
    assert st["nodes"] == ["n0"] and st["availableNodes"] == 1
    assert st["totalAccelerators"] == 8 and st["availableAccelerators"] == 6
    # a node going NotReady drops out of the available count
    n0 = cl.store.get("v1", "Node", "n0")
    n0["status"]["conditions"] = [{"type": "Ready", "status": "False"}]
    cl.store.update_status(n0)
    cl.step(2)
    assert cl.store.get(API, "AcceleratorClass", "amd-mi355x")["status"]["availableNodes"] == 0


def test_benchmark_job_builds_job(cl):
    cl.apply([_rt(engineConfig={"runner": RUNNER})])
    cl.apply([_isvc(engine={})])
    cl.step(2)
    bj = {"apiVersion": API, "kind": "BenchmarkJob", "metadata": {"name": "bj", "namespace": "default"},
               "spec": {"task": "text-to-text", "endpoint": {"inferenceService": {"name": "svc", "namespace": "default"}},
                        "trafficScenarios": ["D(100,100)"], "numConcurrency": [1, 4], "maxTimePerIteration": 1,
                        "maxRequestsPerIteration": 10, "outputLocation": {"storageUri": "local:///tmp/bench-out"}}}
    cl.apply([bj])
    cl.step(2)
    assert not [o for o in cl.store.all() if o["kind"] == "Job"]  # waits for the ISVC to be Ready
    _mark_available(cl, "apps/v1", "Deployment", "svc-engine")
    cl.step(3)
    jobs = [o for o in cl.store.all() if o["kind"] == "Job"]
    assert len(jobs) == 1
    c = jobs[0]["spec"]["template"]["spec"]["containers"][0]
    cmd = " ".join(c.get("command", []) + c.get("args", []))
    assert "D(100,100)" in cmd and "svc" in cmd and "--experiment-base-dir /tmp/bench-out" in cmd
    assert jobs[0]["metadata"]["ownerReferences"][0]["kind"] == "BenchmarkJob"

"""Admission webhooks (``pkg/webhook/admission/{isvc,servingruntime,benchmark,pod}``): defaulting,
validation and the pod mutator's injector chain, exercised through the store's admission hooks
exactly as the manager wires them."""
import json

import pytest

from ome_amd.admission import webhooks as W
from ome_amd.api import constants as C
from ome_amd.bench import scenarios as SC
from ome_amd.store.store import Invalid, Store

API = C.API_VERSION


def _store():
    s = Store()
    W.install(s)
    s.create({"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "llama"},
              "spec": {"modelFormat": {"name": "safetensors", "version": "1.0.0"},
                       "modelFramework": {"name": "transformers", "version": "4.46.0"},
                       "modelArchitecture": "LlamaForCausalLM", "modelParameterSize": "8B",
                       "storage": {"storageUri": "hf://meta-llama/Meta-Llama-3-8B-Instruct"}}})
    s.create(_runtime("rt-a"))
    return s


def _runtime(name, priority=1, fmt="safetensors", proto=("openAI",), **extra):
    return {"apiVersion": API, "kind": "ClusterServingRuntime", "metadata": {"name": name},
            "spec": {"protocolVersions": list(proto), "modelSizeRange": {"min": "1B", "max": "10B"},
                     "supportedModelFormats": [{"name": fmt, "modelFormat": {"name": fmt, "version": "1.0.0"},
                                                "modelFramework": {"name": "transformers", "version": "4.46.0"},
                                                "modelArchitecture": "LlamaForCausalLM", "autoSelect": True,
                                                "priority": priority}], **extra}}


def _isvc(name="svc", ann=None, **spec):
    return {"apiVersion": API, "kind": "InferenceService",
            "metadata": {"name": name, "namespace": "default", "annotations": dict(ann or {})},
            "spec": {"model": {"name": "llama"}, **spec}}


# ------------------------------------------------------------------ ISVC defaulting
def test_isvc_defaults_modes_and_replicas():
    s = _store()
    raw = s.create(_isvc("raw", engine={}))
    assert raw["metadata"]["annotations"][C.DEPLOYMENT_MODE] == C.DeploymentMode.RAW
    assert raw["spec"]["engine"]["minReplicas"] == 1 and raw["spec"]["engine"]["maxReplicas"] == 3
    pd = s.create(_isvc("pd", engine={}, decoder={}, router={}))
    assert pd["metadata"]["annotations"][C.DEPLOYMENT_MODE] == C.DeploymentMode.PD
    assert pd["spec"]["router"]["maxReplicas"] == 2
    mn = s.create(_isvc("mn", engine={"leader": {}, "worker": {"size": 1}}))
    assert mn["metadata"]["annotations"][C.DEPLOYMENT_MODE] == C.DeploymentMode.MULTINODE
    explicit = s.create(_isvc("ex", ann={C.DEPLOYMENT_MODE: C.DeploymentMode.SERVERLESS}, engine={"minReplicas": 0}))
    assert explicit["metadata"]["annotations"][C.DEPLOYMENT_MODE] == C.DeploymentMode.SERVERLESS
    assert explicit["spec"]["engine"]["minReplicas"] == 0
    legacy = s.create({**_isvc("legacy"), "spec": {"predictor": {"model": {"baseModel": "llama"}}}})
    assert legacy["metadata"]["annotations"][C.DEPRECATION_WARNING].startswith("The Predictor field is deprecated")


# ------------------------------------------------------------------ ISVC validation
@pytest.mark.parametrize("obj,msg", [
    (_isvc("Bad_Name", engine={}), "invalid InferenceService name"),
    (_isvc(ann={C.AUTOSCALER_CLASS: "magic"}, engine={}), "not a supported autoscaler class"),
    (_isvc(ann={C.TARGET_UTILIZATION: "150"}, engine={}), "[1-100]"),
    (_isvc(ann={C.TARGET_UTILIZATION: "x"}, engine={}), "[1-100]"),
    (_isvc(decoder={}), "decoder cannot be specified without engine"),
    ({**_isvc(engine={}), "spec": {"model": {"name": "ghost"}, "engine": {}}}, "not found"),
    (_isvc(ann={C.AUTOSCALER_CLASS: C.AUTOSCALER_KEDA}, engine={}, kedaConfig={"scalingOperator": "Around"}),
     "invalid KEDA scaling operator"),
    (_isvc(engine={}, kedaConfig={"scalingThreshold": "lots"}), "invalid KEDA scaling threshold"),
    (_isvc(engine={}, kedaConfig={"promServerAddress": "ftp://prom"}), "scheme must be http"),
    (_isvc(engine={}, kedaConfig={"authModes": "bearer"}), "requires authenticationRef"),
    (_isvc(engine={}, runtime={"name": "missing-rt"}), "does not support model"),
])
def test_isvc_validation_rejects(obj, msg):
    with pytest.raises(Invalid) as e:
        _store().create(obj)
    assert msg in str(e.value)


def test_isvc_runtime_selection_at_admission():
    s = _store()
    s.create(_isvc("ok", engine={}))  # auto-selects rt-a
    s.create(_isvc("pinned", engine={}, runtime={"name": "rt-a"}))
    # a full runner lets an engine through without any matching runtime
    s.delete(API, "ClusterServingRuntime", "rt-a")
    with pytest.raises(Invalid, match="no supporting runtime"):
        s.create(_isvc("none", engine={}))
    s.create(_isvc("own", engine={"runner": {"name": "ome-container", "image": "img"}}))


# ------------------------------------------------------------------ ServingRuntime validation
def test_runtime_priority_rules():
    s = _store()
    with pytest.raises(Invalid, match="same priority"):
        s.create(_runtime("rt-b"))  # same format, same protocol, same size range, same priority
    s.create(_runtime("rt-c", priority=2))
    s.create(_runtime("rt-d", proto=("grpc",)))  # different protocol: no clash
    bad = _runtime("rt-e", priority=3)
    bad["spec"]["supportedModelFormats"].append({**bad["spec"]["supportedModelFormats"][0], "priority": 4,
                                                 "modelArchitecture": "MistralForCausalLM"})
    with pytest.raises(Invalid, match="different priorities"):
        s.create(bad)
    s.create(_runtime("rt-off", disabled=True))  # disabled runtimes skip validation


def test_runtime_worker_and_accelerator_rules():
    s = _store()
    with pytest.raises(Invalid, match="workers.size > 0"):
        s.create(_runtime("mn", priority=5, engineConfig={}, workers={"size": 0}))
    with pytest.raises(Invalid, match="AcceleratorClasses do not exist"):
        s.create(_runtime("acc", priority=6, acceleratorRequirements={"acceleratorClasses": ["amd-mi355x"]}))
    s.create({"apiVersion": API, "kind": "AcceleratorClass", "metadata": {"name": "amd-mi355x"}, "spec": {}})
    s.create(_runtime("acc", priority=6, acceleratorRequirements={"acceleratorClasses": ["amd-mi355x"]}))


# ------------------------------------------------------------------ BenchmarkJob
def _bj(**spec):
    base = {"task": "text-to-text", "endpoint": {"inferenceService": {"name": "svc", "namespace": "default"}}}
    return {"apiVersion": API, "kind": "BenchmarkJob", "metadata": {"name": "bj", "namespace": "default"},
            "spec": {**base, **spec}}


def test_benchmark_defaults():
    bj = _store().create(_bj())
    sp = bj["spec"]
    assert sp["trafficScenarios"] == SC.DEFAULT_SCENARIOS["text-to-text"]
    assert sp["numConcurrency"] == SC.DEFAULT_CONCURRENCY
    assert sp["maxTimePerIteration"] == 15 and sp["maxRequestsPerIteration"] == 100


@pytest.mark.parametrize("spec,msg", [
    ({"endpoint": {}}, "endpoint or InferenceService must be specified"),
    ({"endpoint": {"endpoint": {"url": "http://x"}, "inferenceService": {"name": "a"}}}, "cannot be specified together"),
    ({"task": "text-to-music"}, "unsupported task"),
    ({"trafficScenarios": ["N(480,240)/(300,150)", "X(1,2)"]}, "failed to validate scenario"),
    ({"trafficScenarios": ["E(64)"]}, "failed to validate scenario"),
    ({"additionalRequestParams": {"temperature": "warm"}}, "invalid temperature"),
    ({"additionalRequestParams": {"ignore_eos": "yes"}}, "ignore_eos"),
    ({"outputLocation": {"storageUri": ""}}, "storageUri cannot be empty"),
    ({"outputLocation": {"storageUri": "nosuch://x"}}, "error parsing storage URI"),
])
def test_benchmark_validation(spec, msg):
    with pytest.raises(Invalid, match=msg.replace("(", r"\(").replace(")", r"\)")):
        _store().create(_bj(**spec))


@pytest.mark.parametrize("task,s,ok", [
    ("text-to-text", "D(100,100)", True), ("text-to-text", "N(480,240)/(300,150)", True),
    ("text-to-text", "U(50,100)/(50,100)", True), ("text-to-text", "U(50,100)", True),
    ("text-to-text", "D(100)", False), ("text-to-embeddings", "E(1024)", True), ("text-to-embeddings", "D(1,1)", False),
    ("image-text-to-text", "I(512,512)", True), ("unknown", "D(1,1)", False),
])
def test_scenario_grammar(task, s, ok):
    assert SC.validate(s, task) == ok


# ------------------------------------------------------------------ Pod mutator
def _pod(ann=None, gpus=8):
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": "p", "namespace": "default", "labels": {C.ISVC_LABEL: "svc"},
                         "annotations": dict(ann or {})},
            "spec": {"containers": [{"name": C.MAIN_CONTAINER, "image": "img",
                                     "env": [{"name": C.MODEL_PATH_ENV, "value": "/raid/models/llama"}],
                                     "resources": {"limits": {"amd.com/gpu": str(gpus)}}}]}}


def test_pod_injectors_chain_and_order():
    s = _store()
    ann = {C.MODEL_INIT_INJECTION: "true", C.BASE_MODEL_NAME_ANN: "llama", C.FT_ADAPTER_INJECTION: "ft-a",
           C.SERVING_SIDECAR_INJECTION: "true", C.RDMA_AUTO_INJECT: "true"}
    p = s.create(_pod(ann))
    inits = [c["name"] for c in p["spec"]["initContainers"]]
    assert inits == [C.MODEL_INIT_CONTAINER, C.FT_ADAPTER_CONTAINER]
    mi = p["spec"]["initContainers"][0]
    env = {e["name"]: e["value"] for e in mi["env"]}
    assert env["LOCAL_PATH"] == "/raid/models/llama" and env["GPU_COUNT"] == "8" and env["MODEL_NAME"] == "llama"
    names = [c["name"] for c in p["spec"]["containers"]]
    assert C.SERVING_SIDECAR_CONTAINER in names
    main = p["spec"]["containers"][0]
    menv = {e["name"]: e["value"] for e in main["env"]}
    assert menv["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and "NCCL_MIN_NCHANNELS" in menv  # amd-xgmi profile
    assert {"name": "dshm", "mountPath": "/dev/shm"} in main["volumeMounts"]
    assert "IPC_LOCK" in main["securityContext"]["capabilities"]["add"]


def test_pod_mutator_skips_unlabelled_and_rejects_unknown_profile():
    s = _store()
    plain = _pod()
    plain["metadata"]["labels"] = {}
    out = s.create(plain)
    assert "initContainers" not in out["spec"]
    with pytest.raises(Invalid, match="unknown RDMA profile"):
        s.create({**_pod({C.RDMA_AUTO_INJECT: "true", C.RDMA_PROFILE: "nvlink-9000"}),
                  "metadata": {"name": "q", "namespace": "default", "labels": {C.ISVC_LABEL: "svc"},
                               "annotations": {C.RDMA_AUTO_INJECT: "true", C.RDMA_PROFILE: "nvlink-9000"}}})


def test_metrics_aggregator_sidecar():
    s = _store()
    s.create({"apiVersion": "v1", "kind": "ConfigMap",
              "metadata": {"name": C.INFERENCESERVICE_CONFIGMAP, "namespace": C.OME_NAMESPACE},
              "data": {"metricsAggregator": json.dumps({"enableMetricAggregation": "true",
                                                        "enablePrometheusScraping": "true"})}})
    p = s.create(_pod())
    agg = [c for c in p["spec"]["containers"] if c["name"] == "metrics-aggregator"]
    assert agg and p["metadata"]["annotations"][C.PROMETHEUS_SCRAPE] == "true"
    assert p["metadata"]["annotations"][C.PROMETHEUS_PORT] == "9088"

"""Admission case tables (the reference's ``webhook/admission/isvc/inference_service_validation_test.go``,
``servingruntime_webhook_test.go`` and ``benchmark`` webhook cases): InferenceService name /
autoscaler / utilisation / KEDA / decoder / runner / model-reference rules, ServingRuntime priority
and worker-size rules, BenchmarkJob endpoint / scenario / parameter / storage rules."""
import copy

import pytest

from ome_amd.admission.webhooks import has_full_runner, validate_benchmark, validate_isvc, validate_runtime
from ome_amd.api import constants as C
from ome_amd.store.store import Invalid, Store

API = C.API_VERSION


def _isvc(name="my-isvc", ann=None, spec=None, ns="default"):
    return {"apiVersion": API, "kind": "InferenceService",
            "metadata": {"name": name, "namespace": ns, "annotations": dict(ann or {})}, "spec": spec or {}}


def _store_with_model(disabled=False, ns_model=None, runtimes=True):
    s = Store()
    m = {"vendor": "meta", "modelFormat": {"name": "safetensors", "version": "1.0.0"},
         "modelFramework": {"name": "transformers", "version": "4.46.0"}, "modelArchitecture": "LlamaForCausalLM",
         "modelParameterSize": "8B", "storage": {"storageUri": "hf://meta-llama/x"}}
    if disabled:
        m["disabled"] = True
    if ns_model:
        s.create({"apiVersion": API, "kind": "BaseModel", "metadata": {"name": "ns-model", "namespace": ns_model},
                  "spec": copy.deepcopy(m)})
    s.create({"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": "llama"}, "spec": m})
    if runtimes:
        s.create({"apiVersion": API, "kind": "ClusterServingRuntime", "metadata": {"name": "rt"},
                  "spec": {"supportedModelFormats": [{"modelFormat": {"name": "safetensors", "version": "1.0.0"},
                                                      "modelFramework": {"name": "transformers", "version": "4.46.0"},
                                                      "modelArchitecture": "LlamaForCausalLM", "autoSelect": True,
                                                      "priority": 1}],
                           "protocolVersions": ["openAI"], "modelSizeRange": {"min": "1B", "max": "10B"},
                           "engineConfig": {"runner": {"name": "ome-container", "image": "x"}}}})
    return s


def _check(obj, store, err):
    if err is None:
        validate_isvc("CREATE", obj, None, store)
    else:
        with pytest.raises(Invalid, match=err):
            validate_isvc("CREATE", obj, None, store)


# ------------------------------------------------------------------ names / annotations
@pytest.mark.parametrize("name,err", [
    ("valid-name", None), ("a", None), ("abc-123", None),
    ("Invalid-Name", "invalid InferenceService name"), ("bad_name", "invalid InferenceService name"),
    ("bad.name", "invalid InferenceService name"), ("-lead", "invalid InferenceService name"),
    ("trail-", "invalid InferenceService name"), ("1abc", "invalid InferenceService name"),
])
def test_isvc_names(name, err):
    _check(_isvc(name), Store(), err)


@pytest.mark.parametrize("ann,err", [
    ({}, None),                                                              # no autoscaler class
    ({C.AUTOSCALER_CLASS: C.AUTOSCALER_HPA}, None),
    ({C.AUTOSCALER_CLASS: C.AUTOSCALER_EXTERNAL}, None),
    ({C.AUTOSCALER_CLASS: C.AUTOSCALER_KEDA}, None),
    ({C.AUTOSCALER_CLASS: "bogus"}, "not a supported autoscaler class"),
    ({C.AUTOSCALER_CLASS: C.AUTOSCALER_HPA, C.AUTOSCALER_METRICS: "cpu"}, None),
    ({C.AUTOSCALER_CLASS: C.AUTOSCALER_HPA, C.AUTOSCALER_METRICS: "memory"}, None),
    ({C.AUTOSCALER_CLASS: C.AUTOSCALER_HPA, C.AUTOSCALER_METRICS: "invalid-metric"}, "not a supported metric"),
    ({C.TARGET_UTILIZATION: "50"}, None), ({C.TARGET_UTILIZATION: "1"}, None), ({C.TARGET_UTILIZATION: "100"}, None),
    ({C.TARGET_UTILIZATION: "0"}, r"\[1-100\]"), ({C.TARGET_UTILIZATION: "101"}, r"\[1-100\]"),
    ({C.TARGET_UTILIZATION: "abc"}, r"\[1-100\]"),
])
def test_isvc_autoscaling_annotations(ann, err):
    _check(_isvc(ann=ann), Store(), err)


@pytest.mark.parametrize("keda,ann,err", [
    (None, {}, None),
    ({"scalingOperator": "GreaterThanOrEqual", "scalingThreshold": "10", "promServerAddress": "http://prom:9090",
      "customPromQuery": "sum(x)"}, {}, None),
    ({"promServerAddress": "https://prom.example.com:9090"}, {}, None),
    ({"scalingOperator": "Bigger"}, {}, "invalid KEDA scaling operator"),
    (None, {C.KEDA_OPERATOR: "Bigger"}, "invalid KEDA scaling operator"),
    ({"scalingThreshold": "ten"}, {}, "invalid KEDA scaling threshold"),
    (None, {C.KEDA_THRESHOLD: "x1"}, "invalid KEDA scaling threshold"),
    ({"promServerAddress": "prom:9090"}, {}, "scheme must be http or https"),
    ({"promServerAddress": "ftp://prom:9090"}, {}, "scheme must be http or https"),
    ({"promServerAddress": "http://"}, {}, "host is required"),
    ({"authModes": "basic,bearer", "authenticationRef": {"name": "a"}}, {}, None),
    ({"authModes": "kerberos", "authenticationRef": {"name": "a"}}, {}, "invalid KEDA auth mode"),
    ({"authModes": "basic"}, {}, "requires authenticationRef"),
])
def test_isvc_keda(keda, ann, err):
    spec = {"kedaConfig": keda} if keda else {}
    _check(_isvc(ann={C.AUTOSCALER_CLASS: C.AUTOSCALER_KEDA, **ann}, spec=spec), Store(), err)


# ------------------------------------------------------------------ components / runners / models
RUNNER = {"runner": {"name": "ome-container", "image": "img"}}


@pytest.mark.parametrize("spec,err", [
    ({}, None),                                                                       # no decoder, no engine
    ({"engine": dict(RUNNER), "decoder": dict(RUNNER)}, None),                        # engine + decoder
    ({"decoder": dict(RUNNER)}, "decoder cannot be specified without engine"),
    ({"engine": {}}, "model reference is required"),                                  # empty engine
    ({"engine": {"runner": {"name": "c"}}}, "model reference is required"),           # runner without image
    ({"engine": dict(RUNNER)}, None),                                                 # runner with image
    ({"engine": {"leader": {"runner": {"image": "a"}}, "worker": {"runner": {"image": "b"}}}}, None),
    ({"engine": {"leader": {"runner": {"image": "a"}}}}, "model reference is required"),   # leader, no worker
    ({"engine": {"worker": {"runner": {"image": "b"}}}}, "model reference is required"),   # worker, no leader
    ({"engine": {"leader": {"runner": {}}, "worker": {"runner": {"image": "b"}}}}, "model reference is required"),
    ({"engine": {}, "runtime": {"name": "rt"}}, None),                                # runtime named
])
def test_isvc_components(spec, err):
    _check(_isvc(spec=spec), Store(), err)


@pytest.mark.parametrize("engine,ok", [
    (None, False), ({}, False), ({"runner": {"name": "x"}}, False), ({"runner": {"image": "i"}}, True),
    ({"leader": {"runner": {"image": "a"}}, "worker": {"runner": {"image": "b"}}}, True),
    ({"leader": {"runner": {"image": "a"}}, "worker": {"runner": {}}}, False),
    ({"containers": [{"name": "c", "image": "i"}]}, True), ({"containers": [{"name": "c"}]}, False),
])
def test_has_full_runner(engine, ok):
    assert has_full_runner(engine) is ok


@pytest.mark.parametrize("case,err", [
    ("model exists (cluster)", None),
    ("model not found", "not found in namespace"),
    ("model disabled", "is disabled"),
    ("no supporting runtime", "no supporting runtime found"),
    ("runtime named and compatible", None),
    ("runtime named but missing", "does not support model"),
    ("namespaced BaseModel in the same namespace", None),
    ("namespaced BaseModel in another namespace", "not found in namespace"),
    ("full runner skips runtime resolution", None),
])
def test_isvc_model_references(case, err):
    store = _store_with_model(disabled=case == "model disabled",
                              ns_model="team-a" if "namespaced" in case else None,
                              runtimes=case != "no supporting runtime")
    spec = {"model": {"name": "llama"}, "engine": {}}
    ns = "default"
    if case == "model not found":
        spec["model"]["name"] = "nope"
    if case.startswith("runtime named"):
        spec["runtime"] = {"name": "rt" if "compatible" in case else "missing-rt"}
    if "namespaced" in case:
        spec["model"]["name"] = "ns-model"
        ns = "team-a" if "same" in case else "team-b"
    if case == "full runner skips runtime resolution":
        store = _store_with_model(runtimes=False)
        spec["engine"] = dict(RUNNER)
    _check(_isvc(spec=spec, ns=ns), store, err)


# ------------------------------------------------------------------ ServingRuntime
def _rt(name, prio=1, auto=True, fmt="safetensors", size=("1B", "10B"), proto=("openAI",), workers=None,
        kind="ClusterServingRuntime", extra_formats=(), mode=None):
    f = {"modelFormat": {"name": fmt, "version": "1.0.0"}, "name": fmt, "modelArchitecture": "LlamaForCausalLM",
         "autoSelect": auto, "priority": prio}
    spec = {"supportedModelFormats": [f, *extra_formats], "protocolVersions": list(proto),
            "modelSizeRange": {"min": size[0], "max": size[1]}, "engineConfig": {"runner": {"image": "x"}}}
    if workers is not None:
        spec["workers"] = {"size": workers}
    if mode:
        spec["containers"] = [{"name": "c", "env": [{"name": "DEPLOYMENT_MODE", "value": mode}]}]
    return {"apiVersion": API, "kind": kind, "metadata": {"name": name}, "spec": spec}


@pytest.mark.parametrize("existing,new,err", [
    (None, _rt("a"), None),
    (_rt("a", prio=1), _rt("b", prio=2), None),                                           # distinct priorities
    (_rt("a", prio=1), _rt("b", prio=1), "same priority assigned"),                       # same priority, same format
    (_rt("a", prio=1), _rt("b", prio=1, fmt="onnx"), None),                               # different format
    (_rt("a", prio=1), _rt("b", prio=1, size=("20B", "80B")), None),                      # different size range
    (_rt("a", prio=1), _rt("b", prio=1, proto=("grpc",)), None),                          # no shared protocol
    (_rt("a", prio=1), _rt("b", prio=1, auto=False), None),                               # not auto-selected
    (None, _rt("a", extra_formats=[{"modelFormat": {"name": "safetensors"}, "name": "safetensors",
                                     "autoSelect": True, "priority": 2}]), "different priorities assigned"),
    (None, _rt("a", workers=0), "workers.size > 0"),
    (None, _rt("a", workers=2), None),                                                   # workers imply MultiNode
    (None, _rt("a", workers=2, mode=C.DeploymentMode.RAW), "RawDeployment must not define workers"),
    (None, _rt("a", mode=C.DeploymentMode.MULTINODE), "workers.size > 0"),
    (None, _rt("a", workers=2, mode=C.DeploymentMode.MULTINODE), None),
])
def test_runtime_validation(existing, new, err):
    s = Store()
    if existing is not None:
        s.create(existing)
    if err is None:
        validate_runtime("CREATE", new, None, s)
    else:
        with pytest.raises(Invalid, match=err):
            validate_runtime("CREATE", new, None, s)


def test_disabled_runtime_skips_validation():
    s = Store()
    s.create(_rt("a", prio=1))
    new = _rt("b", prio=1)
    new["spec"]["disabled"] = True
    validate_runtime("CREATE", new, None, s)


def test_runtime_missing_accelerator_class():
    new = _rt("a")
    new["spec"]["acceleratorRequirements"] = {"acceleratorClasses": ["amd-mi355x"]}
    with pytest.raises(Invalid, match="AcceleratorClasses do not exist"):
        validate_runtime("CREATE", new, None, Store())


# ------------------------------------------------------------------ BenchmarkJob
def _bj(**spec):
    base = {"endpoint": {"inferenceService": {"name": "svc", "namespace": "default"}}, "task": "text-to-text"}
    base.update(spec)
    return {"apiVersion": API, "kind": "BenchmarkJob", "metadata": {"name": "b", "namespace": "default"},
            "spec": base}


@pytest.mark.parametrize("spec,err", [
    ({}, None),
    ({"endpoint": {}}, "endpoint or InferenceService must be specified"),
    ({"endpoint": {"endpoint": {"url": "http://x"}, "inferenceService": {"name": "s"}}}, "cannot be specified together"),
    ({"endpoint": {"endpoint": {"url": "http://x", "apiFormat": "openai"}}}, None),
    ({"task": "text-to-video"}, "unsupported task"),
    ({"trafficScenarios": ["N(480,240)/(300,150)", "D(100,100)"]}, None),
    ({"trafficScenarios": ["Q(1,2)"]}, "failed to validate scenario"),
    ({"task": "text-to-embeddings", "trafficScenarios": ["E(64)"]}, None),
    ({"additionalRequestParams": {"temperature": "0.7"}}, None),
    ({"additionalRequestParams": {"temperature": "hot"}}, "invalid temperature"),
    ({"additionalRequestParams": {"ignore_eos": "true"}}, None),
    ({"additionalRequestParams": {"ignore_eos": "yes"}}, "ignore_eos must be"),
    ({"outputLocation": {"storageUri": "oci://n/ns/b/bucket/o/prefix"}}, None),
    ({"outputLocation": {"storageUri": ""}}, "storageUri cannot be empty"),
    ({"outputLocation": {"storageUri": "nope://x"}}, "error parsing storage URI"),
])
def test_benchmark_validation(spec, err):
    obj = _bj(**spec)
    if err is None:
        validate_benchmark("CREATE", obj, None, Store())
    else:
        with pytest.raises(Invalid, match=err):
            validate_benchmark("CREATE", obj, None, Store())

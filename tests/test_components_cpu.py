"""Component builders and status propagation, case by case (the reference's
``components/engine_test.go``, ``decoder_test.go``, ``base_test.go`` and
``status/status_reconciler_test.go`` / ``status_util_test.go`` case tables): deployment modes,
object metadata, worker pod specs, resource / affinity merge precedence (ISVC > AcceleratorClass >
runtime), accelerator overrides, fine-tuned serving, node selectors, the router's env / RBAC, the
readiness of every workload kind, model status from pods and the top-level Ready condition."""
import copy

import pytest

from ome_amd.api import constants as C
from ome_amd.api import v1beta1 as V
from ome_amd.controllers.config import ControllerConfig
from ome_amd.controllers.isvc import status as S
from ome_amd.controllers.isvc.components import ComponentContext, make_component
from ome_amd.store.store import Store

RAW, MN, RAY, KN = (C.DeploymentMode.RAW, C.DeploymentMode.MULTINODE, C.DeploymentMode.MULTINODE_RAY_VLLM,
                    C.DeploymentMode.SERVERLESS)
CBM = {"apiVersion": C.API_VERSION, "kind": "ClusterBaseModel", "metadata": {"name": "llama", "annotations": {}},
       "spec": {"vendor": "meta", "modelFormat": {"name": "safetensors", "version": "1.0.0"},
                "storage": {"storageUri": "hf://meta/llama", "path": "/raid/models/llama"}}}
BM = {"apiVersion": C.API_VERSION, "kind": "BaseModel", "metadata": {"name": "mine", "namespace": "team"},
      "spec": {"modelFormat": {"name": "safetensors"}, "storage": {"path": "/raid/models/mine"}}}
RUNNER = {"name": "ome-container", "image": "rt:1", "args": ["--tp-size", "1", "--model-path", "$(MODEL_PATH)"],
          "resources": {"limits": {"amd.com/gpu": "1"}}}


def _isvc(ann=None, labels=None, **spec):
    return {"apiVersion": C.API_VERSION, "kind": "InferenceService",
            "metadata": {"name": "svc", "namespace": "default", "uid": "uid-svc", "annotations": dict(ann or {}),
                         "labels": dict(labels or {})},
            "spec": {"model": {"name": "llama"}, **spec}}


def _ctx(mode=RAW, base=CBM, isvc=None, runtime_spec=None, ft=None, ac_name="", ac_spec=None, fmt=None):
    store = Store()
    return ComponentContext(store, isvc or _isvc(), ControllerConfig.from_store(store), mode,
                            copy.deepcopy(base) if base else None, "rt", runtime_spec or {}, fmt, ac_name, ac_spec,
                            ft or [])


def _env(c):
    return {e["name"]: e.get("value") for e in c.get("env") or []}


def _ft(strategy="lora"):
    return {"metadata": {"name": "ft-1"}, "spec": {"hyperParameters": {"strategy": strategy}}}


# ------------------------------------------------------------------ engine modes
def test_raw_deployment_with_basic_engine_spec():
    ctx = _ctx()
    info = make_component(C.ENGINE, ctx, {"runner": copy.deepcopy(RUNNER), "minReplicas": 1}).reconcile()
    assert info["mode"] == RAW and info["object"]["kind"] == "Deployment"
    pod = info["object"]["spec"]["template"]["spec"]
    c = pod["containers"][0]
    assert _env(c)[C.MODEL_PATH_ENV] == "/raid/models/llama" and _env(c)[C.PARALLELISM_SIZE_ENV] == "1"
    assert {"name": "llama", "mountPath": "/raid/models/llama", "readOnly": True} in c["volumeMounts"]
    assert {"name": "llama", "hostPath": {"path": "/raid/models/llama"}} in pod["volumes"]
    assert pod["nodeSelector"] == {C.model_label(None, "llama", True): "Ready"}


def test_multinode_leader_and_worker():
    ctx = _ctx(MN)
    spec = {"leader": {"runner": copy.deepcopy(RUNNER)}, "worker": {"size": 3, "runner": copy.deepcopy(RUNNER)}}
    info = make_component(C.ENGINE, ctx, spec).reconcile()
    lws = info["object"]
    assert lws["kind"] == "LeaderWorkerSet"
    tpl = lws["spec"]["leaderWorkerTemplate"]
    assert tpl["size"] == 4
    for part in ("leaderTemplate", "workerTemplate"):
        c = tpl[part]["spec"]["containers"][0]
        assert _env(c)[C.PARALLELISM_SIZE_ENV] == "4"   # gpus per pod x (1 + workers)


def test_multinode_ray_vllm_builds_probers():
    info = make_component(C.ENGINE, _ctx(RAY), {"runner": copy.deepcopy(RUNNER)}).reconcile()
    assert info["mode"] == RAY and "objects" in info


def test_serverless_knative_service():
    info = make_component(C.ENGINE, _ctx(KN), {"runner": copy.deepcopy(RUNNER), "minReplicas": 0}).reconcile()
    assert info["object"]["kind"] == "Service" and info["object"]["apiVersion"].startswith("serving.knative.dev")


def test_fine_tuned_serving_single_weight():
    ctx = _ctx(ft=[_ft()])
    comp = make_component(C.ENGINE, ctx, {"runner": copy.deepcopy(RUNNER)})
    pod = comp.leader_pod_spec()
    c = pod["containers"][0]
    env = _env(c)
    assert env[C.MODEL_PATH_ENV] == "/opt/ml/model" and env[C.SERVED_MODEL_NAME_ENV] == "/data/ft-1"
    assert {"name": "model-empty-dir", "mountPath": "/opt/ml/model"} in c["volumeMounts"]
    assert {"name": "model-empty-dir", "emptyDir": {"medium": "Memory"}} in pod["volumes"]
    a = comp.annotations()
    assert a[C.FT_ADAPTER_INJECTION] == "ft-1" and a[f"{C.GROUP}/fine-tuned-weight-ft-strategy"] == "lora"
    assert comp.labels()[C.FT_SERVING_LABEL] == "true"


def test_cluster_base_model_node_selector_merges_runtime_and_isvc_selectors():
    isvc = _isvc(engine={"nodeSelector": {"pool": "gpu"}})
    ctx = _ctx(isvc=isvc, runtime_spec={"nodeSelector": {"rt": "yes"}})
    pod = make_component(C.ENGINE, ctx, {"runner": copy.deepcopy(RUNNER)}).leader_pod_spec()
    assert pod["nodeSelector"] == {C.model_label(None, "llama", True): "Ready", "rt": "yes", "pool": "gpu"}


def test_namespaced_base_model_node_selector():
    pod = make_component(C.ENGINE, _ctx(base=BM), {"runner": copy.deepcopy(RUNNER)}).leader_pod_spec()
    assert pod["nodeSelector"] == {C.model_label("team", "mine", False): "Ready"}


def test_engine_without_runner_or_containers_errors():
    with pytest.raises(ValueError, match="no containers"):
        make_component(C.ENGINE, _ctx(), {}).leader_pod_spec()


def test_engine_without_base_model_has_no_model_plumbing():
    pod = make_component(C.ENGINE, _ctx(base=None), {"runner": copy.deepcopy(RUNNER)}).leader_pod_spec()
    assert "nodeSelector" not in pod and C.MODEL_PATH_ENV not in _env(pod["containers"][0])


def test_existing_model_path_env_is_not_overwritten():
    r = copy.deepcopy(RUNNER)
    r["env"] = [{"name": C.MODEL_PATH_ENV, "value": "/custom"}]
    pod = make_component(C.ENGINE, _ctx(), {"runner": r}).leader_pod_spec()
    assert _env(pod["containers"][0])[C.MODEL_PATH_ENV] == "/custom"


# ------------------------------------------------------------------ metadata
def test_basic_object_metadata():
    isvc = _isvc(ann={"team": "x", "kubectl.kubernetes.io/last-applied-configuration": "{}"}, labels={"app": "a"})
    comp = make_component(C.ENGINE, _ctx(isvc=isvc), {"runner": RUNNER, "labels": {"extra": "1"},
                                                      "annotations": {"note": "n"}})
    m = comp.meta()
    assert m["name"] == "svc-engine" and m["namespace"] == "default"
    assert m["labels"][C.ISVC_LABEL] == "svc" and m["labels"][C.COMPONENT_LABEL] == C.ENGINE
    assert m["labels"]["app"] == "a" and m["labels"]["extra"] == "1"
    assert m["labels"][C.BASE_MODEL_NAME_LABEL] == "llama" and m["labels"][C.BASE_MODEL_TYPE_LABEL] == "Serving"
    assert m["labels"][C.BASE_MODEL_SIZE_LABEL] == "SMALL" and m["labels"][C.BASE_MODEL_VENDOR_LABEL] == "meta"
    a = m["annotations"]
    assert "kubectl.kubernetes.io/last-applied-configuration" not in a and a["team"] == "x" and a["note"] == "n"
    assert a[C.BASE_MODEL_NAME_ANN] == "llama" and a[C.BASE_MODEL_FORMAT_ANN] == "safetensors"
    assert a[C.BASE_MODEL_FORMAT_VERSION_ANN] == "1.0.0" and a[C.SERVING_RUNTIME_ANN] == "rt"


def test_model_category_label_and_decryption_annotations():
    base = copy.deepcopy(CBM)
    base["metadata"]["annotations"] = {C.MODEL_CATEGORY: "LARGE", C.BASE_MODEL_DECRYPTION_KEY: "k",
                                       C.BASE_MODEL_DECRYPTION_SECRET: "s"}
    comp = make_component(C.ENGINE, _ctx(base=base), {"runner": RUNNER})
    assert comp.labels()[C.BASE_MODEL_SIZE_LABEL] == "LARGE"
    a = comp.annotations()
    assert a[C.BASE_MODEL_DECRYPTION_KEY] == "k" and a[C.BASE_MODEL_DECRYPTION_SECRET] == "s"


def test_fine_tuned_metadata_without_strategy():
    ft = {"metadata": {"name": "ft-2"}, "spec": {}}
    a = make_component(C.ENGINE, _ctx(ft=[ft]), {"runner": RUNNER}).annotations()
    assert a[C.FT_ADAPTER_INJECTION] == "ft-2" and f"{C.GROUP}/fine-tuned-weight-ft-strategy" not in a


# ------------------------------------------------------------------ worker pod spec
def test_worker_with_runner():
    comp = make_component(C.ENGINE, _ctx(MN), {"leader": {"runner": RUNNER},
                                               "worker": {"size": 1, "runner": copy.deepcopy(RUNNER)}})
    ws = comp.worker_pod_spec()
    assert ws["containers"][0]["image"] == "rt:1" and comp.worker_size() == 1


def test_worker_without_runner_uses_its_containers():
    w = {"size": 2, "containers": [{"name": "ome-container", "image": "w:2"}]}
    ws = make_component(C.ENGINE, _ctx(MN), {"leader": {"runner": RUNNER}, "worker": w}).worker_pod_spec()
    assert ws["containers"][0]["image"] == "w:2"


def test_worker_without_runner_or_containers_is_none():
    comp = make_component(C.ENGINE, _ctx(MN), {"leader": {"runner": RUNNER}, "worker": {"size": 2}})
    assert comp.worker_pod_spec() is None


def test_no_worker_spec_returns_none():
    assert make_component(C.ENGINE, _ctx(), {"runner": RUNNER}).worker_pod_spec() is None


# ------------------------------------------------------------------ resource / affinity merge
RT_SPEC = {"containers": [{"name": "ome-container", "resources": {"requests": {"cpu": "8", "memory": "64Gi"},
                                                                  "limits": {"cpu": "8", "memory": "64Gi"}}}]}
AC_SPEC = {"resources": [{"name": "amd.com/gpu", "quantity": "8"}],
           "discovery": {"nodeSelector": {"accel": "mi355x"},
                         "affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                             "nodeSelectorTerms": [{"matchExpressions": [{"key": "gpu", "operator": "Exists"}]}]}}}}}


def test_user_specified_resources_are_not_merged():
    r = copy.deepcopy(RUNNER)
    isvc = _isvc(engine={"runner": {"resources": {"limits": {"amd.com/gpu": "2"}}}})
    r["resources"] = {"limits": {"amd.com/gpu": "2"}}
    pod = make_component(C.ENGINE, _ctx(isvc=isvc, runtime_spec=RT_SPEC, ac_spec=AC_SPEC, ac_name="mi355x"),
                         {"runner": r}).leader_pod_spec()
    assert pod["containers"][0]["resources"] == {"limits": {"amd.com/gpu": "2"}}


def test_unspecified_resources_merge_from_runtime():
    r = {k: v for k, v in RUNNER.items() if k != "resources"}
    pod = make_component(C.ENGINE, _ctx(runtime_spec=RT_SPEC), {"runner": r}).leader_pod_spec()
    res = pod["containers"][0]["resources"]
    assert res["requests"] == {"cpu": "8", "memory": "64Gi"} and res["limits"]["memory"] == "64Gi"


def test_unspecified_resources_merge_from_accelerator_class_over_runtime():
    r = {k: v for k, v in RUNNER.items() if k != "resources"}
    pod = make_component(C.ENGINE, _ctx(runtime_spec=RT_SPEC, ac_spec=AC_SPEC, ac_name="mi355x"),
                         {"runner": r}).leader_pod_spec()
    c = pod["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == "8" and c["resources"]["limits"]["cpu"] == "8"
    assert _env(c)[C.PARALLELISM_SIZE_ENV] == "8"


def test_no_runner_no_resource_merge():
    ps = make_component(C.ENGINE, _ctx(runtime_spec=RT_SPEC, ac_spec=AC_SPEC, ac_name="mi355x"),
                        {"containers": [{"name": "ome-container", "image": "x"}]}).leader_pod_spec()
    assert "resources" not in ps["containers"][0]


def test_user_specified_affinity_is_kept():
    aff = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": []}}
    isvc = _isvc(engine={"affinity": aff})
    pod = make_component(C.ENGINE, _ctx(isvc=isvc, ac_spec=AC_SPEC, ac_name="mi355x"),
                         {"runner": RUNNER, "affinity": aff}).leader_pod_spec()
    assert pod["affinity"] == aff


def test_unspecified_affinity_merges_from_accelerator_class():
    pod = make_component(C.ENGINE, _ctx(ac_spec=AC_SPEC, ac_name="mi355x"), {"runner": RUNNER}).leader_pod_spec()
    assert pod["affinity"] == AC_SPEC["discovery"]["affinity"] and pod["nodeSelector"]["accel"] == "mi355x"


def test_no_accelerator_affinity_stays_unset():
    pod = make_component(C.ENGINE, _ctx(ac_spec={"resources": []}, ac_name="x"), {"runner": RUNNER}).leader_pod_spec()
    assert "affinity" not in pod


# ------------------------------------------------------------------ accelerator overrides
def _fmt(**cfg):
    return V.SupportedModelFormat.model_validate({"name": "safetensors", "acceleratorConfig": {"mi355x": cfg}})


@pytest.mark.parametrize("override,want_tp", [({"tensorParallelSize": 4}, "4"), ({}, "1")])
def test_tensor_parallelism_override(override, want_tp):
    fmt = _fmt(tensorParallelismOverride=override) if override else _fmt()
    r = copy.deepcopy(RUNNER)
    pod = make_component(C.ENGINE, _ctx(fmt=fmt, ac_name="mi355x"), {"runner": r}).leader_pod_spec()
    args = pod["containers"][0]["args"]
    assert args[args.index("--tp-size") + 1] == want_tp


def test_pipeline_and_data_parallel_override_rewrite_existing_flags():
    fmt = _fmt(tensorParallelismOverride={"pipelineParallelSize": 2, "dataParallelSize": 4})
    r = copy.deepcopy(RUNNER)
    r["args"] += ["--pipeline-parallel-size=1", "--dp", "1"]
    pod = make_component(C.ENGINE, _ctx(fmt=fmt, ac_name="mi355x"), {"runner": r}).leader_pod_spec()
    args = pod["containers"][0]["args"]
    assert "--pipeline-parallel-size=2" in args and args[args.index("--dp") + 1] == "4"
    # flags the runner does not carry are not invented (rewrite-only, as the reference)
    pod = make_component(C.ENGINE, _ctx(fmt=fmt, ac_name="mi355x"), {"runner": copy.deepcopy(RUNNER)}).leader_pod_spec()
    assert pod["containers"][0]["args"] == RUNNER["args"]


def test_runtime_args_and_environment_override():
    fmt = _fmt(runtimeArgsOverride=["--mem-frac", "0.8", "--tp-size", "2"], environmentOverride={"HIP_FORCE": "1"})
    pod = make_component(C.ENGINE, _ctx(fmt=fmt, ac_name="mi355x"), {"runner": copy.deepcopy(RUNNER)}).leader_pod_spec()
    c = pod["containers"][0]
    assert c["args"][c["args"].index("--tp-size") + 1] == "2" and "--mem-frac" in c["args"]
    assert _env(c)["HIP_FORCE"] == "1"


def test_accelerator_config_ignored_without_selected_class():
    fmt = _fmt(environmentOverride={"HIP_FORCE": "1"})
    pod = make_component(C.ENGINE, _ctx(fmt=fmt), {"runner": copy.deepcopy(RUNNER)}).leader_pod_spec()
    assert "HIP_FORCE" not in _env(pod["containers"][0])


# ------------------------------------------------------------------ decoder / router
def test_decoder_raw_deployment_name_and_component_label():
    info = make_component(C.DECODER, _ctx(), {"runner": copy.deepcopy(RUNNER)}).reconcile()
    assert info["object"]["metadata"]["name"] == "svc-decoder"
    assert info["object"]["spec"]["template"]["metadata"]["labels"][C.COMPONENT_LABEL] == C.DECODER


def test_decoder_rejects_serverless():
    with pytest.raises(ValueError, match="serverless"):
        make_component(C.DECODER, _ctx(KN), {"runner": copy.deepcopy(RUNNER)}).reconcile()


def test_decoder_multinode():
    spec = {"leader": {"runner": copy.deepcopy(RUNNER)}, "worker": {"size": 1, "runner": copy.deepcopy(RUNNER)}}
    info = make_component(C.DECODER, _ctx(MN), spec).reconcile()
    assert info["object"]["kind"] == "LeaderWorkerSet" and info["object"]["metadata"]["name"] == "lws-svc-decoder"


def test_router_env_rbac_and_annotations():
    ctx = _ctx(isvc=_isvc(ann={"a": "1"}))
    comp = make_component(C.ROUTER, ctx, {"runner": {"name": "router", "image": "r:1"},
                                          "config": {"policy": "cache_aware", "port": 8080}})
    pod = comp.leader_pod_spec()
    env = _env(pod["containers"][0])
    assert env["policy"] == "cache_aware" and env["port"] == "8080"
    assert env["INFERENCESERVICE_NAME"] == "svc" and env["NAMESPACE"] == "default"
    assert pod["serviceAccountName"]
    a = comp.annotations()
    assert a["a"] == "1" and a[C.SERVING_RUNTIME_ANN] == "rt" and C.BASE_MODEL_NAME_ANN not in a
    kinds = {o["kind"] for o in ctx.store.all()}
    assert {"ServiceAccount", "Role", "RoleBinding"} <= kinds


def test_router_does_not_get_model_plumbing():
    pod = make_component(C.ROUTER, _ctx(), {"runner": {"name": "router", "image": "r:1"}}).leader_pod_spec()
    assert "nodeSelector" not in pod and C.MODEL_PATH_ENV not in _env(pod["containers"][0])


def test_placeholders_replaced_in_runner():
    r = copy.deepcopy(RUNNER)
    r["args"] = ["--served-model-name", "{{ .Name }}-{{ .Namespace }}"]
    pod = make_component(C.ENGINE, _ctx(), {"runner": r}).leader_pod_spec()
    assert pod["containers"][0]["args"][-1] == "svc-default"


# ------------------------------------------------------------------ status: workload readiness
def _obj(conds, name="w"):
    return {"metadata": {"name": name}, "status": {"conditions": conds}}


@pytest.mark.parametrize("mode,info,want", [
    (RAW, {"object": _obj([])}, ("Unknown", "DeploymentPending")),
    (RAW, {"object": _obj([{"type": "Available", "status": "True", "reason": "MinimumReplicasAvailable"}])},
     ("True", "MinimumReplicasAvailable")),
    (RAW, {"object": _obj([{"type": "Available", "status": "False", "reason": "ProgressDeadlineExceeded"}])},
     ("False", "ProgressDeadlineExceeded")),
    (MN, {"object": _obj([])}, ("Unknown", "LeaderWorkerSetPending")),
    (MN, {"object": _obj([{"type": "Available", "status": "True"}])}, ("True", "")),
    (RAY, {"objects": []}, ("False", "NoDeployments")),
    (RAY, {"objects": [_obj([{"type": "Available", "status": "True"}], "p0"), _obj([], "p1")]},
     ("False", "ProberUnavailable")),
    (RAY, {"objects": [_obj([{"type": "Available", "status": "True"}], "p0")]}, ("True", "")),
    (KN, {"object": _obj([])}, ("Unknown", "KnativePending")),
    (KN, {"object": _obj([{"type": "Ready", "status": "True"}])}, ("True", "")),
    ("Bogus", {"object": None}, ("Unknown", "")),
])
def test_workload_ready(mode, info, want):
    st, reason, _ = S.workload_ready({"mode": mode, **info})
    assert (st, reason) == want


# ------------------------------------------------------------------ status: model state from pods
def _pod(name, ready=False, exit_code=None, phase="Running", last=False):
    st = {"phase": phase, "conditions": [{"type": "Ready", "status": "True" if ready else "False"}]}
    if exit_code is not None:
        term = {"exitCode": exit_code, "message": "OOM", "reason": "Error"}
        st["containerStatuses"] = [{"lastState" if last else "state": {"terminated": term}}]
    return {"metadata": {"name": name}, "status": st}


def test_model_status_no_pods_pending():
    s = S.model_status_from_pods([])
    assert s["transitionStatus"] == "InProgress" and s["modelRevisionStates"]["activeModelState"] == "Pending"


def test_model_status_loading():
    s = S.model_status_from_pods([_pod("a")])
    assert s["modelRevisionStates"] == {"activeModelState": "Loading", "targetModelState": "Loaded"}
    assert s["modelCopies"] == {"failedCopies": 0, "totalCopies": 1}


def test_model_status_loaded_wins_over_a_failed_copy():
    s = S.model_status_from_pods([_pod("a", ready=True), _pod("b", exit_code=137, phase="Failed")])
    assert s["transitionStatus"] == "UpToDate" and s["modelCopies"] == {"failedCopies": 1, "totalCopies": 2}


@pytest.mark.parametrize("last", [False, True])
def test_model_status_failed_to_load(last):
    s = S.model_status_from_pods([_pod("a", exit_code=1, last=last)])
    assert s["transitionStatus"] == "BlockedByFailedLoad"
    f = s["lastFailureInfo"]
    assert f["location"] == "a" and f["exitCode"] == 1 and f["message"] == "OOM"


def test_zero_exit_is_not_a_failure():
    s = S.model_status_from_pods([_pod("a", exit_code=0)])
    assert s["transitionStatus"] == "InProgress"


# ------------------------------------------------------------------ status: conditions / Ready
def test_set_condition_updates_transition_only_on_change():
    st = {}
    S.set_condition(st, "EngineReady", "False", "X")
    t0 = S.get_condition(st, "EngineReady")["lastTransitionTime"]
    S.set_condition(st, "EngineReady", "False", "Y")
    assert S.get_condition(st, "EngineReady")["lastTransitionTime"] == t0
    assert S.get_condition(st, "EngineReady")["reason"] == "Y"


def test_conditions_sorted_by_type():
    st = {}
    for t in ("RouterReady", "EngineReady", "IngressReady"):
        S.set_condition(st, t, "True")
    assert [c["type"] for c in st["conditions"]] == ["EngineReady", "IngressReady", "RouterReady"]


@pytest.mark.parametrize("comps,conds,want", [
    ([C.ENGINE], {"IngressReady": "True", "EngineReady": "True"}, "True"),
    ([C.ENGINE], {"IngressReady": "True", "EngineReady": "False"}, "False"),
    ([C.ENGINE], {"IngressReady": "True"}, "Unknown"),
    ([C.ENGINE, C.DECODER], {"IngressReady": "True", "EngineReady": "True"}, "Unknown"),
    ([C.ENGINE, C.DECODER], {"IngressReady": "True", "EngineReady": "True", "DecoderReady": "True"}, "True"),
    ([C.ENGINE, C.ROUTER], {"IngressReady": "True", "EngineReady": "True", "RouterReady": "False"}, "False"),
    ([C.ENGINE], {"IngressReady": "False", "EngineReady": "True"}, "False"),
    ([C.PREDICTOR], {"IngressReady": "True", "PredictorReady": "True"}, "True"),
])
def test_finalize_ready(comps, conds, want):
    st = {}
    for k, v in conds.items():
        S.set_condition(st, k, v, "R" if v != "True" else "")
    S.finalize_ready(st, comps)
    assert S.get_condition(st, "Ready")["status"] == want
    assert S.is_ready({"status": st}) == (want == "True")


def test_finalize_ready_message_names_missing_conditions():
    st = {}
    S.set_condition(st, "IngressReady", "True")
    S.finalize_ready(st, [C.ENGINE, C.ROUTER])
    c = S.get_condition(st, "Ready")
    assert "EngineReady" in c["message"] and "RouterReady" in c["message"]


def test_component_pods_select_by_isvc_and_component():
    store = Store()
    for n, comp in (("a", C.ENGINE), ("b", C.ENGINE), ("c", C.DECODER)):
        store.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": n, "namespace": "default",
                                                                       "labels": {C.ISVC_LABEL: "svc",
                                                                                  C.COMPONENT_LABEL: comp}}})
    store.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "z", "namespace": "default",
                                                                   "labels": {C.ISVC_LABEL: "other",
                                                                              C.COMPONENT_LABEL: C.ENGINE}}})
    got = sorted(p["metadata"]["name"] for p in S.component_pods(store, _isvc(), C.ENGINE))
    assert got == ["a", "b"]

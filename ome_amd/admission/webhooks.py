"""Admission webhooks as store hooks (``pkg/webhook/admission/{isvc,servingruntime,benchmark,pod}``).

Defaulting:
  * InferenceService: ``ome.io/deploymentMode`` (PDDisaggregated if engine+decoder; MultiNode
    if engine leader+worker with size>0; else the config default), deprecation warning for
    ``predictor``, replica defaults engine/decoder 1..3 and router 1..2.
  * BenchmarkJob: default traffic scenarios per task and the concurrency sweep.
Validation:
  * InferenceService: DNS name, autoscaler class, target utilisation 1..100, KEDA
    operator/threshold/server/auth modes, decoder requires engine, model exists (and is
    enabled), runtime valid or auto-selectable unless the engine carries a full runner.
  * (Cluster)ServingRuntime: auto-select priority identical across a runtime's formats, no
    equal priority on an equal format among runtimes speaking the same protocol, MultiNode /
    Raw worker-size sanity, referenced AcceleratorClasses exist.
  * BenchmarkJob: endpoint XOR, scenario grammar per task, request params, storage URI.
Pod mutation (pods labelled ``ome.io/inferenceservice``): metrics aggregation -> model-init
(decryption) -> fine-tuned adapter -> serving sidecar -> interconnect profile injection, with
model-init ordered before the adapter among init containers.
"""
from __future__ import annotations

import json
import re
from urllib.parse import urlparse

from ome_amd.api import constants as C
from ome_amd.bench import scenarios as SC
from ome_amd.controllers.config import ControllerConfig
from ome_amd.policy.runtime_selector import RuntimeSelector, SelectorError
from ome_amd.api import v1beta1 as V
from ome_amd.storage import uri as U
from ome_amd.store.store import Forbidden, Invalid, Store

ISVC_NAME_RE = re.compile(r"^[a-z]([-a-z0-9]*[a-z0-9])?$")
DEPRECATION_WARNING_PREDICTOR = ("The Predictor field is deprecated and will be removed in a future release. "
                                 "Please use Engine and Model fields instead.")
KEDA_OPERATORS = ("GreaterThan", "GreaterThanOrEqual", "LessThan", "LessThanOrEqual", "Equal", "NotEqual")
KEDA_AUTH_MODES = ("basic", "bearer", "tls", "custom")


# ------------------------------------------------------------------ InferenceService
def default_isvc(op, obj, old, store: Store):
    meta = obj.setdefault("metadata", {})
    ann = meta.setdefault("annotations", {})
    sp = obj.setdefault("spec", {})
    cfg = ControllerConfig.from_store(store)
    if C.DEPLOYMENT_MODE not in ann:
        eng, dec = sp.get("engine"), sp.get("decoder")
        if eng is not None and dec is not None:
            ann[C.DEPLOYMENT_MODE] = C.DeploymentMode.PD
        elif eng is not None:
            w = eng.get("worker") or {}
            if eng.get("leader") is not None and w and (w.get("size") or 0) > 0:
                ann[C.DEPLOYMENT_MODE] = C.DeploymentMode.MULTINODE
            elif cfg.deploy.defaultDeploymentMode == C.DeploymentMode.RAW:
                ann[C.DEPLOYMENT_MODE] = C.DeploymentMode.RAW
        elif cfg.deploy.defaultDeploymentMode == C.DeploymentMode.RAW:
            ann[C.DEPLOYMENT_MODE] = C.DeploymentMode.RAW
    if sp.get("predictor"):
        ann.setdefault(C.DEPRECATION_WARNING, DEPRECATION_WARNING_PREDICTOR)
    for comp, mx in (("engine", 3), ("decoder", 3), ("router", 2)):
        c = sp.get(comp)
        if c is not None:
            if c.get("minReplicas") is None:
                c["minReplicas"] = 1
            if not c.get("maxReplicas"):
                c["maxReplicas"] = mx
    return obj


def _validate_keda(keda: dict | None, ann: dict) -> None:
    keda = keda or {}
    for v in ([keda.get("scalingOperator")] if keda.get("scalingOperator") else []) + \
             ([ann[C.KEDA_OPERATOR]] if C.KEDA_OPERATOR in ann else []):
        if v not in KEDA_OPERATORS:
            raise Invalid(f"invalid KEDA scaling operator {v!r}, must be one of: {', '.join(KEDA_OPERATORS)}")
    for v in ([keda.get("scalingThreshold")] if keda.get("scalingThreshold") else []) + \
             ([ann[C.KEDA_THRESHOLD]] if C.KEDA_THRESHOLD in ann else []):
        try:
            float(v)
        except ValueError:
            raise Invalid(f"invalid KEDA scaling threshold {v!r}: must be a valid number") from None
    for v in ([keda.get("promServerAddress")] if keda.get("promServerAddress") else []) + \
             ([ann[C.KEDA_SERVER_ADDRESS]] if C.KEDA_SERVER_ADDRESS in ann else []):
        u = urlparse(v)
        if u.scheme not in ("http", "https"):
            raise Invalid(f"invalid KEDA Prometheus server address {v!r}: scheme must be http or https")
        if not u.netloc:
            raise Invalid(f"invalid KEDA Prometheus server address {v!r}: host is required")
    if keda.get("authModes"):
        for m in [x.strip() for x in keda["authModes"].split(",")]:
            if m not in KEDA_AUTH_MODES:
                raise Invalid(f"invalid KEDA auth mode {m!r}, must be one of: {', '.join(KEDA_AUTH_MODES)}")
        if not keda.get("authenticationRef"):
            raise Invalid("KEDA authModes requires authenticationRef")


def has_full_runner(engine: dict | None) -> bool:
    if not engine:
        return False
    if (engine.get("runner") or {}).get("image"):
        return True
    if engine.get("leader") and engine.get("worker"):
        return bool(((engine["leader"].get("runner") or {}).get("image")) and
                    ((engine["worker"].get("runner") or {}).get("image")))
    return any(c.get("image") for c in engine.get("containers") or [])


def validate_isvc(op, obj, old, store: Store):
    meta, sp = obj["metadata"], obj.get("spec") or {}
    name = meta.get("name", "")
    if not ISVC_NAME_RE.match(name):
        raise Invalid(f"invalid InferenceService name {name!r}, must match {ISVC_NAME_RE.pattern!r}")
    ann = meta.get("annotations") or {}
    cls = ann.get(C.AUTOSCALER_CLASS)
    if cls is not None and cls not in C.AUTOSCALER_CLASSES:
        raise Invalid(f"[{cls}] is not a supported autoscaler class type")
    if cls == C.AUTOSCALER_HPA and C.AUTOSCALER_METRICS in ann and \
            ann[C.AUTOSCALER_METRICS] not in C.AUTOSCALER_METRICS_ALLOWED:
        raise Invalid(f"[{ann[C.AUTOSCALER_METRICS]}] is not a supported metric")
    if C.TARGET_UTILIZATION in ann:
        try:
            t = int(ann[C.TARGET_UTILIZATION])
        except ValueError:
            raise Invalid("the target utilization percentage should be a [1-100] integer") from None
        if not 1 <= t <= 100:
            raise Invalid("the target utilization percentage should be a [1-100] integer")
    if cls == C.AUTOSCALER_KEDA or sp.get("kedaConfig"):
        _validate_keda(sp.get("kedaConfig"), ann)
    if sp.get("decoder") is not None and sp.get("engine") is None:
        raise Invalid("decoder cannot be specified without engine")
    model = sp.get("model") or {}
    bm = None
    if model.get("name"):
        ns = meta.get("namespace", "default")
        bm = store.try_get(C.API_VERSION, "BaseModel", model["name"], ns) or \
            store.try_get(C.API_VERSION, "ClusterBaseModel", model["name"])
        if bm is None:
            raise Invalid(f"referenced model {model['name']!r} not found in namespace {ns!r}: ensure a BaseModel "
                          "exists in this namespace or a ClusterBaseModel exists cluster-wide with this name")
    if sp.get("engine") is not None:
        if sp.get("runtime") is None and not has_full_runner(sp["engine"]) and not model.get("name"):
            raise Invalid("model reference is required when runtime is not specified and engine does not have "
                          "complete runner configuration")
        if bm is not None:
            bspec = V.spec_of(bm)
            if bspec.disabled:
                raise Invalid(f"model {model['name']} is disabled")
            sel = RuntimeSelector(store)
            rt = (sp.get("runtime") or {}).get("name")
            try:
                if rt:
                    sel.validate(rt, bspec, obj, meta.get("namespace", "default"))
                elif not has_full_runner(sp["engine"]):
                    sel.select(bspec, obj, meta.get("namespace", "default"))
            except SelectorError as e:
                if rt:
                    raise Invalid(f"runtime {rt} does not support model {model['name']}: {e}") from None
                raise Invalid(f"no supporting runtime found for model {model['name']} and engine does not have "
                              f"complete runner configuration: {e}") from None
    return None


# ------------------------------------------------------------------ ServingRuntime
def _fmt_key(f: dict) -> tuple:
    return ((f.get("name") or "").lower(), f.get("version"), f.get("quantization"),
            json.dumps(f.get("modelFramework"), sort_keys=True), json.dumps(f.get("modelFormat"), sort_keys=True),
            f.get("modelArchitecture"))


def validate_runtime_configuration(spec: dict) -> None:
    has_e, has_d = spec.get("engineConfig") is not None, spec.get("decoderConfig") is not None
    if has_e and has_d:
        return
    ws = (spec.get("workers") or {}).get("size")
    if ws is not None and ws <= 0:
        raise Invalid("MultiNode deployment requires workers.size > 0")
    explicit = None
    for c in spec.get("containers") or []:
        for e in c.get("env") or []:
            if e.get("name") == "DEPLOYMENT_MODE" and e.get("value") in (C.DeploymentMode.MULTINODE,
                                                                          C.DeploymentMode.RAW):
                explicit = e["value"]
    if has_e:
        multi = explicit == C.DeploymentMode.MULTINODE or (explicit is None and (ws or 0) > 0)
        if multi and not (ws and ws > 0):
            raise Invalid("MultiNode deployment requires workers.size > 0")
        if not multi and (ws or 0) > 0:
            raise Invalid("RawDeployment must not define workers with size > 0")


def validate_runtime(op, obj, old, store: Store):
    spec = obj.get("spec") or {}
    if spec.get("disabled"):
        return None
    validate_runtime_configuration(spec)
    acs = (spec.get("acceleratorRequirements") or {}).get("acceleratorClasses") or []
    missing = [a for a in acs if store.try_get(C.API_VERSION, "AcceleratorClass", a) is None]
    if missing:
        raise Invalid(f"referenced AcceleratorClasses do not exist: {', '.join(missing)}")
    prio: dict[str, int | None] = {}
    for f in spec.get("supportedModelFormats") or []:
        if f.get("autoSelect"):
            n = f.get("name")
            if n in prio and prio[n] is not None and f.get("priority") is not None and prio[n] != f["priority"]:
                raise Invalid(f"different priorities assigned for the model format {n} in {obj['metadata']['name']}")
            prio.setdefault(n, f.get("priority"))
    ns = obj["metadata"].get("namespace") if obj["kind"] == "ServingRuntime" else None
    for other in store.list(C.API_VERSION, obj["kind"], namespace=ns):
        if other["metadata"]["name"] == obj["metadata"]["name"]:
            continue
        osp = other.get("spec") or {}
        if osp.get("disabled"):
            continue
        if not set(osp.get("protocolVersions") or []) & set(spec.get("protocolVersions") or []):
            continue
        if (osp.get("modelSizeRange") or None) != (spec.get("modelSizeRange") or None):
            continue
        for of in osp.get("supportedModelFormats") or []:
            for nf in spec.get("supportedModelFormats") or []:
                if of.get("autoSelect") and nf.get("autoSelect") and _fmt_key(of) == _fmt_key(nf) and \
                        of.get("priority") is not None and of.get("priority") == nf.get("priority"):
                    raise Invalid(f"same priority assigned for the model format {nf.get('name')} in runtimes "
                                  f"{other['metadata']['name']} and {obj['metadata']['name']}")
    return None


# ------------------------------------------------------------------ BenchmarkJob
def default_benchmark(op, obj, old, store: Store):
    sp = obj.setdefault("spec", {})
    task = sp.get("task", "text-to-text")
    if not sp.get("trafficScenarios"):
        sp["trafficScenarios"] = list(SC.DEFAULT_SCENARIOS.get(task, []))
    if not sp.get("numConcurrency"):
        sp["numConcurrency"] = list(SC.DEFAULT_CONCURRENCY)
    sp.setdefault("maxTimePerIteration", 15)
    sp.setdefault("maxRequestsPerIteration", 100)
    return obj


def validate_benchmark(op, obj, old, store: Store):
    sp = obj.get("spec") or {}
    ep = sp.get("endpoint") or {}
    if not ep.get("endpoint") and not ep.get("inferenceService"):
        raise Invalid("invalid endpoint: endpoint or InferenceService must be specified")
    if ep.get("endpoint") and ep.get("inferenceService"):
        raise Invalid("invalid endpoint: endpoint and InferenceService cannot be specified together")
    task = sp.get("task")
    if task not in SC.TASK_SCENARIOS:
        raise Invalid(f"invalid traffic scenarios: unsupported task {task!r}")
    for s in sp.get("trafficScenarios") or SC.DEFAULT_SCENARIOS.get(task, []):
        if not SC.validate(s, task):
            raise Invalid(f"invalid traffic scenarios: failed to validate scenario {s!r} for task {task!r}")
    for k, v in (sp.get("additionalRequestParams") or {}).items():
        if k == "temperature":
            try:
                float(v)
            except ValueError:
                raise Invalid(f"invalid additional request parameters: invalid temperature {v!r}") from None
        if k == "ignore_eos" and v not in ("true", "false"):
            raise Invalid("invalid additional request parameters: ignore_eos must be 'true' or 'false'")
    out = sp.get("outputLocation")
    if out is not None:
        if not out.get("storageUri"):
            raise Invalid("invalid storage: storageUri cannot be empty")
        try:
            U.validate(out["storageUri"])
        except U.StorageURIError as e:
            raise Invalid(f"invalid storage: error parsing storage URI: {e}") from None
    return None


# ------------------------------------------------------------------ Pod mutator
INTERCONNECT_PROFILES = {
    # MI355X single node: 8 GPUs fully connected by xGMI (7 links per GPU).  RCCL reads NCCL_*.
    "amd-xgmi": {
        "env": {"NCCL_DEBUG": "WARN", "NCCL_MIN_NCHANNELS": "112", "NCCL_IGNORE_CPU_AFFINITY": "1",
                "RCCL_MSCCL_ENABLE": "1", "RCCL_MSCCLPP_ENABLE": "1", "HSA_FORCE_FINE_GRAIN_PCIE": "1",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0", "TORCH_NCCL_HIGH_PRIORITY": "1",
                "GLOO_SOCKET_IFNAME": "lo", "NCCL_SOCKET_IFNAME": "lo", "NCCL_CUMEM_ENABLE": "0"},
        "volumes": [{"name": "dshm", "emptyDir": {"medium": "Memory"}}],
        "mounts": [{"name": "dshm", "mountPath": "/dev/shm"}],
        "devices": ["/dev/kfd", "/dev/dri"],
        "securityContext": {"capabilities": {"add": ["IPC_LOCK", "SYS_PTRACE"]}},
    },
    # multi-node RoCE (reference profile, rdma_injector.go:25-90) for clusters of MI355X nodes
    "oci-roce": {
        "env": {"NCCL_NET_PLUGIN": "none", "NCCL_DEBUG": "INFO", "NCCL_CROSS_NIC": "2", "NCCL_SOCKET_NTHREADS": "16",
                "NCCL_CUMEM_ENABLE": "0", "NCCL_IB_SPLIT_DATA_ON_QPS": "0", "NCCL_IB_QPS_PER_CONNECTION": "16",
                "NCCL_IB_GID_INDEX": "3", "NCCL_IB_TC": "41", "NCCL_IB_SL": "0", "NCCL_IB_TIMEOUT": "22",
                "HCOLL_ENABLE_MCAST_ALL": "0", "coll_hcoll_enable": "0", "UCX_TLS": "tcp", "UCX_NET_DEVICES": "eth0",
                "RX_QUEUE_LEN": "8192", "IB_RX_QUEUE_LEN": "8192", "NCCL_SOCKET_IFNAME": "eth0",
                "NCCL_IGNORE_CPU_AFFINITY": "1", "GLOO_SOCKET_IFNAME": "eth0"},
        "volumes": [{"name": "dshm", "emptyDir": {"medium": "Memory"}},
                    {"name": "devinf", "hostPath": {"path": "/dev/infiniband"}}],
        "mounts": [{"name": "dshm", "mountPath": "/dev/shm"}, {"name": "devinf", "mountPath": "/dev/infiniband"}],
        "securityContext": {"capabilities": {"add": ["IPC_LOCK", "CAP_SYS_ADMIN"]}, "privileged": True},
    },
}
DEFAULT_INTERCONNECT_PROFILE = "amd-xgmi"


def _cm_json(cm: dict, key: str) -> dict:
    try:
        return json.loads((cm.get("data") or {}).get(key) or "{}")
    except json.JSONDecodeError:
        return {}


def inject_metrics_aggregation(pod: dict, cm: dict) -> None:
    cfg = _cm_json(cm, "metricsAggregator")
    ann = pod["metadata"].setdefault("annotations", {})
    enable = ann.get(C.ENABLE_METRIC_AGGREGATION, cfg.get("enableMetricAggregation", "false"))
    scrape = ann.get(C.ENABLE_PROMETHEUS_SCRAPING, cfg.get("enablePrometheusScraping", "false"))
    if str(scrape).lower() == "true":
        ann.setdefault(C.PROMETHEUS_SCRAPE, "true")
        ann.setdefault(C.PROMETHEUS_PORT, ann.get(C.CONTAINER_PROMETHEUS_PORT, str(C.DEFAULT_HTTP_PORT)))
        ann.setdefault(C.PROMETHEUS_PATH, ann.get(C.CONTAINER_PROMETHEUS_PATH, C.DEFAULT_PROMETHEUS_PATH))
    if str(enable).lower() == "true":
        port = ann.get(C.CONTAINER_PROMETHEUS_PORT, str(C.DEFAULT_HTTP_PORT))
        path = ann.get(C.CONTAINER_PROMETHEUS_PATH, C.DEFAULT_PROMETHEUS_PATH)
        for c in pod["spec"].get("containers") or []:
            if c.get("name") == C.MAIN_CONTAINER:
                env = c.setdefault("env", [])
                env.append({"name": "CONTAINER_PROMETHEUS_METRICS_PORT", "value": port})
                env.append({"name": "CONTAINER_PROMETHEUS_METRICS_PATH", "value": path})
        # no Knative queue-proxy to host the merge in raw / multi-node modes: add the aggregator
        # sidecar (ome_amd.metrics_aggregator) and point Prometheus at it
        names = {c.get("name") for c in pod["spec"].get("containers") or []}
        if "queue-proxy" not in names and "metrics-aggregator" not in names:
            agg = str(cfg.get("aggregatePort", 9088))
            pod["spec"].setdefault("containers", []).append({
                "name": "metrics-aggregator", "image": cfg.get("image", "ome-amd/metrics-aggregator:latest"),
                "command": ["python", "-m", "ome_amd.metrics_aggregator"],
                "env": [{"name": "AGGREGATE_PROMETHEUS_METRICS_PORT", "value": agg},
                        {"name": "CONTAINER_PROMETHEUS_METRICS_PORT", "value": port},
                        {"name": "CONTAINER_PROMETHEUS_METRICS_PATH", "value": path},
                        {"name": "QUEUE_PROXY_METRICS_PORT", "value": ""}],
                "ports": [{"containerPort": int(agg), "name": "agg-metrics"}],
                "resources": {"requests": {"cpu": "50m", "memory": "64Mi"}, "limits": {"cpu": "200m", "memory": "256Mi"}}})
            if str(scrape).lower() == "true":
                ann[C.PROMETHEUS_PORT] = agg


def inject_model_init(pod: dict, cm: dict) -> None:
    ann = pod["metadata"].get("annotations") or {}
    if ann.get(C.MODEL_INIT_INJECTION) != "true":
        return
    cfg = _cm_json(cm, "modelInit")
    main = next((c for c in pod["spec"].get("containers") or [] if c.get("name") == C.MAIN_CONTAINER), None)
    model_path = None
    for e in (main or {}).get("env") or []:
        if e.get("name") == C.MODEL_PATH_ENV:
            model_path = e.get("value")
    env = [{"name": "MODEL_NAME", "value": ann.get(C.BASE_MODEL_NAME_ANN, "")},
           {"name": "LOCAL_PATH", "value": model_path or "/mnt/models"}]
    if ann.get(C.DISABLE_MODEL_DECRYPTION) != "true":
        env += [{"name": "DECRYPTION_KEY_NAME", "value": ann.get(C.BASE_MODEL_DECRYPTION_KEY, "")},
                {"name": "DECRYPTION_SECRET_NAME", "value": ann.get(C.BASE_MODEL_DECRYPTION_SECRET, "")}]
    gpus = 0
    for c in pod["spec"].get("containers") or []:
        for n in C.GPU_RESOURCE_NAMES:
            v = ((c.get("resources") or {}).get("limits") or {}).get(n)
            if v is not None:
                gpus += int(str(v))
    env.append({"name": "GPU_COUNT", "value": str(gpus)})  # never panics when no GPU limit is set
    init = {"name": C.MODEL_INIT_CONTAINER, "image": cfg.get("image", "ome-amd/ome-agent:latest"),
            "command": ["python", "-m", "ome_amd.agent", "enigma"], "env": env,
            "resources": {"requests": {"cpu": cfg.get("cpuRequest", "4"), "memory": cfg.get("memoryRequest", "16Gi")},
                          "limits": {"cpu": cfg.get("cpuLimit", "4"), "memory": cfg.get("memoryLimit", "16Gi")}}}
    inits = pod["spec"].setdefault("initContainers", [])
    if not any(c.get("name") == C.MODEL_INIT_CONTAINER for c in inits):
        inits.append(init)


def inject_ft_adapter(pod: dict, cm: dict) -> None:
    ann = pod["metadata"].get("annotations") or {}
    ft = ann.get(C.FT_ADAPTER_INJECTION)
    if not ft:
        return
    inits = pod["spec"].setdefault("initContainers", [])
    if any(c.get("name") == C.FT_ADAPTER_CONTAINER for c in inits):
        return
    inits.append({"name": C.FT_ADAPTER_CONTAINER, "image": _cm_json(cm, "modelInit").get("image", "ome-amd/ome-agent"),
                  "command": ["python", "-m", "ome_amd.agent", "fine-tuned-adapter"],
                  "env": [{"name": "FINE_TUNED_WEIGHT_NAME", "value": ft}],
                  "volumeMounts": [{"name": "model-empty-dir", "mountPath": "/mnt/finetuned/download"}]})


def inject_serving_sidecar(pod: dict, cm: dict) -> None:
    ann = pod["metadata"].get("annotations") or {}
    if ann.get(C.SERVING_SIDECAR_INJECTION) != "true":
        return
    cs = pod["spec"].setdefault("containers", [])
    if any(c.get("name") == C.SERVING_SIDECAR_CONTAINER for c in cs):
        return
    cs.append({"name": C.SERVING_SIDECAR_CONTAINER, "image": _cm_json(cm, "modelInit").get("image", "ome-amd/ome-agent"),
               "command": ["python", "-m", "ome_amd.agent", "serving-agent"],
               "volumeMounts": [{"name": "model-empty-dir", "mountPath": "/mnt/finetuned"}]})


def inject_interconnect(pod: dict, cm: dict) -> None:
    ann = pod["metadata"].get("annotations") or {}
    if ann.get(C.RDMA_AUTO_INJECT) != "true":
        return
    pname = ann.get(C.RDMA_PROFILE) or DEFAULT_INTERCONNECT_PROFILE
    prof = INTERCONNECT_PROFILES.get(pname)
    if prof is None:
        raise Invalid(f"unknown RDMA profile: {pname}")
    target = ann.get(C.RDMA_CONTAINER_NAME) or C.MAIN_CONTAINER
    c = next((c for c in pod["spec"].get("containers") or [] if c.get("name") == target), None)
    if c is None:
        return
    vols = pod["spec"].setdefault("volumes", [])
    for v in prof["volumes"]:
        if not any(x.get("name") == v["name"] for x in vols):
            vols.append(dict(v))
    env = c.setdefault("env", [])
    for k in sorted(prof["env"]):
        env.append({"name": k, "value": prof["env"][k]})
    vms = c.setdefault("volumeMounts", [])
    for m in prof["mounts"]:
        if not any(x.get("name") == m["name"] for x in vms):
            vms.append(dict(m))
    c["securityContext"] = {**(c.get("securityContext") or {}), **prof["securityContext"]}


def mutate_pod(op, obj, old, store: Store):
    if op != "CREATE":
        return None
    lab = obj.get("metadata", {}).get("labels") or {}
    if C.ISVC_LABEL not in lab:
        return None
    cm = store.try_get("v1", "ConfigMap", C.INFERENCESERVICE_CONFIGMAP, C.OME_NAMESPACE) or {}
    for fn in (inject_metrics_aggregation, inject_model_init, inject_ft_adapter, inject_serving_sidecar,
               inject_interconnect):
        fn(obj, cm)
    inits = obj["spec"].get("initContainers")
    if inits:
        order = {C.MODEL_INIT_CONTAINER: 0, C.FT_ADAPTER_CONTAINER: 1}
        inits.sort(key=lambda c: order.get(c.get("name"), 2))
    return obj


def install(store: Store) -> None:
    """Register the webhook chain on a store (``cmd/manager/main.go:309-347``)."""
    store.add_mutating(default_isvc, ["InferenceService"])
    store.add_mutating(default_benchmark, ["BenchmarkJob"])
    store.add_mutating(mutate_pod, ["Pod"])
    store.add_validating(validate_isvc, ["InferenceService"])
    store.add_validating(validate_runtime, ["ServingRuntime", "ClusterServingRuntime"])
    store.add_validating(validate_benchmark, ["BenchmarkJob"])


__all__ = ["install", "Forbidden", "Invalid"]

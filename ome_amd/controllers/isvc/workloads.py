"""Workload object builders + create/update reconciliation for ISVC components.

Raw:        Deployment + Service + HPA | KEDA ScaledObject | none (external) + PDB
            (``reconcilers/{raw,deployment,service,autoscaler,hpa,keda,pdb}``)
MultiNode:  LeaderWorkerSet ``lws-<name>`` (size = workers + 1, LeaderCreated startup,
            RecreateGroupOnPodRestart) + Service selecting the leader (``reconcilers/lws``)
RayVLLM:    one RayCluster per replica + head Service + multinode-prober Deployment, with the
            unavailable-since self-heal (``reconcilers/multinodevllm``)
Serverless: Knative Service (``reconcilers/knative``)
Router RBAC, Ingress / HTTPRoute / VirtualService, external Service and the ModelConfig
ConfigMap live here too.
"""
from __future__ import annotations

import copy
import json
import time

from ome_amd.api import constants as C
from ome_amd.controllers.config import ControllerConfig, IngressConfig, render_template
from ome_amd.store.store import Store, owner_ref

DEPLOYMENT_API = "apps/v1"


def truncate(name: str, n: int = 63) -> str:
    return C.truncate_name(name, n)


def ensure(store: Store, desired: dict, owner: dict | None, ignore_spec_fields=(), compare_status=False) -> dict:
    """Create the object, or update it when its spec / labels / annotations drifted."""
    if owner is not None:
        desired.setdefault("metadata", {})["ownerReferences"] = [owner_ref(owner)]
    m = desired["metadata"]
    cur = store.try_get(desired["apiVersion"], desired["kind"], m["name"], m.get("namespace"))
    if cur is None:
        return store.create(desired)
    new = copy.deepcopy(cur)
    changed = False
    for f, v in desired.items():
        if f in ("metadata", "status", "apiVersion", "kind"):
            continue
        if f == "spec" and ignore_spec_fields:
            v = copy.deepcopy(v)
            for ig in ignore_spec_fields:
                if ig in cur.get("spec", {}):
                    v[ig] = cur["spec"][ig]
                else:
                    v.pop(ig, None)
        if new.get(f) != v:
            new[f] = copy.deepcopy(v)
            changed = True
    for f in ("labels", "annotations", "ownerReferences"):
        want = m.get(f)
        if want is not None and new["metadata"].get(f) != want:
            new["metadata"][f] = want
            changed = True
    return store.update(new) if changed else cur


def delete_if_exists(store: Store, api: str, kind: str, name: str, ns: str | None) -> bool:
    return store.delete(api, kind, name, ns, ignore_missing=True) is not None


# ------------------------------------------------------------------ pod defaults
def set_default_pod_spec(ps: dict) -> dict:
    ps.setdefault("dnsPolicy", "ClusterFirst")
    ps.setdefault("restartPolicy", "Always")
    ps.setdefault("terminationGracePeriodSeconds", 30)
    ps.setdefault("securityContext", {})
    ps.setdefault("schedulerName", "default-scheduler")
    for c in ps.get("containers") or []:
        c.setdefault("terminationMessagePath", "/dev/termination-log")
        c.setdefault("terminationMessagePolicy", "File")
        c.setdefault("imagePullPolicy", "IfNotPresent")
        if c.get("name") == C.MAIN_CONTAINER and "readinessProbe" not in c:
            port = (c.get("ports") or [{}])[0].get("containerPort", C.DEFAULT_HTTP_PORT)
            c["readinessProbe"] = {"tcpSocket": {"port": port}, "timeoutSeconds": 1, "periodSeconds": 10,
                                   "successThreshold": 1, "failureThreshold": 3}
    return ps


POD_ONLY_ANNOTATIONS = (C.PROMETHEUS_SCRAPE, C.PROMETHEUS_PORT, C.PROMETHEUS_PATH, C.RDMA_AUTO_INJECT,
                        C.RDMA_PROFILE, C.RDMA_CONTAINER_NAME, C.MODEL_INIT_INJECTION, C.FT_ADAPTER_INJECTION,
                        C.SERVING_SIDECAR_INJECTION)


def _meta(meta: dict, name: str | None = None) -> dict:
    m = {"name": name or meta["name"], "namespace": meta["namespace"], "labels": dict(meta.get("labels") or {}),
         "annotations": dict(meta.get("annotations") or {})}
    return m


# ------------------------------------------------------------------ Raw
def build_deployment(meta: dict, pod_spec: dict, ext: dict) -> dict:
    app = truncate(meta["name"])
    pod_meta = _meta(meta)
    pod_meta["labels"]["app"] = app
    pod_meta.pop("name")
    pod_meta.pop("namespace")
    spec = {
        "selector": {"matchLabels": {"app": app}},
        "template": {"metadata": pod_meta, "spec": set_default_pod_spec(copy.deepcopy(pod_spec))},
        "replicas": max(int(ext.get("minReplicas") if ext.get("minReplicas") is not None else 1), 1),
        "strategy": copy.deepcopy(ext.get("deploymentStrategy") or
                                  {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": 0, "maxSurge": 1}}),
        "revisionHistoryLimit": 10,
        "progressDeadlineSeconds": 600,
    }
    dm = _meta(meta)
    dm["labels"]["app"] = app
    return {"apiVersion": DEPLOYMENT_API, "kind": "Deployment", "metadata": dm, "spec": spec}


def build_service(meta: dict, pod_spec: dict, selector: dict | None = None, name: str | None = None) -> dict:
    sm = _meta(meta, name)
    sm["annotations"] = {k: v for k, v in sm["annotations"].items() if k not in POD_ONLY_ANNOTATIONS}
    sm["name"] = truncate(sm["name"])
    ports = []
    c0 = (pod_spec.get("containers") or [{}])[0]
    for p in c0.get("ports") or []:
        ports.append({"name": p.get("name"), "port": p["containerPort"], "targetPort": p["containerPort"],
                      "protocol": p.get("protocol", "TCP")})
    if not ports:
        ports = [{"name": c0.get("name"), "port": C.DEFAULT_HTTP_PORT, "targetPort": C.DEFAULT_HTTP_PORT,
                  "protocol": "TCP"}]
    stype = (meta.get("annotations") or {}).get(C.SERVICE_TYPE, "ClusterIP")
    if stype not in ("ClusterIP", "LoadBalancer", "NodePort"):
        stype = "ClusterIP"
    spec = {"type": stype, "selector": selector or {"app": truncate(meta["name"])}, "ports": ports}
    lb = (meta.get("annotations") or {}).get(C.LOAD_BALANCER_IP)
    if stype == "LoadBalancer" and lb:
        spec["loadBalancerIP"] = lb
    return {"apiVersion": "v1", "kind": "Service", "metadata": sm, "spec": spec}


def autoscaler_class(meta: dict) -> str:
    return (meta.get("annotations") or {}).get(C.AUTOSCALER_CLASS, C.AUTOSCALER_HPA)


def build_hpa(meta: dict, ext: dict) -> dict:
    mn = ext.get("minReplicas")
    mn = 1 if mn is None or mn < 1 else int(mn)
    mx = max(int(ext.get("maxReplicas") or 0), mn)
    ann = meta.get("annotations") or {}
    util = int(ann.get(C.TARGET_UTILIZATION) or ext.get("scaleTarget") or C.DEFAULT_CPU_UTILIZATION)
    res = ext.get("scaleMetric") if ext.get("scaleMetric") in C.AUTOSCALER_METRICS_ALLOWED else "cpu"
    return {"apiVersion": "autoscaling/v2", "kind": "HorizontalPodAutoscaler", "metadata": _meta(meta),
            "spec": {"scaleTargetRef": {"apiVersion": DEPLOYMENT_API, "kind": "Deployment", "name": meta["name"]},
                     "minReplicas": mn, "maxReplicas": mx,
                     "metrics": [{"type": "Resource", "resource": {"name": res, "target": {
                         "type": "Utilization", "averageUtilization": util}}}]}}


def keda_query(name: str, keda: dict | None) -> str:
    if keda and keda.get("customPromQuery"):
        q = keda["customPromQuery"]
        return q % name if "%s" in q else q
    # default query over the runtime's vLLM-compatible metric names (keda_reconciler.go:197-222)
    return (f'sum(avg_over_time(vllm:avg_generation_throughput_toks_per_s{{ome_io_inferenceservice="{name}"}}[5m])'
            f' < bool 10) * sum(rate(vllm:request_success_total{{ome_io_inferenceservice="{name}"}}[1m]) > bool 0.50)')


def build_scaled_object(meta: dict, ext: dict, isvc_keda: dict | None, defaults) -> dict:
    ann = meta.get("annotations") or {}
    k = {**{"promServerAddress": defaults.promServerAddress, "scalingThreshold": defaults.scalingThreshold,
            "scalingOperator": "LessThanOrEqual"}, **(isvc_keda or {}), **(ext.get("kedaConfig") or {})}
    mn = ext.get("minReplicas")
    mn = 1 if mn is None else int(mn)
    mx = max(int(ext.get("maxReplicas") or 0), mn)
    trig = {"type": "prometheus", "metadata": {
        "serverAddress": ann.get(C.KEDA_SERVER_ADDRESS, k["promServerAddress"]),
        "query": ann.get(C.KEDA_QUERY, keda_query(meta["name"], k)),
        "threshold": ann.get(C.KEDA_THRESHOLD, str(k["scalingThreshold"])),
        "operator": ann.get(C.KEDA_OPERATOR, k["scalingOperator"])}}
    if k.get("authenticationRef"):
        trig["authenticationRef"] = k["authenticationRef"]
    if k.get("authModes"):
        trig["metadata"]["authModes"] = k["authModes"]
    return {"apiVersion": "keda.sh/v1alpha1", "kind": "ScaledObject", "metadata": _meta(meta),
            "spec": {"scaleTargetRef": {"name": meta["name"]}, "minReplicaCount": mn, "maxReplicaCount": mx,
                     "triggers": [trig]}}


def build_pdb(meta: dict, ext: dict) -> dict | None:
    if ext.get("minAvailable") is None and ext.get("maxUnavailable") is None:
        return None
    spec = {"selector": {"matchLabels": {"app": truncate(meta["name"])}}}
    if ext.get("minAvailable") is not None:
        spec["minAvailable"] = ext["minAvailable"]
    else:
        spec["maxUnavailable"] = ext["maxUnavailable"]
    return {"apiVersion": "policy/v1", "kind": "PodDisruptionBudget", "metadata": _meta(meta), "spec": spec}


def reconcile_raw(store: Store, isvc: dict, meta: dict, pod_spec: dict, ext: dict, cfg: ControllerConfig) -> dict:
    dep = build_deployment(meta, pod_spec, ext)
    ns, name = meta["namespace"], meta["name"]
    cls = autoscaler_class(meta)
    if cls in (C.AUTOSCALER_HPA, C.AUTOSCALER_EXTERNAL):
        delete_if_exists(store, "keda.sh/v1alpha1", "ScaledObject", name, ns)
        if cls == C.AUTOSCALER_HPA:
            ensure(store, build_hpa(meta, ext), isvc)
        else:
            delete_if_exists(store, "autoscaling/v2", "HorizontalPodAutoscaler", name, ns)
    elif cls == C.AUTOSCALER_KEDA:
        delete_if_exists(store, "autoscaling/v2", "HorizontalPodAutoscaler", name, ns)
        ensure(store, build_scaled_object(meta, ext, (isvc.get("spec") or {}).get("kedaConfig"), cfg.keda), isvc)
    else:
        raise ValueError(f"unknown autoscaler class type: {cls}")
    # replicas are owned by the autoscaler once the Deployment exists
    d = ensure(store, dep, isvc, ignore_spec_fields=("replicas",))
    ensure(store, build_service(meta, pod_spec), isvc)
    pdb = build_pdb(meta, ext)
    if pdb is not None:
        ensure(store, pdb, isvc)
    else:
        delete_if_exists(store, "policy/v1", "PodDisruptionBudget", name, ns)
    return d


# ------------------------------------------------------------------ MultiNode (LWS)
def build_lws(meta: dict, leader_ps: dict, worker_ps: dict | None, worker_size: int, ext: dict) -> dict:
    name = C.lws_name(meta["name"])
    pod_meta = _meta(meta)
    pod_meta.pop("name")
    pod_meta.pop("namespace")
    leader_meta = copy.deepcopy(pod_meta)
    leader_meta["labels"][C.RAY_NODE_TYPE_LABEL] = "head"
    worker_meta = copy.deepcopy(pod_meta)
    worker_meta["annotations"] = {k: v for k, v in worker_meta["annotations"].items()
                                  if not k.startswith("prometheus.io/")}
    replicas = ext.get("minReplicas")
    replicas = 1 if replicas is None else int(replicas)
    spec = {
        "replicas": replicas,
        "startupPolicy": "LeaderCreated",
        "rolloutStrategy": {"type": "RollingUpdate", "rollingUpdateConfiguration": {"maxSurge": 1,
                                                                                     "maxUnavailable": 1}},
        "networkConfig": {"subdomainPolicy": "Shared"},
        "leaderWorkerTemplate": {
            "size": worker_size + 1,
            "restartPolicy": "RecreateGroupOnPodRestart",
            "leaderTemplate": {"metadata": leader_meta, "spec": set_default_pod_spec(copy.deepcopy(leader_ps))},
            "workerTemplate": {"metadata": worker_meta,
                               "spec": set_default_pod_spec(copy.deepcopy(worker_ps or leader_ps))},
        },
    }
    lm = _meta(meta, name)
    return {"apiVersion": "leaderworkerset.x-k8s.io/v1", "kind": "LeaderWorkerSet", "metadata": lm, "spec": spec}


def reconcile_multinode(store: Store, isvc: dict, meta: dict, leader_ps: dict, worker_ps: dict | None,
                        worker_size: int, ext: dict) -> dict:
    lws = ensure(store, build_lws(meta, leader_ps, worker_ps, worker_size, ext), isvc)
    sel = {C.LWS_NAME_LABEL: lws["metadata"]["name"], C.RAY_NODE_TYPE_LABEL: "head"}
    ensure(store, build_service(meta, leader_ps, selector=sel), isvc)
    if (meta.get("labels") or {}).get(C.ISTIO_SIDECAR_INJECT) == "true":
        ensure(store, {"apiVersion": "networking.istio.io/v1beta1", "kind": "Sidecar",
                       "metadata": _meta(meta),
                       "spec": {"workloadSelector": {"labels": {C.LWS_NAME_LABEL: lws["metadata"]["name"]}},
                                "outboundTrafficPolicy": {"mode": "ALLOW_ANY"}}}, isvc)
    return lws


# ------------------------------------------------------------------ MultiNodeRayVLLM
def reconcile_ray(store: Store, isvc: dict, meta: dict, head_ps: dict, ext: dict, cfg: ControllerConfig,
                  now: float | None = None) -> tuple[list[dict], float | None]:
    """One RayCluster per replica + head Service + prober Deployment; self-heal when the prober
    stays unavailable past ``unavailableThresholdSeconds`` while Ray claims Ready (``ray.go:107-233``).
    Returns (prober deployments, requeue_after)."""
    now = now or time.time()
    replicas = ext.get("minReplicas")
    replicas = 1 if replicas is None else int(replicas)
    probers, requeue = [], None
    for i in range(replicas):
        name = C.ray_head_service_name(meta["name"], i)
        head = copy.deepcopy(head_ps)
        for c in head.get("containers") or []:
            c.setdefault("lifecycle", {"preStop": {"exec": {"command": ["/bin/sh", "-c", "ray stop"]}}})
        worker = copy.deepcopy(head_ps)
        for c in worker.get("containers") or []:
            c["command"] = ["/bin/sh", "-c", "$KUBERAY_GEN_RAY_START_CMD"]
            c.pop("args", None)
        rc = {"apiVersion": "ray.io/v1", "kind": "RayCluster", "metadata": _meta(meta, name),
              "spec": {"headGroupSpec": {"rayStartParams": {"dashboard-host": "0.0.0.0"},
                                         "template": {"spec": set_default_pod_spec(head)}},
                       "workerGroupSpecs": [{"groupName": "worker", "replicas": 1, "minReplicas": 1,
                                             "maxReplicas": 1, "rayStartParams": {},
                                             "template": {"spec": set_default_pod_spec(worker)}}]}}
        cur = store.try_get("ray.io/v1", "RayCluster", name, meta["namespace"])
        mnp_name = f"{name}-mnp"
        mnp = store.try_get(DEPLOYMENT_API, "Deployment", mnp_name, meta["namespace"])
        if cur is not None and mnp is not None:
            unavailable = not _deployment_available(mnp)
            ray_ready = (cur.get("status") or {}).get("state") == "ready"
            since = (cur["metadata"].get("annotations") or {}).get(C.RAY_UNAVAILABLE_SINCE)
            if unavailable and ray_ready:
                if since is None:
                    ann = dict(cur["metadata"].get("annotations") or {})
                    ann[C.RAY_UNAVAILABLE_SINCE] = str(now)
                    store.patch("ray.io/v1", "RayCluster", name, {"metadata": {"annotations": ann}},
                                meta["namespace"])
                    requeue = 10.0
                elif now - float(since) > cfg.prober.unavailableThresholdSeconds:
                    store.delete("ray.io/v1", "RayCluster", name, meta["namespace"])
                    cur = None
                else:
                    requeue = 10.0
            elif since is not None and not unavailable:
                ann = dict(cur["metadata"].get("annotations") or {})
                ann.pop(C.RAY_UNAVAILABLE_SINCE, None)
                store.patch("ray.io/v1", "RayCluster", name, {"metadata": {"annotations": {C.RAY_UNAVAILABLE_SINCE: None}}},
                            meta["namespace"])
        rc_meta_ann = (cur or {}).get("metadata", {}).get("annotations") if cur else None
        if rc_meta_ann:
            rc["metadata"]["annotations"].update({k: v for k, v in rc_meta_ann.items() if k == C.RAY_UNAVAILABLE_SINCE})
        ensure(store, rc, isvc)
        head_svc = build_service(meta, head_ps, selector={"ray.io/cluster": name, C.RAY_NODE_TYPE_LABEL: "head"},
                                 name=f"{name}-head")
        ensure(store, head_svc, isvc)
        probers.append(ensure(store, build_prober_deployment(meta, name, head_ps, cfg), isvc))
    return probers, requeue


def _deployment_available(d: dict) -> bool:
    for c in (d.get("status") or {}).get("conditions") or []:
        if c.get("type") == "Available":
            return c.get("status") == "True"
    return False


def build_prober_deployment(meta: dict, cluster: str, head_ps: dict, cfg: ControllerConfig) -> dict:
    port = ((head_ps.get("containers") or [{}])[0].get("ports") or [{"containerPort": C.DEFAULT_HTTP_PORT}])[0]
    port = port.get("containerPort", C.DEFAULT_HTTP_PORT)
    endpoint = f"http://{cluster}-head.{meta['namespace']}.svc.cluster.local:{port}"
    p = cfg.prober
    c = {"name": C.MULTINODE_PROBER_CONTAINER, "image": p.image,
         "command": ["python", "-m", "ome_amd.prober"],
         "args": ["--addr", ":8080", "--vllm-endpoint", endpoint],
         "ports": [{"containerPort": 8080, "name": "prober"}],
         "resources": {"requests": {"cpu": p.cpuRequest, "memory": p.memoryRequest},
                       "limits": {"cpu": p.cpuLimit, "memory": p.memoryLimit}},
         "startupProbe": {"httpGet": {"path": "/startupz", "port": 8080},
                          "failureThreshold": p.startupFailureThreshold, "periodSeconds": p.startupPeriodSeconds,
                          "timeoutSeconds": p.startupTimeoutSeconds,
                          "initialDelaySeconds": p.startupInitialDelaySeconds},
         "readinessProbe": {"httpGet": {"path": "/readyz", "port": 8080}},
         "livenessProbe": {"httpGet": {"path": "/healthz", "port": 8080}}}
    pm = {"name": f"{cluster}-mnp", "namespace": meta["namespace"], "labels": {"app": f"{cluster}-mnp"},
          "annotations": {}}
    return build_deployment(pm, {"containers": [c]}, {"minReplicas": 1})


# ------------------------------------------------------------------ Serverless
def build_ksvc(meta: dict, pod_spec: dict, ext: dict) -> dict:
    ann = dict(meta.get("annotations") or {})
    if ext.get("minReplicas") is not None:
        ann["autoscaling.knative.dev/min-scale"] = str(ext["minReplicas"])
    if ext.get("maxReplicas"):
        ann["autoscaling.knative.dev/max-scale"] = str(ext["maxReplicas"])
    if ext.get("scaleTarget"):
        ann["autoscaling.knative.dev/target"] = str(ext["scaleTarget"])
    if ext.get("scaleMetric"):
        ann["autoscaling.knative.dev/metric"] = str(ext["scaleMetric"])
    tmpl_spec = copy.deepcopy(pod_spec)
    if ext.get("containerConcurrency") is not None:
        tmpl_spec["containerConcurrency"] = ext["containerConcurrency"]
    if ext.get("timeoutSeconds") is not None:
        tmpl_spec["timeoutSeconds"] = ext["timeoutSeconds"]
    spec = {"template": {"metadata": {"labels": dict(meta.get("labels") or {}), "annotations": ann},
                         "spec": tmpl_spec}}
    if ext.get("canaryTrafficPercent") is not None:
        spec["traffic"] = [{"latestRevision": True, "percent": ext["canaryTrafficPercent"]}]
    return {"apiVersion": "serving.knative.dev/v1", "kind": "Service", "metadata": _meta(meta), "spec": spec}


# ------------------------------------------------------------------ Router RBAC
def reconcile_router_rbac(store: Store, isvc: dict, meta: dict) -> str:
    name, ns = meta["name"], meta["namespace"]
    ensure(store, {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": name, "namespace": ns}}, isvc)
    ensure(store, {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                   "metadata": {"name": name, "namespace": ns},
                   "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "list", "watch"]}]}, isvc)
    ensure(store, {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                   "metadata": {"name": name, "namespace": ns},
                   "subjects": [{"kind": "ServiceAccount", "name": name, "namespace": ns}],
                   "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": name}}, isvc)
    return name


# ------------------------------------------------------------------ ingress / URLs
def domain_name(name: str, meta: dict, ic: IngressConfig) -> str:
    vals = {"Name": name, "Namespace": meta.get("namespace", ""), "IngressDomain": ic.ingressDomain,
            "Annotations": meta.get("annotations") or {}, "Labels": meta.get("labels") or {}}
    return render_template(ic.domainTemplate, vals)


def url_path(isvc: dict, ic: IngressConfig) -> str:
    if not ic.pathTemplate:
        return ""
    m = isvc["metadata"]
    return render_template(ic.pathTemplate, {"Name": m["name"], "Namespace": m["namespace"]})


def entrypoint_component(isvc_spec: dict) -> str:
    # a component present with an empty spec (``router: {}``) still exists (the reference tests
    # ``Spec.Router != nil``)
    if isvc_spec.get("router") is not None:
        return C.ROUTER
    if isvc_spec.get("decoder") is not None:
        return C.DECODER
    return C.ENGINE


def reconcile_ingress(store: Store, isvc: dict, ic: IngressConfig, mode: str, entry_service: str) -> dict:
    """Returns the IngressReady condition.  Serverless -> VirtualService; Raw/MultiNode ->
    Ingress or Gateway-API HTTPRoute (``reconcilers/ingress``)."""
    m = isvc["metadata"]
    if ic.disableIngressCreation:
        return {"type": "IngressReady", "status": "True", "reason": "IngressDisabled",
                "message": "Ingress creation is disabled"}
    host = domain_name(m["name"], m, ic)
    path = url_path(isvc, ic) or "/"
    hosts = [host] + list(ic.additionalIngressDomains or [])
    backend_port = C.DEFAULT_HTTP_PORT
    if mode == C.DeploymentMode.SERVERLESS:
        if not ic.disableIstioVirtualHost:
            vs = {"apiVersion": "networking.istio.io/v1beta1", "kind": "VirtualService",
                  "metadata": {"name": m["name"], "namespace": m["namespace"]},
                  "spec": {"hosts": hosts, "gateways": [ic.ingressGateway, ic.localGateway],
                           "http": [{"match": [{"uri": {"prefix": path}}],
                                     "route": [{"destination": {"host": f"{entry_service}.{m['namespace']}.svc.cluster.local",
                                                                "port": {"number": 80}}}]}]}}
            ensure(store, vs, isvc)
    elif ic.enableGatewayAPI:
        gw_ns, _, gw = (ic.omeIngressGateway or "ome/ome-gateway").partition("/")
        route = {"apiVersion": "gateway.networking.k8s.io/v1", "kind": "HTTPRoute",
                 "metadata": {"name": m["name"], "namespace": m["namespace"]},
                 "spec": {"parentRefs": [{"name": gw or gw_ns, "namespace": gw_ns if gw else m["namespace"]}],
                          "hostnames": hosts,
                          "rules": [{"matches": [{"path": {"type": "PathPrefix", "value": path}}],
                                     "backendRefs": [{"name": entry_service, "port": backend_port}]}]}}
        ensure(store, route, isvc)
    else:
        ing = {"apiVersion": "networking.k8s.io/v1", "kind": "Ingress",
               "metadata": {"name": m["name"], "namespace": m["namespace"]},
               "spec": {"ingressClassName": ic.ingressClassName,
                        "rules": [{"host": h, "http": {"paths": [{"path": path, "pathType": "Prefix", "backend": {
                            "service": {"name": entry_service, "port": {"number": backend_port}}}}]}} for h in hosts]}}
        ensure(store, ing, isvc)
    return {"type": "IngressReady", "status": "True", "reason": "", "message": ""}


def reconcile_external_service(store: Store, isvc: dict, entry_component: str, ic: IngressConfig) -> dict | None:
    """``<isvc>`` Service selecting the entrypoint component when ingress creation is disabled."""
    m = isvc["metadata"]
    if not ic.disableIngressCreation:
        delete_if_exists(store, "v1", "Service", m["name"], m["namespace"])
        return None
    comp_name = C.component_name(m["name"], entry_component)
    svc = {"apiVersion": "v1", "kind": "Service",
           "metadata": {"name": m["name"], "namespace": m["namespace"],
                        "labels": {C.ISVC_LABEL: m["name"]}},
           "spec": {"type": "ClusterIP", "selector": {"app": truncate(comp_name)},
                    "ports": [{"name": "http", "port": C.DEFAULT_HTTP_PORT, "targetPort": C.DEFAULT_HTTP_PORT,
                               "protocol": "TCP"}]}}
    return ensure(store, svc, isvc)


def reconcile_modelconfig(store: Store, isvc: dict, base_model_name: str, base_spec: dict,
                          ft_specs: list[dict] | None = None) -> dict:
    m = isvc["metadata"]
    entry = {"modelName": base_model_name, "modelSpec": {k: v for k, v in base_spec.items()
                                                         if k in ("storage", "modelFormat", "modelType",
                                                                  "modelArchitecture", "modelParameterSize")}}
    if ft_specs:
        entry["fineTunedWeightSpec"] = ft_specs[0]
    cm = {"apiVersion": "v1", "kind": "ConfigMap",
          "metadata": {"name": C.modelconfig_name(m["name"]), "namespace": m["namespace"],
                       "labels": {C.ISVC_LABEL: m["name"]}},
          "data": {"models.json": json.dumps([entry], sort_keys=True)}}
    return ensure(store, cm, isvc)

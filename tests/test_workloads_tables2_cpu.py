"""More workload / routing tables (the reference's ``reconcilers/{multinode,knative,ingress,
rbac}`` and ``utils`` cases): LeaderWorkerSet shape, Knative Service autoscaling annotations and
traffic, ingress objects per mode (Istio VirtualService, Gateway-API HTTPRoute, Ingress; hosts,
paths, additional domains, disabled creation), the external Service of a disabled ingress, the
entrypoint component, and the router's RBAC objects."""
import dataclasses

import pytest

from ome_amd.api import constants as C
from ome_amd.controllers.config import ControllerConfig
from ome_amd.controllers.isvc import workloads as W
from ome_amd.store.store import Store

META = {"name": "ds-engine", "namespace": "team", "labels": {"app.kubernetes.io/name": "ds"},
        "annotations": {"prometheus.io/scrape": "true", "keep": "1"}}
LEADER = {"containers": [{"name": "leader", "image": "img", "ports": [{"containerPort": 8080, "name": "http"}]}]}
WORKER = {"containers": [{"name": "worker", "image": "img"}]}


def _isvc(st, spec=None):
    return st.create({"apiVersion": C.API_VERSION, "kind": "InferenceService",
                      "metadata": {"name": "ds", "namespace": "team", "uid": "u1"}, "spec": spec or {}})


def _ic(**kw):
    return dataclasses.replace(ControllerConfig.from_store(Store()).ingress, **kw)


# ------------------------------------------------------------------ LeaderWorkerSet
@pytest.mark.parametrize("size,ext,replicas", [(1, {}, 1), (3, {"minReplicas": 2}, 2), (0, {"minReplicas": 0}, 0)])
def test_lws_shape(size, ext, replicas):
    lws = W.build_lws(META, LEADER, WORKER, size, ext)
    sp = lws["spec"]
    t = sp["leaderWorkerTemplate"]
    assert lws["metadata"]["name"] == C.lws_name("ds-engine") and sp["replicas"] == replicas
    assert t["size"] == size + 1 and t["restartPolicy"] == "RecreateGroupOnPodRestart"
    assert sp["startupPolicy"] == "LeaderCreated" and sp["networkConfig"] == {"subdomainPolicy": "Shared"}
    assert t["leaderTemplate"]["metadata"]["labels"][C.RAY_NODE_TYPE_LABEL] == "head"
    assert C.RAY_NODE_TYPE_LABEL not in t["workerTemplate"]["metadata"]["labels"]
    # workers are not scraped: prometheus annotations stay on the leader only
    assert "prometheus.io/scrape" in t["leaderTemplate"]["metadata"]["annotations"]
    assert t["workerTemplate"]["metadata"]["annotations"] == {"keep": "1"}
    assert t["leaderTemplate"]["spec"]["containers"][0]["name"] == "leader"
    assert t["workerTemplate"]["spec"]["containers"][0]["name"] == "worker"


def test_lws_worker_defaults_to_leader_and_service_selects_head():
    lws = W.build_lws(META, LEADER, None, 1, {})
    assert lws["spec"]["leaderWorkerTemplate"]["workerTemplate"]["spec"]["containers"][0]["name"] == "leader"
    st = Store()
    isvc = _isvc(st)
    W.reconcile_multinode(st, isvc, META, LEADER, WORKER, 1, {})
    svc = st.get("v1", "Service", "ds-engine", "team")
    assert svc["spec"]["selector"] == {C.LWS_NAME_LABEL: C.lws_name("ds-engine"), C.RAY_NODE_TYPE_LABEL: "head"}


# ------------------------------------------------------------------ Knative Service
@pytest.mark.parametrize("ext,ann", [
    ({}, {}),
    ({"minReplicas": 0}, {"autoscaling.knative.dev/min-scale": "0"}),
    ({"minReplicas": 1, "maxReplicas": 4}, {"autoscaling.knative.dev/min-scale": "1",
                                            "autoscaling.knative.dev/max-scale": "4"}),
    ({"scaleTarget": 10, "scaleMetric": "concurrency"}, {"autoscaling.knative.dev/target": "10",
                                                         "autoscaling.knative.dev/metric": "concurrency"}),
    ({"maxReplicas": 0}, {}),                                   # 0 = unbounded: no max-scale
])
def test_ksvc_autoscaling_annotations(ext, ann):
    k = W.build_ksvc(META, LEADER, ext)
    got = {a: v for a, v in k["spec"]["template"]["metadata"]["annotations"].items()
           if a.startswith("autoscaling.knative.dev/")}
    assert got == ann and k["apiVersion"] == "serving.knative.dev/v1"


def test_ksvc_concurrency_timeout_and_canary():
    k = W.build_ksvc(META, LEADER, {"containerConcurrency": 4, "timeoutSeconds": 600, "canaryTrafficPercent": 10})
    t = k["spec"]["template"]["spec"]
    assert t["containerConcurrency"] == 4 and t["timeoutSeconds"] == 600
    assert k["spec"]["traffic"] == [{"latestRevision": True, "percent": 10}]
    assert "traffic" not in W.build_ksvc(META, LEADER, {})["spec"]


# ------------------------------------------------------------------ entrypoint + ingress
@pytest.mark.parametrize("spec,want", [({}, C.ENGINE), ({"engine": {}}, C.ENGINE), ({"engine": {}, "decoder": {}}, C.DECODER),
                                       ({"engine": {}, "decoder": {}, "router": {}}, C.ROUTER),
                                       ({"engine": {}, "router": {}}, C.ROUTER)])
def test_entrypoint_component(spec, want):
    assert W.entrypoint_component(spec) == want


@pytest.mark.parametrize("tmpl,want", [
    ("{{ .Name }}.{{ .Namespace }}.{{ .IngressDomain }}", "ds.team.example.com"),
    ("{{ .Name }}-{{ .Namespace }}.{{ .IngressDomain }}", "ds-team.example.com"),
    ("{{ .Name }}.{{ .IngressDomain }}", "ds.example.com"),
])
def test_domain_template(tmpl, want):
    ic = _ic(domainTemplate=tmpl, ingressDomain="example.com")
    assert W.domain_name("ds", {"namespace": "team"}, ic) == want


def test_ingress_disabled_and_external_service():
    st = Store()
    isvc = _isvc(st, {"engine": {}, "router": {}})
    ic = _ic(disableIngressCreation=True)
    cond = W.reconcile_ingress(st, isvc, ic, C.DeploymentMode.RAW, "ds-router")
    assert cond["reason"] == "IngressDisabled" and cond["status"] == "True"
    assert st.try_get("networking.k8s.io/v1", "Ingress", "ds", "team") is None
    svc = W.reconcile_external_service(st, isvc, C.ROUTER, ic)
    assert svc["spec"]["selector"] == {"app": C.component_name("ds", C.ROUTER)}
    assert svc["metadata"]["labels"] == {C.ISVC_LABEL: "ds"}
    # ingress enabled again: the external Service goes away
    assert W.reconcile_external_service(st, isvc, C.ROUTER, _ic(disableIngressCreation=False)) is None
    assert st.try_get("v1", "Service", "ds", "team") is None


@pytest.mark.parametrize("mode,kw,kind,api", [
    (C.DeploymentMode.RAW, {}, "Ingress", "networking.k8s.io/v1"),
    (C.DeploymentMode.MULTINODE, {}, "Ingress", "networking.k8s.io/v1"),
    (C.DeploymentMode.RAW, {"enableGatewayAPI": True, "omeIngressGateway": "gw-ns/gw"}, "HTTPRoute",
     "gateway.networking.k8s.io/v1"),
    (C.DeploymentMode.SERVERLESS, {}, "VirtualService", "networking.istio.io/v1beta1"),
])
def test_ingress_object_per_mode(mode, kw, kind, api):
    st = Store()
    isvc = _isvc(st)
    ic = _ic(disableIngressCreation=False, ingressDomain="example.com", additionalIngressDomains=["alt.example.com"],
             **kw)
    assert W.reconcile_ingress(st, isvc, ic, mode, "ds-engine")["status"] == "True"
    obj = st.get(api, kind, "ds", "team")
    sp = obj["spec"]
    if kind == "Ingress":
        assert [r["host"] for r in sp["rules"]] == ["ds.team.example.com", "alt.example.com"]
        b = sp["rules"][0]["http"]["paths"][0]
        assert b["path"] == "/" and b["backend"]["service"] == {"name": "ds-engine", "port": {"number": 8080}}
        assert sp["ingressClassName"] == ic.ingressClassName
    elif kind == "HTTPRoute":
        assert sp["parentRefs"] == [{"name": "gw", "namespace": "gw-ns"}]
        assert sp["hostnames"] == ["ds.team.example.com", "alt.example.com"]
        assert sp["rules"][0]["backendRefs"] == [{"name": "ds-engine", "port": 8080}]
    else:
        assert sp["hosts"] == ["ds.team.example.com", "alt.example.com"]
        assert sp["gateways"] == [ic.ingressGateway, ic.localGateway]
        assert sp["http"][0]["route"][0]["destination"]["host"] == "ds-engine.team.svc.cluster.local"


def test_ingress_path_template_and_istio_virtual_host_off():
    st = Store()
    isvc = _isvc(st)
    ic = _ic(disableIngressCreation=False, pathTemplate="/serving/{{ .Namespace }}/{{ .Name }}")
    W.reconcile_ingress(st, isvc, ic, C.DeploymentMode.RAW, "ds-engine")
    ing = st.get("networking.k8s.io/v1", "Ingress", "ds", "team")
    assert ing["spec"]["rules"][0]["http"]["paths"][0]["path"] == "/serving/team/ds"
    st2 = Store()
    isvc2 = _isvc(st2)
    W.reconcile_ingress(st2, isvc2, _ic(disableIngressCreation=False, disableIstioVirtualHost=True),
                        C.DeploymentMode.SERVERLESS, "ds-engine")
    assert st2.try_get("networking.istio.io/v1beta1", "VirtualService", "ds", "team") is None


# ------------------------------------------------------------------ router RBAC
def test_router_rbac_objects():
    st = Store()
    isvc = _isvc(st)
    name = W.reconcile_router_rbac(st, isvc, {"name": "ds-router", "namespace": "team"})
    assert name == "ds-router"
    role = st.get("rbac.authorization.k8s.io/v1", "Role", "ds-router", "team")
    assert role["rules"] == [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "list", "watch"]}]
    rb = st.get("rbac.authorization.k8s.io/v1", "RoleBinding", "ds-router", "team")
    assert rb["subjects"] == [{"kind": "ServiceAccount", "name": "ds-router", "namespace": "team"}]
    assert rb["roleRef"]["name"] == "ds-router"
    assert st.try_get("v1", "ServiceAccount", "ds-router", "team") is not None
    # idempotent
    W.reconcile_router_rbac(st, isvc, {"name": "ds-router", "namespace": "team"})

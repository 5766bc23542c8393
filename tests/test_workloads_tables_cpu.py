"""Raw-deployment workload builder tables (the reference's ``reconcilers/{deployment,service,hpa,
keda,pdb}`` test cases): Deployment replicas / strategy / labels, Service type / ports / load
balancer / annotation filtering, HPA bounds / metric / utilisation, KEDA ScaledObject defaults,
overrides, annotations and auth, PodDisruptionBudget, and the autoscaler-class switch of
``reconcile_raw`` (objects of the other class are removed)."""
import pytest

from ome_amd.api import constants as C
from ome_amd.controllers.config import ControllerConfig, KedaDefaults
from ome_amd.controllers.isvc import workloads as W
from ome_amd.store.store import Store

META = {"name": "llama-engine", "namespace": "team", "labels": {"app.kubernetes.io/name": "llama"},
        "annotations": {}}
POD = {"containers": [{"name": "ome-container", "image": "img", "ports": [{"containerPort": 8080, "name": "http1"}]}]}


def _meta(**ann):
    return {**META, "annotations": dict(ann)}


# ------------------------------------------------------------------ Deployment
@pytest.mark.parametrize("ext,replicas", [({}, 1), ({"minReplicas": 0}, 1), ({"minReplicas": 3}, 3),
                                          ({"minReplicas": None}, 1), ({"minReplicas": 2, "maxReplicas": 5}, 2)])
def test_deployment_replicas(ext, replicas):
    assert W.build_deployment(META, POD, ext)["spec"]["replicas"] == replicas


def test_deployment_defaults_and_labels():
    d = W.build_deployment(META, POD, {})
    sp = d["spec"]
    assert sp["strategy"] == {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": 0, "maxSurge": 1}}
    assert sp["selector"]["matchLabels"] == {"app": "llama-engine"}
    assert sp["template"]["metadata"]["labels"]["app"] == "llama-engine"
    assert sp["template"]["metadata"]["labels"]["app.kubernetes.io/name"] == "llama"
    assert "name" not in sp["template"]["metadata"] and d["metadata"]["labels"]["app"] == "llama-engine"
    assert sp["revisionHistoryLimit"] == 10 and sp["progressDeadlineSeconds"] == 600
    custom = {"type": "Recreate"}
    assert W.build_deployment(META, POD, {"deploymentStrategy": custom})["spec"]["strategy"] == custom


def test_deployment_name_truncated_to_63():
    long = {**META, "name": "x" * 80}
    d = W.build_deployment(long, POD, {})
    assert len(d["spec"]["selector"]["matchLabels"]["app"]) <= 63


# ------------------------------------------------------------------ Service
@pytest.mark.parametrize("ann,stype,lb", [
    ({}, "ClusterIP", None),
    ({C.SERVICE_TYPE: "LoadBalancer"}, "LoadBalancer", None),
    ({C.SERVICE_TYPE: "LoadBalancer", C.LOAD_BALANCER_IP: "10.0.0.5"}, "LoadBalancer", "10.0.0.5"),
    ({C.SERVICE_TYPE: "NodePort"}, "NodePort", None),
    ({C.SERVICE_TYPE: "ExternalName"}, "ClusterIP", None),            # unsupported type -> ClusterIP
    ({C.SERVICE_TYPE: "ClusterIP", C.LOAD_BALANCER_IP: "10.0.0.5"}, "ClusterIP", None),   # IP only for LB
])
def test_service_type(ann, stype, lb):
    s = W.build_service(_meta(**ann), POD)
    assert s["spec"]["type"] == stype and s["spec"].get("loadBalancerIP") == lb


def test_service_ports_selector_and_annotation_filter():
    s = W.build_service(_meta(**{"prometheus.io/scrape": "true", "keep.me/x": "1"}), POD)
    assert s["spec"]["ports"] == [{"name": "http1", "port": 8080, "targetPort": 8080, "protocol": "TCP"}]
    assert s["spec"]["selector"] == {"app": "llama-engine"}
    assert s["metadata"]["annotations"] == {"keep.me/x": "1"}   # pod-only annotations stay off the Service
    bare = W.build_service(META, {"containers": [{"name": "c"}]})
    assert bare["spec"]["ports"] == [{"name": "c", "port": C.DEFAULT_HTTP_PORT, "targetPort": C.DEFAULT_HTTP_PORT,
                                      "protocol": "TCP"}]
    multi = W.build_service(META, {"containers": [{"name": "c", "ports": [
        {"containerPort": 8080, "name": "http"}, {"containerPort": 30000, "name": "grpc", "protocol": "TCP"}]}]})
    assert [p["port"] for p in multi["spec"]["ports"]] == [8080, 30000]
    custom = W.build_service(META, POD, selector={"component": "engine"}, name="svc")
    assert custom["spec"]["selector"] == {"component": "engine"} and custom["metadata"]["name"] == "svc"


# ------------------------------------------------------------------ HPA
@pytest.mark.parametrize("ext,ann,want", [
    ({}, {}, (1, 1, "cpu", 80)),
    ({"minReplicas": 0, "maxReplicas": 0}, {}, (1, 1, "cpu", 80)),
    ({"minReplicas": 2, "maxReplicas": 5}, {}, (2, 5, "cpu", 80)),
    ({"minReplicas": 4, "maxReplicas": 2}, {}, (4, 4, "cpu", 80)),           # max never below min
    ({"scaleMetric": "memory", "scaleTarget": 60}, {}, (1, 1, "memory", 60)),
    ({"scaleMetric": "concurrency"}, {}, (1, 1, "cpu", 80)),               # not a resource metric -> cpu
    ({"scaleTarget": 60}, {C.TARGET_UTILIZATION: "35"}, (1, 1, "cpu", 35)),   # annotation wins
])
def test_hpa(ext, ann, want):
    h = W.build_hpa(_meta(**ann), ext)
    sp = h["spec"]
    res = sp["metrics"][0]["resource"]
    assert (sp["minReplicas"], sp["maxReplicas"], res["name"], res["target"]["averageUtilization"]) == want
    assert sp["scaleTargetRef"] == {"apiVersion": "apps/v1", "kind": "Deployment", "name": "llama-engine"}
    assert res["target"]["type"] == "Utilization"


# ------------------------------------------------------------------ KEDA
DEF = KedaDefaults()


def test_keda_defaults():
    so = W.build_scaled_object(META, {}, None, DEF)
    t = so["spec"]["triggers"][0]
    assert t["type"] == "prometheus" and t["metadata"]["serverAddress"] == DEF.promServerAddress
    assert t["metadata"]["threshold"] == str(DEF.scalingThreshold)
    assert t["metadata"]["operator"] == "LessThanOrEqual"
    assert 'ome_io_inferenceservice="llama-engine"' in t["metadata"]["query"]
    assert (so["spec"]["minReplicaCount"], so["spec"]["maxReplicaCount"]) == (1, 1)
    assert so["spec"]["scaleTargetRef"] == {"name": "llama-engine"} and "authenticationRef" not in t


@pytest.mark.parametrize("isvc_keda,ext_keda,ann,key,want", [
    ({"promServerAddress": "http://p:9090"}, None, {}, "serverAddress", "http://p:9090"),
    ({"promServerAddress": "http://p:9090"}, {"promServerAddress": "http://q:9090"}, {}, "serverAddress",
     "http://q:9090"),                                                    # component config overrides the ISVC's
    (None, None, {C.KEDA_SERVER_ADDRESS: "http://a:9090"}, "serverAddress", "http://a:9090"),   # annotation wins
    ({"scalingThreshold": "25"}, None, {}, "threshold", "25"),
    (None, None, {C.KEDA_THRESHOLD: "7"}, "threshold", "7"),
    ({"scalingOperator": "GreaterThanOrEqual"}, None, {}, "operator", "GreaterThanOrEqual"),
    (None, None, {C.KEDA_OPERATOR: "GreaterThanOrEqual"}, "operator", "GreaterThanOrEqual"),
    ({"customPromQuery": "sum(rate(x[1m]))"}, None, {}, "query", "sum(rate(x[1m]))"),
    ({"customPromQuery": 'sum(x{svc="%s"})'}, None, {}, "query", 'sum(x{svc="llama-engine"})'),   # name templated
    (None, None, {C.KEDA_QUERY: "up"}, "query", "up"),
])
def test_keda_overrides(isvc_keda, ext_keda, ann, key, want):
    ext = {"kedaConfig": ext_keda} if ext_keda else {}
    so = W.build_scaled_object(_meta(**ann), ext, isvc_keda, DEF)
    assert so["spec"]["triggers"][0]["metadata"][key] == want


def test_keda_auth_and_bounds():
    so = W.build_scaled_object(META, {"minReplicas": 0, "maxReplicas": 4},
                               {"authenticationRef": {"name": "prom-auth"}, "authModes": "bearer"}, DEF)
    t = so["spec"]["triggers"][0]
    assert t["authenticationRef"] == {"name": "prom-auth"} and t["metadata"]["authModes"] == "bearer"
    assert (so["spec"]["minReplicaCount"], so["spec"]["maxReplicaCount"]) == (0, 4)   # KEDA may scale to zero


# ------------------------------------------------------------------ PDB
@pytest.mark.parametrize("ext,want", [({}, None), ({"minAvailable": 1}, {"minAvailable": 1}),
                                      ({"maxUnavailable": "25%"}, {"maxUnavailable": "25%"}),
                                      ({"minAvailable": 2, "maxUnavailable": 1}, {"minAvailable": 2})])
def test_pdb(ext, want):
    p = W.build_pdb(META, ext)
    if want is None:
        assert p is None
        return
    sp = dict(p["spec"])
    assert sp.pop("selector") == {"matchLabels": {"app": "llama-engine"}}
    assert sp == want


# ------------------------------------------------------------------ reconcile_raw: autoscaler switch
def _isvc():
    return {"apiVersion": C.API_VERSION, "kind": "InferenceService",
            "metadata": {"name": "llama", "namespace": "team", "uid": "u1"}, "spec": {}}


@pytest.mark.parametrize("seq", [["hpa", "keda"], ["keda", "hpa"], ["hpa", "external"], ["keda", "external"]])
def test_reconcile_raw_switches_autoscaler(seq):
    st = Store()
    isvc = st.create(_isvc())
    cfg = ControllerConfig.from_store(st)
    for cls in seq:
        meta = _meta(**{C.AUTOSCALER_CLASS: cls})
        W.reconcile_raw(st, isvc, meta, POD, {"minReplicas": 1, "maxReplicas": 3}, cfg)
        hpa = st.try_get("autoscaling/v2", "HorizontalPodAutoscaler", "llama-engine", "team")
        so = st.try_get("keda.sh/v1alpha1", "ScaledObject", "llama-engine", "team")
        assert (hpa is not None) == (cls == "hpa") and (so is not None) == (cls == "keda"), cls
        assert st.try_get("apps/v1", "Deployment", "llama-engine", "team") is not None
        assert st.try_get("v1", "Service", "llama-engine", "team") is not None


def test_reconcile_raw_pdb_lifecycle_and_unknown_class():
    st = Store()
    isvc = st.create(_isvc())
    cfg = ControllerConfig.from_store(st)
    W.reconcile_raw(st, isvc, META, POD, {"minAvailable": 1}, cfg)
    assert st.try_get("policy/v1", "PodDisruptionBudget", "llama-engine", "team") is not None
    W.reconcile_raw(st, isvc, META, POD, {}, cfg)
    assert st.try_get("policy/v1", "PodDisruptionBudget", "llama-engine", "team") is None
    with pytest.raises(ValueError, match="unknown autoscaler class"):
        W.reconcile_raw(st, isvc, _meta(**{C.AUTOSCALER_CLASS: "bogus"}), POD, {}, cfg)

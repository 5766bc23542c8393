"""InferenceService controller utilities, case by case (the reference's ``utils/annotations_test.go``,
``utils/migration_util_test.go`` and the mode tables of ``controller_test.go``): per-ISVC ingress
annotation overrides, deployment-mode resolution for engine / decoder / router, the deprecated
``predictor`` -> ``engine`` migration, controller ConfigMap parsing and the template renderer."""
import json

import pytest

from ome_amd.api import constants as C
from ome_amd.controllers.config import ControllerConfig, IngressConfig, render_template, resolve_ingress
from ome_amd.controllers.isvc.controller import determine_modes, engine_mode, migrate_predictor, mode_from_annotations
from ome_amd.store.store import Store

RAW, MN, KN, RAY, VIRT = (C.DeploymentMode.RAW, C.DeploymentMode.MULTINODE, C.DeploymentMode.SERVERLESS,
                          C.DeploymentMode.MULTINODE_RAY_VLLM, C.DeploymentMode.VIRTUAL)


# ------------------------------------------------------------------ ingress annotations
def test_no_annotations_returns_base_config():
    base = IngressConfig()
    assert resolve_ingress(base, None) == base and resolve_ingress(base, {}) == base


@pytest.mark.parametrize("ann,field,want", [
    ({C.INGRESS_DOMAIN_TEMPLATE: "{{ .Name }}.example.com"}, "domainTemplate", "{{ .Name }}.example.com"),
    ({C.INGRESS_DOMAIN: "example.com"}, "ingressDomain", "example.com"),
    ({C.INGRESS_URL_SCHEME: "https"}, "urlScheme", "https"),
    ({C.INGRESS_ADDITIONAL_DOMAINS: "a.com, b.com,,"}, "additionalIngressDomains", ["a.com", "b.com"]),
    ({C.INGRESS_PATH_TEMPLATE: "/serving/{{ .Namespace }}/{{ .Name }}"}, "pathTemplate",
     "/serving/{{ .Namespace }}/{{ .Name }}"),
    ({C.INGRESS_DISABLE_ISTIO_VIRTUALHOST: "TRUE"}, "disableIstioVirtualHost", True),
    ({C.INGRESS_DISABLE_CREATION: "false"}, "disableIngressCreation", False),
])
def test_single_annotation_override(ann, field, want):
    out = resolve_ingress(IngressConfig(), ann)
    assert getattr(out, field) == want


def test_comprehensive_override_leaves_base_untouched():
    base = IngressConfig()
    ann = {C.INGRESS_DOMAIN: "x.io", C.INGRESS_URL_SCHEME: "https", C.INGRESS_DISABLE_CREATION: "false",
           C.INGRESS_ADDITIONAL_DOMAINS: "y.io"}
    out = resolve_ingress(base, ann)
    assert (out.ingressDomain, out.urlScheme, out.disableIngressCreation, out.additionalIngressDomains) == \
        ("x.io", "https", False, ["y.io"])
    assert base.ingressDomain == "svc.cluster.local" and base.disableIngressCreation is True


def test_unrelated_annotations_ignored():
    out = resolve_ingress(IngressConfig(), {"team": "a", "ome.io/other": "b"})
    assert out == IngressConfig()


# ------------------------------------------------------------------ deployment modes
@pytest.mark.parametrize("ann,want", [
    (None, None), ({}, None), ({C.DEPLOYMENT_MODE: KN}, KN), ({C.DEPLOYMENT_MODE: RAW}, RAW),
    ({C.DEPLOYMENT_MODE: RAY}, RAY), ({C.DEPLOYMENT_MODE: MN}, MN), ({C.DEPLOYMENT_MODE: VIRT}, VIRT),
    ({C.DEPLOYMENT_MODE: "Bogus"}, None), ({C.DEPLOYMENT_MODE: ""}, None), ({"other": "x"}, None),
])
def test_mode_from_annotations(ann, want):
    assert mode_from_annotations(ann) == want


@pytest.mark.parametrize("engine,want", [
    (None, RAW),
    ({"minReplicas": 1}, RAW),
    ({"minReplicas": 0}, KN),
    ({"leader": {}, "worker": {"size": 1}}, MN),
    ({"worker": {"size": 2}}, MN),
    ({"annotations": {C.DEPLOYMENT_MODE: RAY}, "worker": {"size": 1}}, RAY),   # annotation wins
    ({"annotations": {C.DEPLOYMENT_MODE: "nope"}, "minReplicas": 0}, KN),       # invalid annotation ignored
])
def test_engine_mode(engine, want):
    assert engine_mode(engine) == want


@pytest.mark.parametrize("engine,decoder,router,want", [
    ({"minReplicas": 1}, None, None, (RAW, RAW, RAW)),                                   # single raw engine
    ({"leader": {}, "worker": {"size": 1}}, None, None, (MN, RAW, RAW)),                 # multi-node engine
    ({"minReplicas": 1}, {"minReplicas": 1}, None, (RAW, RAW, RAW)),                     # PD raw
    ({"minReplicas": 1}, {"leader": {}, "worker": {"size": 1}}, None, (RAW, MN, RAW)),   # PD + MN decoder
    ({"minReplicas": 0}, {"minReplicas": 1}, None, (RAW, RAW, RAW)),                     # PD forces raw engine
    ({"minReplicas": 1}, None, {"minReplicas": 0}, (RAW, RAW, KN)),                      # serverless router
    ({"minReplicas": 0}, None, None, (KN, RAW, RAW)),
])
def test_determine_modes(engine, decoder, router, want):
    assert determine_modes(engine, decoder, router) == want


def test_determine_modes_requires_engine():
    with pytest.raises(ValueError):
        determine_modes(None, {"minReplicas": 1}, None)


# ------------------------------------------------------------------ predictor migration
def _isvc(spec):
    return {"metadata": {"name": "svc", "namespace": "default"}, "spec": spec}


def test_predictor_with_model_and_base_model():
    isvc = _isvc({"predictor": {"model": {"baseModel": "llama", "runtime": "rt", "protocolVersion": "openAI"}}})
    assert migrate_predictor(isvc)
    sp = isvc["spec"]
    assert "predictor" not in sp and sp["model"] == {"name": "llama"} and sp["runtime"] == {"name": "rt"}
    assert "runner" not in sp["engine"]   # nothing container-like to carry over


def test_predictor_with_min_replicas_and_extension_fields():
    isvc = _isvc({"predictor": {"minReplicas": 2, "maxReplicas": 5, "scaleMetric": "cpu",
                                "model": {"baseModel": "llama"}}})
    migrate_predictor(isvc)
    e = isvc["spec"]["engine"]
    assert (e["minReplicas"], e["maxReplicas"], e["scaleMetric"]) == (2, 5, "cpu")


def test_predictor_model_container_fields_become_runner():
    isvc = _isvc({"predictor": {"model": {"baseModel": "llama", "image": "x:1", "args": ["--a"],
                                          "resources": {"limits": {"amd.com/gpu": "1"}}}}})
    migrate_predictor(isvc)
    r = isvc["spec"]["engine"]["runner"]
    assert r["name"] == C.MAIN_CONTAINER and r["image"] == "x:1" and r["args"] == ["--a"]


def test_predictor_with_containers_kept_on_engine():
    c = [{"name": "ome-container", "image": "y:2"}]
    isvc = _isvc({"predictor": {"containers": c, "model": {"baseModel": "llama"}}})
    migrate_predictor(isvc)
    assert isvc["spec"]["engine"]["containers"] == c


def test_predictor_with_worker_spec_becomes_multinode():
    isvc = _isvc({"predictor": {"model": {"baseModel": "llama"}, "workerSpec": {"size": 2}}})
    migrate_predictor(isvc)
    e = isvc["spec"]["engine"]
    assert e["worker"] == {"size": 2} and e["leader"] == {} and engine_mode(e) == MN


def test_predictor_fine_tuned_weights_carried():
    isvc = _isvc({"predictor": {"model": {"baseModel": "llama", "fineTunedWeights": ["ft-a"]}}})
    migrate_predictor(isvc)
    assert isvc["spec"]["model"] == {"name": "llama", "fineTunedWeights": ["ft-a"]}


def test_existing_model_and_runtime_not_overwritten():
    isvc = _isvc({"model": {"name": "keep"}, "runtime": {"name": "keep-rt"},
                  "predictor": {"model": {"baseModel": "other", "runtime": "other-rt"}}})
    migrate_predictor(isvc)
    assert isvc["spec"]["model"] == {"name": "keep"} and isvc["spec"]["runtime"] == {"name": "keep-rt"}


def test_empty_predictor_and_no_predictor_are_no_ops():
    a = _isvc({"predictor": {}})
    assert not migrate_predictor(a) and "engine" not in a["spec"]
    b = _isvc({"engine": {"minReplicas": 1}})
    assert not migrate_predictor(b)


def test_no_migration_when_engine_already_exists():
    isvc = _isvc({"engine": {"minReplicas": 1}, "predictor": {"model": {"baseModel": "llama"}}})
    assert not migrate_predictor(isvc) and "predictor" in isvc["spec"]


# ------------------------------------------------------------------ controller config
def _store(**data):
    s = Store()
    s.create({"apiVersion": "v1", "kind": "ConfigMap",
              "metadata": {"name": C.INFERENCESERVICE_CONFIGMAP, "namespace": C.OME_NAMESPACE},
              "data": {k: json.dumps(v) for k, v in data.items()}})
    return s


def test_config_defaults_without_configmap():
    cfg = ControllerConfig.from_store(Store())
    assert cfg.deploy.defaultDeploymentMode == RAW and cfg.ingress.disableIngressCreation is True
    assert cfg.keda.enableKeda is True and cfg.model_init.authType == "InstancePrincipal"


def test_config_keys_override_defaults_and_unknown_fields_ignored():
    cfg = ControllerConfig.from_store(_store(ingress={"ingressDomain": "corp.io", "bogus": 1},
                                             deploy={"defaultDeploymentMode": KN},
                                             multinodeProber={"image": "p:2", "startupFailureThreshold": 9},
                                             kedaConfig={"enableKeda": False, "scalingThreshold": "5"}))
    assert cfg.ingress.ingressDomain == "corp.io" and not hasattr(cfg.ingress, "bogus")
    assert cfg.deploy.defaultDeploymentMode == KN
    assert (cfg.prober.image, cfg.prober.startupFailureThreshold) == ("p:2", 9)
    assert cfg.keda.enableKeda is False and cfg.keda.scalingThreshold == "5"


def test_config_invalid_json_raises():
    s = Store()
    s.create({"apiVersion": "v1", "kind": "ConfigMap",
              "metadata": {"name": C.INFERENCESERVICE_CONFIGMAP, "namespace": C.OME_NAMESPACE},
              "data": {"ingress": "{not json"}})
    with pytest.raises(ValueError, match="invalid JSON"):
        ControllerConfig.from_store(s)


def test_benchmark_config_from_its_configmap():
    s = Store()
    s.create({"apiVersion": "v1", "kind": "ConfigMap",
              "metadata": {"name": C.BENCHMARKJOB_CONFIGMAP, "namespace": C.OME_NAMESPACE},
              "data": {"benchmarkjob": json.dumps({"podConfig": {"image": "lg:3"}})}})
    assert ControllerConfig.from_store(s).benchmark.podConfig == {"image": "lg:3"}


# ------------------------------------------------------------------ templates
@pytest.mark.parametrize("tmpl,want", [
    ("{{ .Name }}.{{ .Namespace }}.{{ .IngressDomain }}", "svc.ns.example.com"),
    ("{{.Name}}-{{.Namespace}}", "svc-ns"),
    ("/v1/{{ .Labels.team }}/{{ .Annotations.route }}", "/v1/ml/r1"),
    ("{{ .Missing }}x", "x"),
    ("no template", "no template"),
])
def test_render_template(tmpl, want):
    vals = {"Name": "svc", "Namespace": "ns", "IngressDomain": "example.com", "Labels": {"team": "ml"},
            "Annotations": {"route": "r1"}}
    assert render_template(tmpl, vals) == want

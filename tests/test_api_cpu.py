"""ome.io/v1beta1 API surface: every reference manifest parses and round-trips through the typed
models (the reference CRDs' wire format, ``pkg/apis/ome/v1beta1``), CRD generation is in sync
with the checked-in ``config/crd``, and the deterministic naming / label-hashing helpers
(``pkg/constants/constants.go:735-930``)."""
import glob
import hashlib
import os

import pytest
import yaml

from ome_amd.api import constants as C
from ome_amd.api import schema
from ome_amd.api import v1beta1 as V

REF = "/root/reference/config"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _norm(x):
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items() if v is not None}
    if isinstance(x, list):
        return [_norm(v) for v in x]
    return x


def _docs(pattern):
    for f in sorted(glob.glob(pattern, recursive=True)):
        for d in yaml.safe_load_all(open(f)):
            if isinstance(d, dict) and d.get("kind") in V.KINDS:
                yield f, d


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_reference_manifests_round_trip():
    ok, failed, kinds = 0, [], {}
    for f, d in _docs(f"{REF}/**/*.yaml"):
        kinds[d["kind"]] = kinds.get(d["kind"], 0) + 1
        try:
            spec = V.spec_of(d)
        except Exception:  # noqa: BLE001
            failed.append(os.path.relpath(f, REF))
            continue
        assert _norm(spec.dump()) == _norm(d.get("spec") or {}), f
        ok += 1
    # the one sample that spells ``model.modelName`` instead of ``model.name`` is rejected
    assert failed == ["samples/isvc/LGAI-EXAONE/exaone-3-5-7-8b-instruct-isvc.yaml"]
    assert ok >= 559 and kinds["ClusterServingRuntime"] >= 200 and kinds["ClusterBaseModel"] >= 200


def test_own_catalog_parses():
    n = 0
    for f, d in _docs(f"{ROOT}/config/**/*.yaml"):
        V.spec_of(d)
        n += 1
    assert n >= 5


def test_crds_in_sync(tmp_path):
    for p in schema.write_all(tmp_path):
        mine = yaml.safe_load(p.read_text())
        checked_in = yaml.safe_load(open(os.path.join(ROOT, "config", "crd", p.name)))
        assert mine == checked_in, p.name
    isvc = schema.crd("InferenceService")
    props = isvc["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["spec"]["properties"]
    assert {"model", "runtime", "engine", "decoder", "router", "predictor"} <= set(props)
    assert isvc["spec"]["scope"] == "Namespaced" and "isvc" in isvc["spec"]["names"]["shortNames"]
    assert schema.crd("ClusterBaseModel")["spec"]["scope"] == "Cluster"


def test_camel_case_aliases_and_extra_fields_round_trip():
    spec = {"engine": {"minReplicas": 1, "maxReplicas": 3, "scaleMetric": "cpu", "scaleTarget": 70,
                       "runner": {"name": "c", "image": "img", "resources": {"limits": {"amd.com/gpu": 8}}},
                       "nodeSelector": {"a": "b"}, "someFutureField": {"x": 1}},
            "model": {"name": "llama-3-8b"}}
    s = V.InferenceServiceSpec.model_validate(spec)
    assert s.engine.min_replicas == 1 and s.engine.max_replicas == 3
    assert s.dump() == spec


def _h8(s):
    return hashlib.sha256(s.encode()).hexdigest()[:8]


def test_model_labels_and_keys():
    assert C.cluster_base_model_label("llama-3-8b-instruct") == "models.ome.io/clusterbasemodel.llama-3-8b-instruct"
    assert C.base_model_label("team-a", "llama") == "models.ome.io/team-a.basemodel.llama"
    long = "a" * 80
    lab = C.cluster_base_model_label(long)
    name = lab.split("clusterbasemodel.", 1)[1]
    assert name == f"{_h8(long)}-{long[-(32 - 9):]}" and len(lab.split("/", 1)[1]) <= 49
    ns, model = "very-long-namespace-name", "b" * 60
    lab = C.base_model_label(ns, model)
    assert len(lab.split("/", 1)[1]) <= 49 and lab.startswith(f"models.ome.io/{_h8(ns)}.basemodel.{_h8(model)}-")
    assert C.model_configmap_key(None, "m", True) == "clusterbasemodel.m"
    assert C.model_configmap_key("ns", "m", False) == "ns.basemodel.m"
    assert C.parse_model_configmap_key("ns.basemodel.m") == ("ns", "m", False)
    assert C.parse_model_configmap_key("clusterbasemodel.m") == ("", "m", True)
    assert C.parse_model_configmap_key("garbage") is None


def test_dns_safe_truncation():
    for n in range(200):
        s = f"inference-service-{n}-" + "x" * 70
        t = C.truncate_name(s, 63)
        assert len(t) == 63 and t[0].isalpha() and t.endswith("x" * 20)
        assert t[1:8] == _h8(s)[1:8]
    assert C.truncate_name("short", 63) == "short"
    assert C.engine_name("a") == "a-engine" and C.decoder_name("a") == "a-decoder" and C.router_name("a") == "a-router"
    assert C.lws_name("a" * 60) == "lws-" + "a" * 50
    assert C.modelconfig_name("b" * 30) == "modelconfig-" + "b" * 20


def test_deployment_modes():
    for m in ("RawDeployment", "Serverless", "MultiNode", "MultiNodeRayVLLM", "PDDisaggregated"):
        assert C.DeploymentMode.is_valid(m)
    assert not C.DeploymentMode.is_valid("Bogus")

"""OpenAPI document + Python SDK (reference ``pkg/openapi/swagger.json`` and the openapi-codegen SDK
of ``hack/python-sdk``): every definition the reference publishes exists here under the same
``v1beta1.*`` name, every ``$ref`` resolves, the committed ``config/openapi/swagger.json`` is
current, and the SDK drives a live manager over HTTP (typed CRUD, dry-run admission errors, merge
patch, status update, apply, waits)."""
import json
import socket
import threading
import time
from pathlib import Path

import pytest
import uvicorn

from ome_amd.api import objects as O
from ome_amd.api import openapi as A
from ome_amd.manager import Cluster, create_api
from ome_amd.sdk import Invalid, NotFound, OmeClient, is_ready
from ome_amd.sdk import models as m

REPO = Path(__file__).resolve().parents[1]
REF_SWAGGER = Path("/root/reference/pkg/openapi/swagger.json")


def test_definitions_cover_the_reference_and_resolve():
    doc = A.swagger()
    defs = doc["definitions"]
    if REF_SWAGGER.exists():   # names only (JSON, loaded with the json module)
        ref = set(json.loads(REF_SWAGGER.read_text())["definitions"])
        assert not ref - set(defs), sorted(ref - set(defs))
    text = json.dumps(doc)
    import re

    refs = set(re.findall(r"#/definitions/([A-Za-z0-9_.]+)", text))
    assert refs <= set(defs), sorted(refs - set(defs))
    assert "nullable" not in text and '"anyOf"' not in text and "$defs" not in text   # swagger 2.0 only
    isvc = defs["v1beta1.InferenceService"]["properties"]
    assert isvc["spec"]["$ref"] == "#/definitions/v1beta1.InferenceServiceSpec"
    assert isvc["status"]["$ref"] == "#/definitions/v1beta1.InferenceServiceStatus"
    ops = {op["operationId"] for p in doc["paths"].values() for op in p.values()}
    assert {"createNamespacedInferenceService", "listClusterBaseModel", "patchNamespacedBenchmarkJob",
            "replaceNamespacedInferenceServiceStatus", "deleteAcceleratorClass"} <= ops
    assert len(ops) == 8 * 7   # list, create, read, replace, patch, delete, replace-status per kind


def test_committed_swagger_is_current():
    assert json.loads((REPO / "config/openapi/swagger.json").read_text()) == json.loads(json.dumps(A.swagger())), \
        "regenerate: python -m ome_amd.api.openapi config/openapi/swagger.json"


def test_sdk_model_names_and_round_trip():
    for name in ("V1beta1InferenceService", "V1beta1InferenceServiceList", "V1beta1InferenceServiceSpec",
                 "V1beta1ClusterServingRuntime", "V1beta1BenchmarkJobStatus", "V1beta1ModelStatus",
                 "V1beta1ComponentStatusSpec", "V1beta1SupportedRuntime", "V1beta1PodSpec"):
        assert hasattr(m, name), name
    d = {"apiVersion": "ome.io/v1beta1", "kind": "InferenceService", "metadata": {"name": "x", "namespace": "ns"},
         "spec": {"model": {"name": "llama"}, "engine": {"minReplicas": 1, "maxReplicas": 2, "runner": {"image": "i"}}},
         "status": {"url": "http://x", "conditions": [{"type": "Ready", "status": "True"}],
                    "components": {"engine": {"latestReadyRevision": "r1", "restURL": "http://e"}},
                    "modelStatus": {"transitionStatus": "UpToDate", "modelCopies": {"failedCopies": 0}}}}
    o = m.V1beta1InferenceService.model_validate(d)
    assert o.status.components["engine"].rest_url == "http://e" and o.spec.engine.max_replicas == 2
    assert o.dump() == d
    assert O.parse(d).dump() == d


@pytest.fixture()
def served(tmp_path):
    # store + admission only (controllers not started): the test owns every status it reads
    cl = Cluster(str(tmp_path), with_agent=False, with_executor=False)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = uvicorn.Server(uvicorn.Config(create_api(cl), host="127.0.0.1", port=port, log_level="error"))
    t = threading.Thread(target=srv.run, daemon=True)
    t.start()
    for _ in range(200):
        if srv.started:
            break
        time.sleep(0.05)
    try:
        yield cl, f"http://127.0.0.1:{port}"
    finally:
        srv.should_exit = True
        t.join(timeout=10)
        cl.shutdown()


MODEL = {"vendor": "meta", "modelFormat": {"name": "safetensors", "version": "1.0.0"},
         "modelFramework": {"name": "transformers", "version": "4.46.0"}, "modelArchitecture": "LlamaForCausalLM",
         "modelParameterSize": "8B", "storage": {"storageUri": "hf://meta-llama/Meta-Llama-3-8B-Instruct"}}
RUNTIME = {"supportedModelFormats": [{"name": "safetensors", "modelFormat": {"name": "safetensors", "version": "1.0.0"},
                                      "modelArchitecture": "LlamaForCausalLM", "autoSelect": True, "priority": 1}],
           "protocolVersions": ["openAI"], "modelSizeRange": {"min": "1B", "max": "10B"},
           "engineConfig": {"runner": {"name": "ome-container", "image": "ome-amd:latest"}}}


def test_sdk_against_a_live_manager(served):
    cl, url = served
    with OmeClient(url) as c:
        assert c.openapi()["swagger"] == "2.0"
        cbm = c.cluster_base_models.create(m.V1beta1ClusterBaseModel(metadata={"name": "llama-3-8b"},
                                                                     spec=m.V1beta1BaseModelSpec.model_validate(MODEL)))
        assert isinstance(cbm, m.V1beta1ClusterBaseModel) and cbm.spec.model_parameter_size == "8B"
        c.cluster_serving_runtimes.create({"metadata": {"name": "rt"}, "spec": RUNTIME})
        # dry run goes through admission and persists nothing
        c.inference_services.create({"metadata": {"name": "dry", "namespace": "default"},
                                     "spec": {"model": {"name": "llama-3-8b"}}}, dry_run=True)
        with pytest.raises(NotFound):
            c.inference_services.get("dry", "default")
        with pytest.raises(Invalid, match="invalid InferenceService name"):
            c.inference_services.create({"metadata": {"name": "Bad_Name", "namespace": "default"}, "spec": {}})
        isvc = c.inference_services.create({"metadata": {"name": "llama", "namespace": "team-a"},
                                            "spec": {"model": {"name": "llama-3-8b"}}})
        assert isvc.metadata.namespace == "team-a"
        lst = c.inference_services.list()
        assert isinstance(lst, m.V1beta1InferenceServiceList) and [i.metadata.name for i in lst.items] == ["llama"]
        assert c.inference_services.list("other").items == []
        p = c.inference_services.patch("llama", {"metadata": {"labels": {"team": "a"}}}, "team-a")
        assert p.metadata.labels == {"team": "a"}
        # status subresource + waits
        cur = c.inference_services.get("llama", "team-a", typed=False)
        cur["status"] = {"url": "http://llama.team-a", "conditions": [{"type": "Ready", "status": "True"}]}
        c.inference_services.replace_status(cur)
        got = c.inference_services.wait_ready("llama", "team-a", timeout=10, poll=0.05)
        assert is_ready(got) and got.status.url == "http://llama.team-a"
        with pytest.raises(TimeoutError):
            c.cluster_base_models.wait_ready("nope", timeout=0.3, poll=0.05)
        # apply: create-or-update through the same chain
        out = c.apply([{"apiVersion": "ome.io/v1beta1", "kind": "ClusterBaseModel", "metadata": {"name": "llama-3-8b"},
                        "spec": {**MODEL, "vendor": "meta-llama"}}])
        assert out and c.cluster_base_models.get("llama-3-8b").spec.vendor == "meta-llama"
        assert c.get("ClusterBaseModel", "llama-3-8b", typed=False)["kind"] == "ClusterBaseModel"
        c.inference_services.delete("llama", "team-a")
        with pytest.raises(NotFound):
            c.inference_services.get("llama", "team-a")

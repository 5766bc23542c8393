"""Web console frontend (H8; reference web-console/frontend): the SPA's scripts parse, the pure
helpers in static/lib.js behave (run under node), and -- the point of the structured forms --
the manifests the form builders emit pass the server's own admission chain and the storage-URI
grammar of ome_amd.storage.uri.  Skips when no node binary is installed."""
import json
import re
import shutil
import subprocess
from pathlib import Path

import pytest
import yaml
from fastapi.testclient import TestClient

from ome_amd.console import create_app
from ome_amd.manager import Cluster
from ome_amd.storage import uri as U

STATIC = Path(__file__).resolve().parents[1] / "ome_amd" / "console" / "static"
NODE = shutil.which("node")
need_node = pytest.mark.skipif(NODE is None, reason="node not installed")


def _node(script: str):
    out = subprocess.run([NODE, "-e", script], capture_output=True, text=True, timeout=60, cwd=str(STATIC))
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout)


@need_node
@pytest.mark.parametrize("name", ["lib.js", "forms.js", "app.js"])
def test_scripts_parse(tmp_path, name):
    # the image's node predates ?. and ??; swapping them for . and || keeps the parse equivalent
    src = (STATIC / name).read_text()
    src = src.replace("?.[", "[").replace("?.(", "(").replace("?.", ".").replace("??", "||")
    f = tmp_path / name
    f.write_text(src)
    r = subprocess.run([NODE, "--check", str(f)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr


URIS = {
    "hf": {"repo": "meta-llama/Llama-3.1-8B-Instruct", "revision": "main"},
    "oci": {"namespace": "ns1", "bucket": "b1", "prefix": "models/llama"},
    "s3": {"bucket": "bk", "region": "us-west-2", "prefix": "m/x"},
    "az": {"account": "acct", "container": "models", "path": "llama/v1"},
    "gs": {"bucket": "bk", "object": "models/llama"},
    "pvc": {"namespace": "team", "claim": "model-store", "subpath": "llama"},
    "github": {"repo": "owner/repo", "tag": "v1"},
    "vendor": {"vendor": "acme", "type": "models", "path": "llama"},
    "local": {"path": "/raid/models/llama"},
    "random": {"preset": "llama-3-8b", "layers": "2"},
}


@need_node
def test_storage_uris_round_trip_and_match_the_server_grammar():
    res = _node(f"""const O = require('./lib.js'); const F = {json.dumps(URIS)}; const out = {{}};
      for (const [s, f] of Object.entries(F)) {{ const u = O.buildUri(s, f); out[s] = [u, O.parseUri(u)]; }}
      out.bad = O.parseUri('ftp://x'); console.log(JSON.stringify(out));""")
    assert res.pop("bad") is None
    for scheme, (built, parsed) in res.items():
        assert parsed == {"scheme": scheme, "fields": URIS[scheme]}, (scheme, built, parsed)
        U.parse(built)   # the server-side parser accepts every URI the form builds


@need_node
def test_yaml_csv_size_helpers():
    obj = {"apiVersion": "ome.io/v1beta1", "kind": "X", "metadata": {"name": "a", "labels": {"k": "yes"}},
           "spec": {"list": [{"a": 1, "b": [1, 2]}, "s: colon", "007", True, None], "empty": {}, "e2": [],
                    "q": "on", "n": 1.5, "nested": {"deep": {"x": "-lead"}}}}
    res = _node(f"""const O = require('./lib.js');
      console.log(JSON.stringify({{y: O.toYaml({json.dumps(obj)}),
        csv: O.toCsv([['name', (r) => r.n], ['v', (r) => r.v]], [{{n: 'a,b', v: 'say "hi"'}}, {{n: 'c', v: {{x: 1}}}}]),
        sizes: ['7B', '1.5B', '480M', '2T', 'x', ''].map(O.parseSize),
        sorted: O.sortRows([{{s: '70B'}}, {{s: '8B'}}, {{s: '1.5B'}}], (r) => r.s).map((r) => r.s),
        bytes: [0, 1536, 3 * 1024 ** 3].map(O.fmtBytes),
        cat: [O.catalogPath('https://github.com/sgl-project/ome/blob/main/config/runtimes/srt/x-rt.yaml'), O.catalogPath('ome-amd/a.yaml')],
        esc: O.esc('<a href="x">&\\'</a>')}}));""")
    assert yaml.safe_load(res["y"]) == obj
    assert res["csv"] == 'name,v\n"a,b","say ""hi"""\nc,"{""x"":1}"\n'
    assert res["sizes"] == [7e9, 1.5e9, 4.8e8, 2e12, None, None]
    assert res["sorted"] == ["1.5B", "8B", "70B"]
    assert res["bytes"] == ["0 B", "1.5 KiB", "3.0 GiB"]
    assert res["cat"] == ["config/runtimes/srt/x-rt.yaml", "ome-amd/a.yaml"]
    assert res["esc"] == "&lt;a href=&quot;x&quot;&gt;&amp;&#39;&lt;/a&gt;"


FORMS = {
    "model": {"name": "llama-3-8b", "vendor": "meta", "architecture": "LlamaForCausalLM", "parameterSize": "8B",
              "formatName": "safetensors", "formatVersion": "1.0.0", "frameworkName": "transformers",
              "frameworkVersion": "4.46.0", "quantization": "", "capabilities": ["TEXT_GENERATION", "CHAT"],
              "storageUri": "hf://meta-llama/Meta-Llama-3-8B-Instruct", "path": "/raid/models/llama-3-8b",
              "nodeSelector": [["node.kubernetes.io/instance-type", "mi355x"]], "parameters": [], "labels": [["team", "a"]],
              "maxTokens": "8192"},
    "runtime": {"name": "my-runtime", "sizeMin": "1B", "sizeMax": "10B", "protocols": ["openAI"], "accelerators": [],
                "formats": [{"formatName": "safetensors", "formatVersion": "1.0.0", "frameworkName": "transformers",
                             "frameworkVersion": "4.46.0", "architecture": "LlamaForCausalLM", "quantization": "",
                             "autoSelect": True, "priority": "3"}],
                "engine": {"name": "ome-container", "image": "ome-amd:latest", "command": "python3 -m ome_amd.runtime.server",
                           "args": "--model-path $(MODEL_PATH)", "gpus": "1", "port": "8080", "cpu": "", "cpuLimit": "",
                           "memory": "", "memoryLimit": "", "env": [["OME_X", "1"]]},
                "volumes": [{"name": "dshm", "claim": "", "hostPath": "", "medium": "Memory"}], "labels": []},
    "multinode": {"name": "mn-runtime", "sizeMin": "100B", "sizeMax": "900B", "protocols": ["openAI"], "multiNode": True,
                  "workers": "1", "formats": [{"formatName": "safetensors", "architecture": "DeepseekV3ForCausalLM",
                                               "autoSelect": False, "priority": ""}],
                  "engine": {"image": "ome-amd:latest", "gpus": "8", "env": []}},
    "service": {"name": "llama", "namespace": "default", "model": "llama-3-8b", "runtime": "", "min": "1", "max": "2",
                "autoscaler": "hpa", "metric": "cpu", "target": "80", "env": []},
    "keda": {"name": "llama-keda", "namespace": "default", "model": "llama-3-8b", "min": "1", "max": "3", "autoscaler": "keda",
             "promServer": "http://prometheus:9090", "promQuery": "sum(rate(x[1m]))", "threshold": "10",
             "operator": "GreaterThanOrEqual", "env": []},
    "bench": {"name": "bench-1", "namespace": "default", "service": "llama", "task": "text-to-text",
              "scenarios": "N(480,240)/(300,150) D(100,100)", "concurrency": "1 8", "maxTime": "15", "maxRequests": "100",
              "output": "local:///tmp/ome-bench-results"},
}
BAD = {
    "model": {"name": "Bad_Name", "storageUri": "ftp://x", "parameterSize": "huge", "maxTokens": "-1"},
    "runtime": {"name": "ok", "formats": [{"formatName": "", "autoSelect": True, "priority": ""}], "sizeMin": "70B",
                "sizeMax": "8B", "engine": {}, "multiNode": True, "workers": "0"},
    "service": {"name": "s", "model": "", "min": "3", "max": "1", "autoscaler": "hpa", "metric": "gpu", "target": "0"},
}


@need_node
def test_form_manifests_pass_admission(tmp_path):
    res = _node(f"""const O = require('./lib.js'); const F = {json.dumps(FORMS)}; const B = {json.dumps(BAD)};
      console.log(JSON.stringify({{
        model: O.buildModel(F.model), runtime: O.buildRuntime(F.runtime), multinode: O.buildRuntime(F.multinode),
        service: O.buildService(F.service), keda: O.buildService(F.keda), bench: O.buildBenchmark(F.bench),
        okErrs: [O.modelErrors(F.model), O.runtimeErrors(F.runtime), O.runtimeErrors(F.multinode), O.serviceErrors(F.service)],
        badErrs: {{model: O.modelErrors(B.model), runtime: O.runtimeErrors(B.runtime), service: O.serviceErrors(B.service)}},
        yamlOfRuntime: O.toYaml(O.buildRuntime(F.runtime))}}));""")
    assert res["okErrs"] == [[], [], [], []]
    bad = res["badErrs"]
    assert len(bad["model"]) == 4 and any("lower-case" in e for e in bad["model"])
    assert any("format name" in e for e in bad["runtime"]) and any("priority is required" in e for e in bad["runtime"])
    assert any("larger than max" in e for e in bad["runtime"]) and any("engine image" in e for e in bad["runtime"])
    assert any("workers.size" in e for e in bad["runtime"])
    assert any("not a supported metric" in e for e in bad["service"]) and any("[1-100]" in e for e in bad["service"])

    rt = res["runtime"]
    assert yaml.safe_load(res["yamlOfRuntime"]) == rt
    runner = rt["spec"]["engineConfig"]["runner"]
    assert runner["command"] == ["python3", "-m", "ome_amd.runtime.server"] and runner["resources"]["limits"]["amd.com/gpu"] == "1"
    assert runner["env"] == [{"name": "OME_X", "value": "1"}] and rt["spec"]["volumes"] == [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]
    assert res["multinode"]["spec"]["engineConfig"]["worker"]["size"] == 1
    assert res["service"]["metadata"]["annotations"] == {"ome.io/autoscalerClass": "hpa", "ome.io/metrics": "cpu",
                                                         "ome.io/targetUtilizationPercentage": "80"}

    c = Cluster(str(tmp_path), with_agent=False, with_executor=False)
    c.start()
    try:
        client = TestClient(create_app(c.store))
        model = dict(res["model"])
        assert model["kind"] == "ClusterBaseModel" and model["spec"]["storage"]["nodeSelector"]
        for key in ("model", "runtime", "multinode"):
            obj = res[key]
            r = client.post("/api/v1/validate/yaml", content=yaml.safe_dump(obj), headers={"content-type": "application/yaml"}).json()
            assert r["valid"], (key, r)
        # create the model + runtime through the console API as the forms do, then the dependent kinds
        assert client.post("/api/v1/models", json=model).status_code == 201
        assert client.post("/api/v1/runtimes", json=res["runtime"]).status_code == 201
        for key in ("service", "keda", "bench"):
            r = client.post("/api/v1/validate/yaml", content=yaml.safe_dump(res[key]), headers={"content-type": "application/yaml"}).json()
            assert r["valid"], (key, r)
        assert client.post("/api/v1/services", json=res["service"]).status_code == 201
        assert client.get("/api/v1/runtimes/recommend", params={"model": "llama-3-8b"}).json()["runtime"] == "my-runtime"
    finally:
        c.shutdown()


def test_runtime_catalog_and_github_import(tmp_path):
    c = Cluster(str(tmp_path), with_agent=False, with_executor=False)
    c.start()
    try:
        client = TestClient(create_app(c.store))
        cat = client.get("/api/v1/runtimes/catalog").json()
        assert cat["total"] > 50 and all(f["path"].endswith(".yaml") for f in cat["files"])
        one = next(f for f in cat["files"] if f["path"].startswith("runtimes/ome-amd/"))
        assert not one["installed"]
        # a GitHub blob URL of a repository laid out like the catalog maps onto the local file
        url = f"https://github.com/acme/ome-amd/blob/main/config/{one['path']}"
        r = client.get("/api/v1/runtimes/fetch-yaml", params={"path": url})
        assert r.status_code == 200 and r.json()["runtime"]["metadata"]["name"] == one["name"]
        rel = client.get("/api/v1/runtimes/fetch-yaml", params={"path": one["path"][len("runtimes/"):]})
        assert rel.status_code == 200
        for bad in ("../../../etc/passwd", "https://github.com/a/b/blob/main/../../../../etc/hosts", "/etc/hostname"):
            assert client.get("/api/v1/runtimes/fetch-yaml", params={"path": bad}).status_code == 400
        # importing marks it installed (the catalog runtimes name the MI355X / MI300X classes)
        for acc in ("amd-mi355x", "amd-mi300x"):
            c.store.create({"apiVersion": "ome.io/v1beta1", "kind": "AcceleratorClass", "metadata": {"name": acc},
                            "spec": {"vendor": "amd"}})
        assert client.post("/api/v1/runtimes", content=r.json()["yaml"], headers={"content-type": "application/yaml"}).status_code == 201
        cat2 = client.get("/api/v1/runtimes/catalog").json()
        assert next(f for f in cat2["files"] if f["path"] == one["path"])["installed"]
    finally:
        c.shutdown()


def test_shell_loads_every_script_and_routes_exist(tmp_path):
    c = Cluster(str(tmp_path), with_agent=False, with_executor=False)
    try:
        client = TestClient(create_app(c.store))
        html = client.get("/").text
        order = [m.group(1) for m in re.finditer(r'<script src="static/([a-z]+\.js)"', html)]
        assert order == ["lib.js", "forms.js", "app.js"]
        for f in order:
            assert client.get(f"/static/{f}").status_code == 200
        app = (STATIC / "app.js").read_text()
        for view in ("RuntimeImport", "BenchmarkNew", "ModelNew", "ServiceDeploy", "dataTable", "loadNamespaces"):
            assert f"function {view}(" in app or f"async function {view}(" in app, view
        for pattern in (r"runtimes\/import", r"benchmarks\/new", r"models\/ns\/"):
            assert pattern in app, pattern
    finally:
        c.shutdown()

"""ome-agent subcommands, prober, metrics aggregator, storage backends (CPU, no network)."""
import base64
import json
import os
import subprocess
import sys
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer
from pathlib import Path

import pytest
import torch

from ome_amd.agent.__main__ import main as agent_main, sync_adapters
from ome_amd.io import native
from ome_amd.io.safetensors import count_params, read_header, save_file
from ome_amd.metrics_aggregator import add_labels
from ome_amd.storage import backends

pytestmark = pytest.mark.skipif(not native.available(), reason="libomeio not built")


def _model(d: Path) -> Path:
    d.mkdir(parents=True, exist_ok=True)
    save_file({"w": torch.arange(12, dtype=torch.float32).view(3, 4), "b": torch.ones(5, dtype=torch.bfloat16)},
              d / "model.safetensors", {"format": "pt"})
    (d / "config.json").write_text(json.dumps({"architectures": ["LlamaForCausalLM"], "model_type": "llama",
                                               "hidden_size": 64, "num_hidden_layers": 2, "num_attention_heads": 4,
                                               "intermediate_size": 128, "vocab_size": 100,
                                               "max_position_embeddings": 256, "torch_dtype": "bfloat16"}))
    return d


def test_safetensors_header_native_matches_python(tmp_path):
    m = _model(tmp_path / "m")
    hdr, off = read_header(m / "model.safetensors")
    assert hdr["w"]["shape"] == [3, 4] and hdr["__metadata__"]["format"] == "pt"
    assert count_params(m / "model.safetensors") == 17
    with pytest.raises(Exception):
        (tmp_path / "bad.safetensors").write_bytes(b"\xff" * 16)
        read_header(tmp_path / "bad.safetensors")


def test_encrypt_enigma_roundtrip(tmp_path, monkeypatch):
    m = _model(tmp_path / "m")
    orig = (m / "model.safetensors").read_bytes()
    mek = base64.b64encode(os.urandom(32)).decode()
    monkeypatch.setenv("OME_MEK", mek)
    assert agent_main(["encrypt", "--local-path", str(m), "--config", "/nonexistent"]) == 0
    enc = (m / "model.safetensors").read_bytes()
    assert enc != orig and len(enc) == len(orig) + 28
    assert (m / "config.json").read_text().startswith("{")  # metadata stays readable
    # wrong master key: authentication fails, weights untouched
    monkeypatch.setenv("OME_MEK", base64.b64encode(os.urandom(32)).decode())
    assert agent_main(["enigma", "--local-path", str(m), "--config", "/nonexistent"]) == 1
    assert (m / "model.safetensors").read_bytes() == enc
    monkeypatch.setenv("OME_MEK", mek)
    assert agent_main(["enigma", "--local-path", str(m), "--config", "/nonexistent"]) == 0
    assert (m / "model.safetensors").read_bytes() == orig
    assert not (m / ".ome-dek").exists()


def test_object_store_fetch_verifies_md5(tmp_path, monkeypatch):
    monkeypatch.setenv("OME_OBJECT_STORE_ROOT", str(tmp_path / "os"))
    src = _model(tmp_path / "os" / "oci" / "ns" / "bkt" / "models" / "m")
    backends.write_manifest(src)
    res = backends.fetch("oci://n/ns/b/bkt/o/models/m", str(tmp_path / "dst"))
    assert (tmp_path / "dst" / "model.safetensors").read_bytes() == (src / "model.safetensors").read_bytes()
    assert res.sha and res.files == 2
    # corrupt the source object after the manifest was written -> MD5 mismatch
    (src / "model.safetensors").write_bytes(b"x" * 10)
    with pytest.raises(backends.FetchError):
        backends.fetch("oci://n/ns/b/bkt/o/models/m", str(tmp_path / "dst2"))


def test_replica_and_random(tmp_path, monkeypatch):
    monkeypatch.setenv("OME_OBJECT_STORE_ROOT", str(tmp_path / "os"))
    assert agent_main(["replica", "--source", "random://tiny-llama", "--target", "s3://bucket/tiny",
                       "--config", "/nonexistent"]) == 0
    out = tmp_path / "os" / "s3" / "bucket" / "tiny"
    assert json.loads((out / "config.json").read_text())["hidden_size"] == 256
    assert (out / ".ome-manifest.json").exists()


def test_serving_agent_sync(tmp_path):
    a1 = _model(tmp_path / "src" / "a1")
    spec = tmp_path / "adapters.json"
    spec.write_text(json.dumps([{"name": "a1", "storageUri": f"local://{a1}"}]))
    added, removed = sync_adapters(spec, tmp_path / "ft")
    assert added == ["a1"] and (tmp_path / "ft" / "a1" / "model.safetensors").exists()
    spec.write_text("[]")
    added, removed = sync_adapters(spec, tmp_path / "ft")
    assert removed == ["a1"] and not (tmp_path / "ft" / "a1").exists()


def test_model_metadata_job(tmp_path, capsys):
    m = _model(tmp_path / "m")
    assert agent_main(["model-metadata", "--model-path", str(m), "--config", "/nonexistent"]) == 0
    patch = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert patch["spec"]["modelArchitecture"] == "LlamaForCausalLM"
    assert patch["spec"]["modelParameterSize"] == "17"  # safetensors header count wins


def test_metrics_aggregator_labels():
    text = "# TYPE x_total untyped\nx_total{a=\"1\"} 3\ny 2\n# TYPE c_created untyped\nc_created 5\n"
    out = add_labels(text, {"service_name": "svc"})
    assert 'x_total{a="1",service_name="svc"} 3' in out and 'y{service_name="svc"} 2' in out
    assert "# TYPE x_total gauge" in out and "# TYPE c_created counter" in out


def test_prober_against_fake_engine():
    from fastapi.testclient import TestClient

    from ome_amd.prober import Prober, create_app

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            body = json.dumps({"data": [{"id": "m1"}]}).encode() if self.path == "/v1/models" else b"ok"
            self.send_response(200)
            self.end_headers()
            self.wfile.write(body)

        def do_POST(self):
            n = int(self.headers["Content-Length"])
            seen.append(json.loads(self.rfile.read(n)))
            self.send_response(200)
            self.end_headers()
            self.wfile.write(b"{}")

    seen = []
    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    c = TestClient(create_app(Prober(f"http://127.0.0.1:{srv.server_port}/health")))
    assert c.get("/healthz").status_code == 200 and c.get("/readyz").status_code == 200
    assert c.get("/startupz").status_code == 200 and seen[0]["model"] == "m1"
    dead = TestClient(create_app(Prober("http://127.0.0.1:1", timeout=0.5)))
    assert dead.get("/healthz").status_code == 503
    assert 'probe="healthz",result="fail"' in dead.get("/metrics").text
    srv.shutdown()

"""Our Hugging Face hub client against a local fake Hub: repo listing with LFS metadata, HEAD
metadata without following the CDN redirect, ranged parallel downloads through the redirect,
SHA-256 verification, glob filters, resume, gated repos, and the hf:// fetch backend."""
import hashlib
import json
import os
import sys
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd.storage import hfhub  # noqa: E402

SHA = "a" * 40


class FakeHub:
    def __init__(self):
        self.files = {"config.json": b'{"architectures": ["LlamaForCausalLM"], "model_type": "llama"}',
                      "model-00001-of-00002.safetensors": os.urandom(5000),
                      "model-00002-of-00002.safetensors": os.urandom(3333),
                      "README.md": b"# hi", "original/consolidated.pth": os.urandom(100)}
        self.lfs = {k for k in self.files if k.endswith((".safetensors", ".pth"))}
        self.gated = set()
        self.corrupt = set()
        self.range_gets = 0
        hub = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body=b"", headers=None):
                self.send_response(code)
                for k, v in (headers or {}).items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                if self.command != "HEAD":
                    self.wfile.write(body)

            def do_HEAD(self):
                self.do_GET()

            def do_GET(self):
                u = urllib.parse.urlsplit(self.path)
                path = urllib.parse.unquote(u.path)
                if path.startswith("/api/models/"):
                    repo = path[len("/api/models/"):].split("/revision/")[0]
                    if repo in hub.gated and self.headers.get("Authorization") != "Bearer good":
                        return self._send(401, b'{"error": "gated"}')
                    if repo != "org/m":
                        return self._send(404, b"{}")
                    sib = []
                    for k, v in hub.files.items():
                        e = {"rfilename": k, "blobId": hashlib.sha1(v).hexdigest()}
                        if k in hub.lfs:
                            e["lfs"] = {"sha256": hashlib.sha256(v).hexdigest(), "size": len(v)}
                        sib.append(e)
                    return self._send(200, json.dumps({"id": repo, "sha": SHA, "siblings": sib}).encode())
                if path.startswith("/cdn/"):
                    name = path[len("/cdn/"):]
                    data = hub.files[name]
                    if name in hub.corrupt:
                        data = data[:-1] + bytes([data[-1] ^ 1])
                    rng = self.headers.get("Range")
                    if rng:
                        hub.range_gets += 1
                        a, b = (int(x) for x in rng.split("=")[1].split("-"))
                        return self._send(206, data[a:b + 1])
                    return self._send(200, data)
                if "/resolve/" in path:
                    repo, rest = path.lstrip("/").split("/resolve/", 1)
                    rev, name = rest.split("/", 1)
                    data = hub.files.get(name)
                    if data is None:
                        return self._send(404)
                    h = {"X-Repo-Commit": SHA, "ETag": f'"{hashlib.sha1(data).hexdigest()}"'}
                    if name in hub.lfs:
                        h.update({"X-Linked-Etag": f'"{hashlib.sha256(data).hexdigest()}"',
                                  "X-Linked-Size": str(len(data)), "Location": f"/cdn/{name}"})
                        return self._send(302, b"", h)
                    rng = self.headers.get("Range")
                    if rng and self.command == "GET":
                        hub.range_gets += 1
                        a, b = (int(x) for x in rng.split("=")[1].split("-"))
                        return self._send(206, data[a:b + 1], h)
                    return self._send(200, data, h)
                return self._send(404)

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()


@pytest.fixture
def hub():
    h = FakeHub()
    yield h
    h.close()


def test_listing_and_head_metadata(hub):
    c = hfhub.HfHub(hub.url)
    sha, files = c.files("org/m")
    assert sha == SHA and {f.name for f in files} == set(hub.files)
    st = next(f for f in files if f.name.endswith("00001-of-00002.safetensors"))
    assert st.sha256_hex == hashlib.sha256(hub.files[st.name]).hexdigest() and st.size == 5000
    md = c.file_metadata("org/m", st.name)
    assert md["etag"] == st.sha256_hex and md["size"] == 5000 and md["commit"] == SHA
    assert md["location"].endswith(f"/cdn/{st.name}")


def test_snapshot_ranged_verified_filtered_and_resumed(hub, tmp_path):
    st = hfhub.snapshot_download("org/m", tmp_path / "m", endpoint=hub.url, part_size=1000, workers=4,
                                 ignore_patterns=["original/*", "*.md"])
    assert st["files"] == 3 and st["verified"] == 2 and st["parts"] == 1 + 5 + 4
    for k in ("config.json", "model-00001-of-00002.safetensors", "model-00002-of-00002.safetensors"):
        assert (tmp_path / "m" / k).read_bytes() == hub.files[k]
    assert not (tmp_path / "m" / "README.md").exists() and (tmp_path / "m" / ".ome-hf-commit").read_text() == SHA
    # second run: everything already present and verified -> no range requests
    n0 = hub.range_gets
    st2 = hfhub.snapshot_download("org/m", tmp_path / "m", endpoint=hub.url, part_size=1000,
                                  ignore_patterns=["original/*", "*.md"])
    assert hub.range_gets == n0 and st2["fetched_parts"] == 0


def test_sha256_mismatch_and_gated(hub, tmp_path):
    hub.corrupt.add("model-00002-of-00002.safetensors")
    with pytest.raises(hfhub.O.ObjectStoreError, match="SHA-256"):
        hfhub.snapshot_download("org/m", tmp_path / "x", endpoint=hub.url, allow_patterns=["*00002*"])
    hub.corrupt.clear()
    hub.gated.add("org/m")
    with pytest.raises(hfhub.HfHubError, match="gated"):
        hfhub.snapshot_download("org/m", tmp_path / "y", endpoint=hub.url)
    st = hfhub.snapshot_download("org/m", tmp_path / "y", endpoint=hub.url, token="good", allow_patterns=["*.json"])
    assert st["files"] == 1


def test_fetch_backend_uses_the_hub_client(hub, tmp_path, monkeypatch):
    from ome_amd.storage.backends import FetchError, fetch

    monkeypatch.setenv("HF_ENDPOINT", hub.url)
    monkeypatch.delenv("HF_HUB_OFFLINE", raising=False)
    monkeypatch.setenv("OME_HF_IGNORE_PATTERNS", "original/*")
    res = fetch("hf://org/m@main", str(tmp_path / "out"))
    assert res.sha == SHA and res.files == 4 and (tmp_path / "out" / "config.json").exists()
    with pytest.raises(FetchError, match="not found"):
        fetch("hf://org/missing", str(tmp_path / "o2"))

"""A streaming client that goes away mid-generation must not keep the engine busy: the server
aborts the request when its SSE generator is closed (found by the e2e sweep, where abandoned
1000-token requests starved the following load points)."""
import json
import os
import socket
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _info(base):
    with urllib.request.urlopen(base + "/get_server_info", timeout=5) as r:
        return json.loads(r.read())


def test_stream_disconnect_aborts_request(tmp_path):
    from ome_amd.bench import e2e

    proc, base = e2e.start_server("tiny-llama", 4, 2048, ["--device", "cpu", "--disable-cuda-graph"],
                                  log_path=str(tmp_path / "server.log"))
    try:
        e2e.wait_ready(base, proc, timeout=300)
        port = int(base.rsplit(":", 1)[1])
        body = json.dumps({"model": "m", "prompt": [5, 6, 7], "max_tokens": 1900, "ignore_eos": True,
                           "stream": True}).encode()
        s = socket.create_connection(("127.0.0.1", port))
        s.sendall(b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                  + f"Content-Length: {len(body)}\r\n\r\n".encode() + body)
        got = b""
        while got.count(b"data: ") < 3:
            got += s.recv(4096)
        assert _info(base)["running"] == 1
        s.close()   # client disappears mid-stream
        t0 = time.time()
        while time.time() - t0 < 5 and _info(base)["running"] != 0:
            time.sleep(0.2)
        assert _info(base)["running"] == 0, open(tmp_path / "server.log").read()[-2000:]
    finally:
        e2e.stop_server(proc)

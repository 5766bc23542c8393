"""Model-agent observability and rate-limit resilience with the reference's contract:
metric series names / labels of pkg/modelagent/metrics.go:142-201, HTTP 429 + Retry-After
handling (gopher.go:1134-1137), deterministic start-up jitter (cmd/model-agent/main.go:229-239)."""
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest
from prometheus_client import generate_latest

from ome_amd.modelagent import metrics as M
from ome_amd.modelagent.__main__ import startup_jitter_s
from ome_amd.storage import objstore as O


class _Srv:
    def __init__(self, plan):
        self.plan, self.hits = list(plan), 0
        srv = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                srv.hits += 1
                code, hdrs = srv.plan.pop(0) if srv.plan else (200, {})
                body = b"payload" if code == 200 else b"slow down"
                self.send_response(code)
                for k, v in hdrs.items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}/x"
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()

    def close(self):
        self.httpd.shutdown()


def test_429_honours_retry_after_and_records_waits():
    srv = _Srv([(429, {"Retry-After": "0.2"}), (429, {}), (200, {})])
    try:
        h = O._Http(None, default_wait=0.1)
        t0 = time.time()
        code, _, body = h("GET", srv.url)
        assert code == 200 and body == b"payload" and srv.hits == 3
        assert h.rate_limit_waits == [0.2, 0.1] and time.time() - t0 >= 0.3
    finally:
        srv.close()


def test_429_budget_exhausted_raises_rate_limit_error():
    srv = _Srv([(429, {"Retry-After": "0"})] * 10)
    try:
        h = O._Http(None, rate_limit_retries=3)
        with pytest.raises(O.RateLimitError) as ei:
            h("GET", srv.url)
        assert ei.value.status == 429 and len(ei.value.waits) == 3 and srv.hits == 4
    finally:
        srv.close()


def test_retry_after_http_date_and_garbage():
    import email.utils

    future = email.utils.formatdate(time.time() + 30, usegmt=True)
    assert 25 <= O.retry_after_seconds(future, 5.0) <= 31
    assert O.retry_after_seconds("soon", 7.0) == 7.0 and O.retry_after_seconds(None, 3.0) == 3.0


def _val(text: str, series: str) -> float:
    for line in text.splitlines():
        if line.startswith(series + " ") or line.startswith(series + "{") and line.split(" ")[0] == series:
            return float(line.rsplit(" ", 1)[1])
    return 0.0


def test_metric_series_names_and_labels():
    cbm = {"kind": "ClusterBaseModel", "metadata": {"name": "llama"}}
    bm = {"kind": "BaseModel", "metadata": {"name": "qwen", "namespace": "team-a"}}
    M.record_success(cbm)
    M.record_failed(bm, "hf_download_error")
    M.record_rate_limit(bm, 4.0)
    M.record_verification(cbm, True)
    M.record_verification(bm, False)
    M.record_bytes(cbm, 1234)
    M.observe_download(cbm, 2.5)
    M.observe_verification(0.3)
    text = generate_latest(M.REGISTRY).decode()
    lab = 'model_type="ClusterBaseModel",name="llama",namespace=""'   # exposition sorts label names
    labb = 'model_type="BaseModel",name="qwen",namespace="team-a"'
    assert _val(text, f"model_agent_downloads_success_total{{{lab}}}") >= 1
    assert _val(text, f"model_agent_downloads_failed_total{{{labb}}}") >= 1
    assert _val(text, f"model_agent_rate_limit_total{{{labb}}}") >= 1
    assert _val(text, f'model_agent_verifications_total{{{lab},result="success"}}') >= 1
    assert _val(text, f'model_agent_verifications_total{{{labb},result="failure"}}') >= 1
    assert _val(text, f"model_agent_md5_checksum_failed_total{{{labb}}}") >= 1
    assert _val(text, f"model_agent_download_bytes_total{{{lab}}}") >= 1234
    for name in ("model_agent_download_duration_seconds_bucket", "model_agent_rate_limit_wait_seconds_bucket",
                 "model_agent_verification_duration_seconds_bucket"):
        assert name in text
    assert 'model_agent_download_duration_seconds_bucket{le="0.1"' in text or \
        'model_agent_download_duration_seconds_bucket{model_type' in text


def test_startup_jitter_is_deterministic_per_node():
    d = [startup_jitter_s(f"node-{i}") for i in range(40)]
    assert all(0 <= x < 30 for x in d) and len(set(d)) > 10          # spread over the window
    assert 0 <= startup_jitter_s("mi355x-node-0-with-a-long-name") < 30   # int64 wrap handled
    assert startup_jitter_s("node-7") == d[7]                          # same node, same delay
    h = 0
    for c in "gpu-n07":                                                 # short: no int64 wrap
        h = h * 31 + ord(c)
    assert startup_jitter_s("gpu-n07") == float(h % 30)                # the reference formula
    assert startup_jitter_s("n", 0) == 0.0 and startup_jitter_s("", 30) == 0.0

"""Local executor: real processes, probes, restarts, LWS group recreation on rank loss (fault
injection), Job completion, service proxy, and the metrics autoscaler's PromQL subset."""
import sys
import time

import pytest

from ome_amd.executor.autoscaler import PromQL, SeriesHistory, desired_from_keda, parse_prom_text
from ome_amd.manager import Cluster

PY = sys.executable
SLEEPER = {"name": "c", "image": "busybox", "command": [PY, "-c", "import time; time.sleep(600)"]}


def _wait(cl, pred, timeout=30.0):
    end = time.time() + timeout
    while time.time() < end:
        cl.step(1)
        if pred():
            return True
        time.sleep(0.1)
    return False


@pytest.fixture
def cluster(tmp_path):
    cl = Cluster(str(tmp_path / "state"), gpus=8, with_agent=False)
    cl.executor.kubelet.restart_backoff = 0.05
    yield cl
    cl.shutdown()


def _ready(p):
    return any(c["type"] == "Ready" and c["status"] == "True" for c in (p.get("status") or {}).get("conditions") or [])


def test_lws_group_restart_on_rank_kill(cluster):
    tmpl = {"metadata": {"labels": {"app": "g"}}, "spec": {"containers": [dict(SLEEPER)]}}
    cluster.apply([{"apiVersion": "leaderworkerset.x-k8s.io/v1", "kind": "LeaderWorkerSet",
                    "metadata": {"name": "grp", "namespace": "default"},
                    "spec": {"replicas": 1, "leaderWorkerTemplate": {"size": 2, "leaderTemplate": tmpl,
                                                                    "workerTemplate": tmpl}}}])
    pods = lambda: {p["metadata"]["name"]: p for p in cluster.store.list("v1", "Pod", "default")}  # noqa: E731
    assert _wait(cluster, lambda: len(pods()) == 2 and all(_ready(p) for p in pods().values()))
    uids = {n: p["metadata"]["uid"] for n, p in pods().items()}
    assert cluster.executor.kubelet.inject_fault("default", "grp-0-1")  # SIGKILL the worker rank
    # the kubelet restarts the container, the LWS controller then recreates the WHOLE group
    assert _wait(cluster, lambda: len(pods()) == 2 and all(p["metadata"]["uid"] != uids[n]
                                                             for n, p in pods().items()) and
                 all(_ready(p) for p in pods().values()), timeout=40)


def test_job_completion_and_failure(cluster):
    ok = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "ok", "namespace": "default"},
          "spec": {"template": {"spec": {"containers": [{"name": "c", "image": "x",
                                                         "command": [PY, "-c", "print('done')"]}]}}}}
    bad = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "bad", "namespace": "default"},
           "spec": {"template": {"spec": {"containers": [{"name": "c", "image": "x",
                                                          "command": [PY, "-c", "import sys; sys.exit(3)"]}]}}}}
    cluster.apply([ok, bad])
    cond = lambda n, t: any(c["type"] == t and c["status"] == "True" for c in  # noqa: E731
                            (cluster.store.get("batch/v1", "Job", n, "default").get("status") or {}).get("conditions")
                            or [])
    assert _wait(cluster, lambda: cond("ok", "Complete") and cond("bad", "Failed"))
    assert "done" in cluster.executor.kubelet.logs("default", "ok-0")


def test_readiness_probe_and_service_proxy(cluster):
    srv = (f"import http.server,os\nclass H(http.server.BaseHTTPRequestHandler):\n"
           f"  def do_GET(s):\n    s.send_response(200); s.end_headers(); s.wfile.write(b'hi')\n"
           f"  def log_message(s,*a): pass\n"
           f"http.server.HTTPServer(('127.0.0.1', int(os.environ['PORT'])), H).serve_forever()")
    dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web", "namespace": "default"},
           "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "web"}},
                    "template": {"metadata": {"labels": {"app": "web"}}, "spec": {"containers": [{
                        "name": "c", "image": "x", "command": [PY, "-c", srv],
                        "env": [{"name": "PORT", "value": "8080"}], "ports": [{"containerPort": 8080}],
                        "readinessProbe": {"httpGet": {"path": "/", "port": 8080}, "periodSeconds": 1}}]}}}}
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web", "namespace": "default"},
           "spec": {"selector": {"app": "web"}, "ports": [{"port": 80, "targetPort": 8080}]}}
    cluster.apply([dep, svc])
    assert _wait(cluster, lambda: (cluster.store.get("apps/v1", "Deployment", "web", "default").get("status") or {})
                 .get("readyReplicas") == 2)
    import json
    import os
    import urllib.request

    os.environ["OME_LOCAL_DNS"] = cluster.executor.kubelet.proxies.dns_path
    from ome_amd.executor.dns import resolve_url

    url = resolve_url("http://web.default.svc.cluster.local:80/")
    assert urllib.request.urlopen(url, timeout=5).read() == b"hi"
    del json


def test_promql_subset_and_keda_math():
    h = SeriesHistory()
    h.add({"vllm:request_success_total": 100.0, "sglang:num_running_reqs": 12.0}, t=1000.0)
    h.add({"vllm:request_success_total": 160.0, "sglang:num_running_reqs": 30.0}, t=1060.0)
    assert PromQL('sum(sglang:num_running_reqs{ome_io_inferenceservice="x"})').eval(h, now=1060) == 30.0
    assert abs(PromQL("sum(rate(vllm:request_success_total[5m]))").eval(h, now=1060) - 1.0) < 1e-9
    assert PromQL("avg_over_time(sglang:num_running_reqs[5m]) > bool 20").eval(h, now=1060) == 1.0
    assert PromQL("sum(rate(vllm:request_success_total[1m]) > bool 0.50) * 2").eval(h, now=1060) == 2.0
    assert desired_from_keda(30.0, 10.0, 1) == 3
    assert parse_prom_text('a{x="1"} 2\na{x="2"} 3\n# c\nb 1e3\n') == {"a": 5.0, "b": 1000.0}


def test_lws_group_restart_when_a_rank_watchdog_exits(cluster, tmp_path):
    """A rank that detects a collective expiry exits with EXIT_COLLECTIVE on its own (the engine
    watchdog, runtime/watchdog.py); the LWS RecreateGroupOnPodRestart path then rebuilds the whole
    group, exactly as for a killed rank."""
    from ome_amd.runtime.watchdog import EXIT_COLLECTIVE

    marker = tmp_path / "fired-once"
    code = ("import os, time\n"
            f"m = {str(marker)!r}\n"
            "if os.environ.get('LWS_WORKER_INDEX', '0') != '0' and not os.path.exists(m):\n"
            "    open(m, 'w').close()\n"
            "    from ome_amd.runtime import watchdog as W\n"
            "    t0 = time.time()\n"
            # the collective error surfaces 5 s in, after the test has recorded the first pod uids
            "    W.register_comm('allreduce(rank 1/2)', lambda: 1 if time.time() > t0 + 5 else 0)\n"
            "    W.Watchdog(60.0, rank=1, poll_s=0.05)\n"
            "time.sleep(600)\n")
    c = {"name": "c", "image": "busybox", "command": [PY, "-c", code]}
    tmpl = {"metadata": {"labels": {"app": "w"}}, "spec": {"containers": [c]}}
    cluster.apply([{"apiVersion": "leaderworkerset.x-k8s.io/v1", "kind": "LeaderWorkerSet",
                    "metadata": {"name": "wd", "namespace": "default"},
                    "spec": {"replicas": 1, "leaderWorkerTemplate": {
                        "size": 2, "restartPolicy": "RecreateGroupOnPodRestart",
                        "leaderTemplate": tmpl, "workerTemplate": tmpl}}}])
    pods = lambda: {p["metadata"]["name"]: p for p in cluster.store.list("v1", "Pod", "default")}  # noqa: E731
    assert _wait(cluster, lambda: len(pods()) == 2 and marker.exists(), timeout=40)
    first = {n: p["metadata"]["uid"] for n, p in pods().items()}
    # the worker exited 75 (its container restart is recorded) and the group was recreated
    assert _wait(cluster, lambda: len(pods()) == 2 and all(p["metadata"]["uid"] != first.get(n)
                                                             for n, p in pods().items())
                 and all(_ready(p) for p in pods().values()), timeout=150)
    assert EXIT_COLLECTIVE == 75

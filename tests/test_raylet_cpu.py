"""MultiNodeRayVLLM without Ray (``ome_amd.raylet``): the executor's command translation maps the
RayCluster pods' ``ray start`` / ``ray_init.sh`` / ``vllm serve --distributed-executor-backend ray``
onto the rendezvous agent and the server; a head store, one worker agent and a TP=2 head server
(one rank per "node", CPU, gloo) form the group and serve a completion."""
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

from ome_amd.executor.kubelet import translate_command


def test_ray_commands_translate_to_the_agent():
    assert translate_command("ray start --head --port=6379").endswith("-m ome_amd.raylet start --head --port=6379")
    t = translate_command("ulimit -n 65536; echo worker; ray start --address=h:6379 --block")
    assert "-m ome_amd.raylet start --address=h:6379 --block" in t and "ulimit -n 65536" in t
    t = translate_command("/workspace/ray_init.sh leader --ray_cluster_size=2; vllm serve /m "
                          "--tensor-parallel-size 16 --distributed-executor-backend ray")
    assert "-m ome_amd.raylet init leader --ray_cluster_size=2" in t
    assert "-m ome_amd.runtime.server --model-path /m --tensor-parallel-size 16" in t
    assert translate_command("ray stop").endswith("-m ome_amd.raylet stop")


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _get(url: str, timeout=5.0):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.status, r.read()


@pytest.mark.timeout(400)
def test_ray_backend_group_serves_over_two_nodes():
    gcs, http, whttp = _port(), _port(), _port()
    env = dict(os.environ, OME_RAY_ADDRESS=f"127.0.0.1:{gcs}", OME_RAY_GPUS_PER_NODE="1",
               OME_RAY_WORKER_PORT=str(whttp), OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    py = sys.executable
    procs = []

    def spawn(args):
        p = subprocess.Popen([py, "-m", *args], env=env, start_new_session=True, stdout=subprocess.DEVNULL,
                             stderr=subprocess.DEVNULL)
        procs.append(p)
        return p

    try:
        spawn(["ome_amd.raylet", "start", "--head", f"--port={gcs}", "--block"])          # head pod's ray start
        spawn(["ome_amd.raylet", "start", f"--address=127.0.0.1:{gcs}", "--block"])       # worker pod
        head = spawn(["ome_amd.runtime.server", "--model-path", "random://tiny-llama", "--device", "cpu",
                      "--dtype", "float32", "--tensor-parallel-size", "2", "--distributed-executor-backend", "ray",
                      "--host", "127.0.0.1", "--port", str(http), "--context-length", "256",
                      "--max-running-requests", "4"])
        t0 = time.time()
        while True:
            assert head.poll() is None, "head server exited"
            try:
                if _get(f"http://127.0.0.1:{http}/health")[0] == 200:
                    break
            except OSError:
                pass
            assert time.time() - t0 < 300, "head server not ready"
            time.sleep(1.0)
        assert _get(f"http://127.0.0.1:{whttp}/health")[0] == 200          # node 1's ranks are up
        req = urllib.request.Request(f"http://127.0.0.1:{http}/v1/completions", method="POST",
                                     data=json.dumps({"prompt": [5, 6, 7, 8], "max_tokens": 5,
                                                      "temperature": 0}).encode(),
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            out = json.loads(r.read())
        assert out["usage"]["completion_tokens"] == 5
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
            p.wait(timeout=30)

"""SURVEY §7.3 slice on a real GPU: ClusterBaseModel (``random://<preset>``) + ClusterServingRuntime
(``amd.com/gpu: 1``) + InferenceService reconciled by the in-process operator; the node executor
launches ``ome_amd.runtime.server`` on the allotted GPU(s); a BenchmarkJob then drives it through
``ome_amd.bench.loadgen`` (the reference's genai-bench contract,
``pkg/controller/v1beta1/benchmark/controller.go:499-557``).  Used by ``tests/test_operator_gpu.py``
(short limits) and ``scripts/operator_bench_gpu.py`` (the protocol sweep)."""
from __future__ import annotations

import json
import os
import time
from pathlib import Path

from ome_amd.api import constants as C
from ome_amd.manager import Cluster

API = C.API_VERSION


def runtime(name: str, served: str, arch: str = "LlamaForCausalLM", size=("1B", "100B"), gpus: int = 1,
            extra_args: list[str] | None = None) -> dict:
    cmd = ["python3", "-m", "sglang.launch_server", "--host", "0.0.0.0", "--port", "8080",
           "--model-path", "$(MODEL_PATH)", "--served-model-name", served, "--enable-metrics",
           "--tp-size", str(gpus)] + list(extra_args or [])
    return {
        "apiVersion": API, "kind": "ClusterServingRuntime", "metadata": {"name": name},
        "spec": {
            "supportedModelFormats": [{"modelFormat": {"name": "safetensors", "version": "1.0.0"},
                                       "modelFramework": {"name": "transformers", "version": "4.46.0"},
                                       "modelArchitecture": arch, "autoSelect": True, "priority": 1}],
            "protocolVersions": ["openAI"], "modelSizeRange": {"min": size[0], "max": size[1]},
            "engineConfig": {"runner": {
                "name": "ome-container", "image": "docker.io/lmsysorg/sglang:v0.5",
                "ports": [{"containerPort": 8080, "name": "http1"}],
                "command": cmd,
                "resources": {"limits": {C.GPU_RESOURCE: gpus}, "requests": {C.GPU_RESOURCE: gpus}},
                "readinessProbe": {"httpGet": {"path": "/health", "port": 8080}, "periodSeconds": 1},
                "startupProbe": {"httpGet": {"path": "/health_generate", "port": 8080}, "periodSeconds": 2,
                                 "failureThreshold": 300, "timeoutSeconds": 60},
                "livenessProbe": {"httpGet": {"path": "/health", "port": 8080}, "periodSeconds": 10,
                                  "failureThreshold": 6, "timeoutSeconds": 30},
            }},
        }}


def base_model(name: str, preset: str, root: Path) -> dict:
    return {"apiVersion": API, "kind": "ClusterBaseModel", "metadata": {"name": name},
            "spec": {"vendor": "meta", "storage": {"storageUri": f"random://{preset}", "path": str(root / name)}}}


def isvc(name: str, model: str) -> dict:
    return {"apiVersion": API, "kind": "InferenceService", "metadata": {"name": name, "namespace": "default"},
            "spec": {"model": {"name": model}, "engine": {"minReplicas": 1, "maxReplicas": 1}}}


def benchmark_job(name: str, svc: str, scenarios, concurrency, max_time: int, max_requests: int, out: Path) -> dict:
    return {"apiVersion": API, "kind": "BenchmarkJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"endpoint": {"inferenceService": {"name": svc, "namespace": "default"}},
                     "task": "text-to-text", "trafficScenarios": list(scenarios), "numConcurrency": list(concurrency),
                     "maxTimePerIteration": max_time, "maxRequestsPerIteration": max_requests,
                     "resultFolderName": "exp", "outputLocation": {"storageUri": f"local://{out}"}}}


def ready(obj: dict) -> bool:
    return any(c.get("type") == "Ready" and c.get("status") == "True"
               for c in (obj.get("status") or {}).get("conditions") or [])


def run(work: Path, preset: str = "llama-3-8b", scenarios=("D(100,100)",), concurrency=(1, 4, 16),
        max_time: int = 5, max_requests: int = 16, gpus: int = 1, extra_args=None, log=print,
        startup_timeout: float = 600, bench_timeout: float = 1200) -> dict:
    """Reconcile the slice, wait for Ready, run the BenchmarkJob; returns {"isvc", "summary",
    "timings"}.  Raises RuntimeError (with pod logs) on a failure."""
    work = Path(work)
    t0 = time.time()
    cl = Cluster(str(work / "state"), gpus=gpus, probe_scale=1.0)
    timings = {}
    try:
        cl.apply([runtime("slice-rt", "llama", gpus=gpus, extra_args=extra_args),
                  base_model("slice-model", preset, work / "models")])
        cl.start()
        if not cl.wait_for(lambda: (cl.store.get(API, "ClusterBaseModel", "slice-model").get("status") or {})
                           .get("state") == "Ready", timeout=120):
            raise RuntimeError(f"base model not Ready: {cl.store.get(API, 'ClusterBaseModel', 'slice-model')}")
        timings["model_ready_s"] = round(time.time() - t0, 1)
        log(f"[slice] ClusterBaseModel Ready after {timings['model_ready_s']} s")
        cl.apply([isvc("slice", "slice-model")])

        def _pods_logs():
            return {p["metadata"]["name"]: cl.executor.kubelet.logs("default", p["metadata"]["name"])[-4000:]
                    for p in cl.store.list("v1", "Pod", "default")}

        t_wait = time.time()
        ok = False
        while time.time() - t_wait < startup_timeout:
            if ready(cl.store.get(API, "InferenceService", "slice", "default")):
                ok = True
                break
            time.sleep(5)
            log(f"[slice] waiting for the InferenceService ({time.time() - t_wait:.0f} s)")
        if not ok:
            raise RuntimeError(f"ISVC not Ready: {cl.store.get(API, 'InferenceService', 'slice', 'default').get('status')}"
                               f"\n{_pods_logs()}")
        timings["isvc_ready_s"] = round(time.time() - t0, 1)
        log(f"[slice] InferenceService Ready after {timings['isvc_ready_s']} s")
        pod = next(p for p in cl.store.list("v1", "Pod", "default") if p["metadata"]["name"].startswith("slice-engine"))
        gpu_ids = (pod["metadata"].get("annotations") or {}).get("ome.io/gpu-ids", "")
        out = work / "bench"
        cl.apply([benchmark_job("bj", "slice", scenarios, concurrency, max_time, max_requests, out)])
        t_b = time.time()
        state = None
        while time.time() - t_b < bench_timeout:
            state = (cl.store.get(API, "BenchmarkJob", "bj", "default").get("status") or {}).get("state")
            if state in ("Completed", "Failed"):
                break
            time.sleep(5)
            log(f"[slice] BenchmarkJob {state} ({time.time() - t_b:.0f} s)")
        if state != "Completed":
            raise RuntimeError(f"BenchmarkJob {state}: {cl.store.get(API, 'BenchmarkJob', 'bj', 'default').get('status')}"
                               f"\n{cl.executor.kubelet.logs('default', 'bj-0')[-4000:]}")
        timings["bench_s"] = round(time.time() - t_b, 1)
        summary = json.loads((out / "exp" / "summary.json").read_text())
        return {"isvc": cl.store.get(API, "InferenceService", "slice", "default"), "summary": summary,
                "timings": timings, "gpu_ids": gpu_ids, "pod_env_visible": os.environ.get("HIP_VISIBLE_DEVICES")}
    finally:
        cl.shutdown()

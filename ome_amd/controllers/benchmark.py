"""BenchmarkJob controller (``pkg/controller/v1beta1/benchmark/controller.go``).

finalizer -> status from the owned ``batch/v1`` Job (Pending / Running / Completed / Failed) ->
if the endpoint is an InferenceService wait (requeue 60 s) until it is Ready -> build the load
generator command (our genai-bench-compatible ``ome_amd.bench.loadgen benchmark ...``: api
backend/base/model name/tokenizer, ``--task``, ``--traffic-scenario`` x N, ``--num-concurrency``
x N, max time / requests per run, server metadata, storage args) -> pin the pod to a node that
has the model (``models.ome.io/...=Ready``) -> strategic-merge ``podOverride`` -> Job.

Fix vs the reference: the API model name is the runtime's
``--served-model-name`` (or the base-model name), not the hardcoded ``vllm-model``.
"""
from __future__ import annotations

import copy

from ome_amd.api import constants as C
from ome_amd.controllers.config import ControllerConfig
from ome_amd.controllers.isvc import merging as M
from ome_amd.controllers.isvc import status as S
from ome_amd.controllers.isvc import workloads as W
from ome_amd.controllers.runtime import Controller, Result
from ome_amd.storage import uri as U
from ome_amd.store.store import Store, now_iso

API = C.API_VERSION
REQUEUE_NOT_READY = 60.0


def storage_args(spec: dict | None) -> list[str]:
    if not spec or not spec.get("storageUri"):
        raise ValueError("outputLocation.storageUri cannot be nil")
    u = U.parse(spec["storageUri"])
    params = spec.get("parameters") or {}
    p = u.parts
    if u.type == "OCI":
        args = ["--storage-provider", "oci", "--storage-bucket", p["bucket"], "--namespace", p["namespace"]]
        if p["prefix"]:
            args += ["--storage-prefix", p["prefix"]]
        for k, f in (("auth", "--storage-auth-type"), ("config_file", "--storage-auth-config-file"),
                     ("profile", "--storage-auth-profile"), ("region", "--storage-region")):
            if k in params:
                args += [f, params[k]]
        return args
    if u.type in ("PVC", "LOCAL"):
        return ["--experiment-base-dir", "/benchmark-results" if u.type == "PVC" else p["path"]]
    if u.type == "S3":
        args = ["--storage-provider", "aws", "--storage-bucket", p["bucket"]]
        if p["prefix"]:
            args += ["--storage-prefix", p["prefix"]]
        if p["region"] or params.get("region"):
            args += ["--storage-region", p["region"] or params["region"]]
        return args
    if u.type == "AZURE":
        return ["--storage-provider", "azure", "--storage-bucket", p["container"], "--storage-account",
                p["account"]] + (["--storage-prefix", p["blob_path"]] if p["blob_path"] else [])
    if u.type == "GCS":
        return ["--storage-provider", "gcp", "--storage-bucket", p["bucket"]] + (
            ["--storage-prefix", p["object"]] if p["object"] else [])
    if u.type == "GITHUB":
        return ["--storage-provider", "github", "--github-owner", p["owner"], "--github-repo", p["repository"]]
    raise ValueError(f"unsupported storage type: {u.type}")


def served_model_name(store: Store, isvc: dict, base_model: dict) -> str:
    """Best effort: ``--served-model-name`` from the ISVC/runtime engine args, else the model name."""
    eng = ((isvc.get("spec") or {}).get("engine") or {})
    args = list((eng.get("runner") or {}).get("args") or [])
    rt = (isvc.get("metadata", {}).get("annotations") or {}).get(C.SERVING_RUNTIME_ANN)
    dep = store.try_get("apps/v1", "Deployment", C.engine_name(isvc["metadata"]["name"]), isvc["metadata"]["namespace"])
    if dep:
        for c in dep["spec"]["template"]["spec"].get("containers") or []:
            args += list(c.get("args") or []) + list(c.get("command") or [])
    flat = " ".join(args).replace("\\\n", " ").split()
    for i, a in enumerate(flat):
        if a == "--served-model-name" and i + 1 < len(flat):
            return flat[i + 1]
        if a.startswith("--served-model-name="):
            return a.split("=", 1)[1]
    del rt
    return base_model["metadata"]["name"]


class BenchmarkJobReconciler:
    def __init__(self, store: Store):
        self.store = store

    def _get_model(self, name: str, ns: str) -> dict | None:
        return self.store.try_get(API, "BaseModel", name, ns) or self.store.try_get(API, "ClusterBaseModel", name)

    def endpoint_args(self, bj: dict) -> tuple[dict, dict | None, dict | None]:
        ep = (bj.get("spec") or {}).get("endpoint") or {}
        if ep.get("endpoint"):
            e = ep["endpoint"]
            return ({"--api-backend": e.get("apiFormat", "openai"), "--api-model-name": e.get("modelName", ""),
                     "--api-base": e["url"]}, None, None)
        ref = ep.get("inferenceService")
        if not ref:
            raise ValueError("invalid EndpointSpec: both Endpoint and InferenceService are nil")
        isvc = self.store.try_get(API, "InferenceService", ref["name"], ref.get("namespace") or
                                  bj["metadata"]["namespace"])
        if isvc is None:
            raise LookupError(f"InferenceService {ref.get('namespace')}/{ref['name']} not found")
        mname = ((isvc.get("spec") or {}).get("model") or {}).get("name") or \
            (((isvc.get("spec") or {}).get("predictor") or {}).get("model") or {}).get("baseModel")
        if not mname:
            raise ValueError("InferenceService has no Model defined")
        bm = self._get_model(mname, isvc["metadata"]["namespace"])
        if bm is None:
            raise LookupError(f"failed to get BaseModel {mname}")
        path = ((bm.get("spec") or {}).get("storage") or {}).get("path")
        if not path:
            raise ValueError(f"BaseModel {mname} has missing Storage or Path information")
        url = (isvc.get("status") or {}).get("url")
        if not url:
            raise ValueError("InferenceService has no URL in status")
        backend = "openai"
        for e in (((isvc.get("spec") or {}).get("engine") or {}).get("runner") or {}).get("env") or []:
            if e.get("name") == "PROTOCOL_VERSION" and e.get("value"):
                backend = e["value"]
        return ({"--api-backend": backend, "--api-base": url.rstrip("/"), "--api-key": "sample-key",
                 "--api-model-name": served_model_name(self.store, isvc, bm), "--model-tokenizer": path}, isvc, bm)

    def build_command(self, bj: dict) -> tuple[list[str], list[str], dict | None, dict | None]:
        sp = bj.get("spec") or {}
        a, isvc, bm = self.endpoint_args(bj)
        args = ["benchmark", "--api-backend", a["--api-backend"], "--api-base", a["--api-base"],
                "--api-model-name", a["--api-model-name"], "--task", sp["task"],
                "--max-time-per-run", str(sp.get("maxTimePerIteration")),
                "--max-requests-per-run", str(sp.get("maxRequestsPerIteration"))]
        if a.get("--api-key"):
            args += ["--api-key", a["--api-key"]]
        if a.get("--model-tokenizer"):
            args += ["--model-tokenizer", a["--model-tokenizer"]]
        for s in sp.get("trafficScenarios") or []:
            args += ["--traffic-scenario", s]
        for c in sp.get("numConcurrency") or []:
            args += ["--num-concurrency", str(c)]
        for k, v in (sp.get("additionalRequestParams") or {}).items():
            args += ["--additional-request-params", f"{k}={v}"]
        if sp.get("resultFolderName"):
            args += ["--experiment-folder-name", sp["resultFolderName"]]
        md = sp.get("serviceMetadata")
        if md:
            args += ["--server-engine", md["engine"], "--server-gpu-type", md["gpuType"], "--server-version",
                     md["version"], "--server-gpu-count", str(md["gpuCount"])]
        args += storage_args(sp.get("outputLocation"))
        return ["python", "-m", "ome_amd.bench.loadgen"], args, isvc, bm

    def pod_spec(self, bj: dict, cfg: ControllerConfig) -> dict:
        cmd, args, isvc, bm = self.build_command(bj)
        pc = cfg.benchmark.podConfig
        c = {"name": "benchmark", "image": pc.get("image"), "command": cmd, "args": args,
             "env": [{"name": "ENABLE_UI", "value": "false"}],
             "resources": {"requests": {"cpu": pc.get("cpuRequest"), "memory": pc.get("memoryRequest")},
                           "limits": {"cpu": pc.get("cpuLimit"), "memory": pc.get("memoryLimit")}}}
        sp = bj.get("spec") or {}
        if sp.get("huggingFaceSecretReference"):
            c["env"].append({"name": "HUGGINGFACE_API_KEY", "valueFrom": {"secretKeyRef": {
                "name": sp["huggingFaceSecretReference"]["name"], "key": "HUGGINGFACE_API_KEY"}}})
        ps = {"containers": [c], "restartPolicy": "Never"}
        if bm is not None:
            path = bm["spec"]["storage"]["path"]
            M.add_volume_mount(c, {"name": bm["metadata"]["name"], "mountPath": path, "readOnly": True})
            M.set_env(c, "MODEL_PATH", path, overwrite=False)
            M.add_volume(ps, {"name": bm["metadata"]["name"], "hostPath": {"path": path}})
            cluster = bm["kind"] == "ClusterBaseModel"
            ps["nodeSelector"] = {C.model_label(bm["metadata"].get("namespace"), bm["metadata"]["name"], cluster):
                                  "Ready"}
        out = sp.get("outputLocation") or {}
        if (out.get("storageUri") or "").startswith("pvc://"):
            pv = U.parse(out["storageUri"]).parts
            M.add_volume_mount(c, {"name": "benchmark-output-storage", "mountPath": "/benchmark-results",
                                   "subPath": pv["subpath"]})
            M.add_volume(ps, {"name": "benchmark-output-storage",
                              "persistentVolumeClaim": {"claimName": pv["pvc"]}})
        ov = sp.get("podOverride")
        if ov:
            for f in ("image", "env", "envFrom", "volumeMounts", "resources"):
                if ov.get(f) is not None:
                    c[f] = M.strategic_merge(c.get(f), ov[f], f)
            for f in ("tolerations", "nodeSelector", "affinity", "volumes"):
                if ov.get(f) is not None:
                    ps[f] = M.strategic_merge(ps.get(f), ov[f], f)
        return ps

    def _sync_status(self, bj: dict) -> dict:
        m = bj["metadata"]
        job = self.store.try_get("batch/v1", "Job", m["name"], m["namespace"])
        st = dict(bj.get("status") or {})
        if job is None:
            if st.get("state") != "Pending":
                st = {"state": "Pending", "lastReconcileTime": now_iso()}
        else:
            js = job.get("status") or {}
            state, ct, msg = "Running", None, ""
            for cnd in js.get("conditions") or []:
                if cnd.get("type") == "Failed" and cnd.get("status") == "True":
                    state, ct, msg = "Failed", cnd.get("lastTransitionTime"), cnd.get("message", "")
            if state != "Failed":
                if js.get("completionTime"):
                    state, ct = "Completed", js["completionTime"]
                for cnd in js.get("conditions") or []:
                    if cnd.get("type") == "Complete" and cnd.get("status") == "True":
                        state, ct = "Completed", cnd.get("lastTransitionTime")
            if st.get("state") != state:
                st.update({"state": state, "lastReconcileTime": now_iso()})
                if not st.get("startTime") and js.get("startTime"):
                    st["startTime"] = js["startTime"]
                if state in ("Failed", "Completed"):
                    st["completionTime"], st["failureMessage"] = ct, msg
                    if js.get("details"):
                        st["details"] = js["details"]
                else:
                    st.pop("completionTime", None)
                    st["failureMessage"] = ""
        if st != (bj.get("status") or {}):
            bj["status"] = st
            bj = self.store.update_status(bj)
        return bj

    def reconcile(self, key) -> Result:
        ns, name = key
        bj = self.store.try_get(API, "BenchmarkJob", name, ns)
        if bj is None:
            return Result()
        if bj["metadata"].get("deletionTimestamp"):
            self.store.remove_finalizer(bj, C.BENCHMARKJOB_FINALIZER)
            return Result()
        if C.BENCHMARKJOB_FINALIZER not in (bj["metadata"].get("finalizers") or []):
            bj = self.store.add_finalizer(bj, C.BENCHMARKJOB_FINALIZER)
        bj = self._sync_status(bj)
        ref = ((bj.get("spec") or {}).get("endpoint") or {}).get("inferenceService")
        if ref:
            isvc = self.store.try_get(API, "InferenceService", ref["name"], ref.get("namespace") or ns)
            if isvc is None or not S.is_ready(isvc):
                return Result(requeue_after=REQUEUE_NOT_READY)
        if self.store.try_get("batch/v1", "Job", name, ns) is None:
            cfg = ControllerConfig.from_store(self.store)
            ps = self.pod_spec(bj, cfg)
            labels = {"app": "benchmark", "benchmark.ome.io/name": name}
            job = {"apiVersion": "batch/v1", "kind": "Job",
                   "metadata": {"name": name, "namespace": ns, "labels": labels},
                   "spec": {"backoffLimit": 0, "template": {"metadata": {"labels": copy.deepcopy(labels)},
                                                            "spec": ps}}}
            W.ensure(self.store, job, bj)
            self._sync_status(self.store.get(API, "BenchmarkJob", name, ns))
        return Result()


def setup(store: Store) -> Controller:
    r = BenchmarkJobReconciler(store)

    def isvc_to_jobs(isvc):
        out = []
        for bj in store.list(API, "BenchmarkJob", isvc["metadata"]["namespace"]):
            ref = ((bj.get("spec") or {}).get("endpoint") or {}).get("inferenceService") or {}
            if ref.get("name") == isvc["metadata"]["name"]:
                out.append(Controller.key_of(bj))
        return out

    c = Controller("benchmarkjob", store, r.reconcile, (API, "BenchmarkJob"), owns=[("batch/v1", "Job")],
                   watches=[("InferenceService", isvc_to_jobs)])
    c.reconciler = r
    return c

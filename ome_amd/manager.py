"""ome-manager: one process hosting the object store, admission webhooks, every controller,
the local node executor and the model agent, plus a Kubernetes-style REST API
(``cmd/manager/main.go`` + the parts of kube-apiserver / kubelet the reference relies on).

    python -m ome_amd.manager --catalog config/ --state-dir /var/lib/ome --port 9443

The REST API mirrors Kubernetes paths so ``omectl`` (``python -m ome_amd.cli``) and external
tooling can drive it:

    /api/v1/[namespaces/{ns}/]{plural}[/{name}[/status|/log]]
    /apis/{group}/{version}/[namespaces/{ns}/]{plural}[/{name}[/status]]
    POST /apply  (multi-document YAML, server-side apply)
"""
from __future__ import annotations

import argparse
import glob
import json
import logging
import os
import threading
import time

import yaml
from fastapi import Request  # module level: FastAPI resolves the string annotations against it

from ome_amd.admission import webhooks
from ome_amd.api import constants as C
from ome_amd.controllers import acceleratorclass, basemodel, benchmark
from ome_amd.controllers.isvc import controller as isvc_controller
from ome_amd.controllers.runtime import Manager
from ome_amd.store.store import CLUSTER_SCOPED, AlreadyExists, Store, group_of

log = logging.getLogger("ome_amd.manager")

PLURALS = {
    "InferenceService": "inferenceservices", "BaseModel": "basemodels", "ClusterBaseModel": "clusterbasemodels",
    "ServingRuntime": "servingruntimes", "ClusterServingRuntime": "clusterservingruntimes",
    "AcceleratorClass": "acceleratorclasses", "BenchmarkJob": "benchmarkjobs", "FineTunedWeight": "finetunedweights",
    "Pod": "pods", "Service": "services", "ConfigMap": "configmaps", "Secret": "secrets", "Node": "nodes",
    "Namespace": "namespaces", "Event": "events", "ServiceAccount": "serviceaccounts",
    "PersistentVolume": "persistentvolumes", "PersistentVolumeClaim": "persistentvolumeclaims",
    "Deployment": "deployments", "Job": "jobs", "LeaderWorkerSet": "leaderworkersets", "Ingress": "ingresses",
    "HorizontalPodAutoscaler": "horizontalpodautoscalers", "ScaledObject": "scaledobjects",
    "PodDisruptionBudget": "poddisruptionbudgets", "RayCluster": "rayclusters", "HTTPRoute": "httproutes",
    "Role": "roles", "RoleBinding": "rolebindings", "ClusterRole": "clusterroles",
    "ClusterRoleBinding": "clusterrolebindings", "VirtualService": "virtualservices",
}
KIND_OF_PLURAL = {v: k for k, v in PLURALS.items()}
KIND_OF_PLURAL["services"] = "Service"  # core v1 wins over knative for the bare plural

# Only the keys we override; everything else uses the controller defaults
# (``ome_amd.controllers.config``, mirroring ``config/configmap/inferenceservice.yaml``).
DEFAULT_ISVC_CONFIG = {"deploy": {"defaultDeploymentMode": "RawDeployment"}}
DEFAULT_BENCH_CONFIG = {"podConfig": {"image": "ome-amd/genai-bench:latest", "cpuRequest": "2", "memoryRequest": "2Gi",
                                      "cpuLimit": "2", "memoryLimit": "2Gi"}}


def load_yaml_docs(text: str) -> list[dict]:
    return [d for d in yaml.safe_load_all(text) if isinstance(d, dict) and d.get("kind")]


class Cluster:
    """Everything the reference needs a Kubernetes cluster + ome-manager + model-agent for."""

    def __init__(self, state_dir: str = "/tmp/ome-state", node_name: str = "mi355x-node-0", gpus: int | None = None,
                 simulate: bool = False, models_root: str | None = None, with_agent: bool = True,
                 with_executor: bool = True, probe_scale: float = 1.0, agent_kw: dict | None = None,
                 store: Store | None = None):
        # a KubeStore (ome_amd.store.kube) runs the same controllers against a real API server;
        # its writes skip the local hooks (the API server calls ours at /admission instead),
        # which read the cluster state from the KubeStore's cache
        self.store = store if store is not None else Store()
        webhooks.install(self.store)
        self.manager = Manager(self.store)
        self.state_dir = os.path.abspath(state_dir)
        os.makedirs(self.state_dir, exist_ok=True)
        for ns in ("default", C.OME_NAMESPACE):
            self._ensure({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
        self._ensure({"apiVersion": "v1", "kind": "ConfigMap",
                      "metadata": {"name": C.INFERENCESERVICE_CONFIGMAP, "namespace": C.OME_NAMESPACE},
                      "data": {k: json.dumps(v) for k, v in DEFAULT_ISVC_CONFIG.items()}})
        self._ensure({"apiVersion": "v1", "kind": "ConfigMap",
                      "metadata": {"name": C.BENCHMARKJOB_CONFIGMAP, "namespace": C.OME_NAMESPACE},
                      "data": {"benchmarkjob": json.dumps(DEFAULT_BENCH_CONFIG)}})
        self.manager.add(isvc_controller.setup(self.store))
        self.manager.add(basemodel.setup(self.store, cluster=False))
        self.manager.add(basemodel.setup(self.store, cluster=True))
        self.manager.add(acceleratorclass.setup(self.store))
        self.manager.add(benchmark.setup(self.store))
        self.executor = None
        if with_executor:
            from ome_amd.executor import NodeExecutor

            self.executor = NodeExecutor(self.store, self.manager, node_name=node_name, gpus=gpus,
                                         state_dir=os.path.join(self.state_dir, "executor"), simulate=simulate,
                                         probe_scale=probe_scale)
        self.agent = None
        if with_agent:
            from ome_amd.modelagent import ModelAgent

            self.agent = ModelAgent(self.store, node_name, models_root or os.path.join(self.state_dir, "models"),
                                    **(agent_kw or {}))
        self._started = False

    def _ensure(self, obj: dict) -> None:
        try:
            self.store.create(obj)
        except AlreadyExists:
            pass

    # ------------------------------------------------------------------ objects
    def apply(self, docs: list[dict] | str) -> list[dict]:
        if isinstance(docs, str):
            docs = load_yaml_docs(docs)
        return [self.store.apply(d) for d in docs]

    def load_catalog(self, path: str) -> int:
        n = 0
        files = [path] if os.path.isfile(path) else sorted(glob.glob(os.path.join(path, "**", "*.yaml"), recursive=True))
        for f in files:
            with open(f) as fh:
                for d in load_yaml_docs(fh.read()):
                    self.store.apply(d)
                    n += 1
        return n

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        if self.agent:
            self.agent.start()
        if self.executor:
            self.executor.start()
        self.manager.start()
        self._started = True

    def step(self, rounds: int = 4) -> None:
        """Deterministic drive for tests (no threads)."""
        for _ in range(rounds):
            self.manager.run_until_idle(fast_forward=6.0)
            if self.agent:
                self.agent.drain(30)
            if self.executor:
                self.executor.kubelet.sync()
        self.manager.run_until_idle(fast_forward=6.0)

    def serve_api(self, host: str = "127.0.0.1", port: int = 0) -> str:
        """Run the REST API in a background thread; pods get it as ``$OME_API_SERVER``."""
        import socket

        import uvicorn

        if port == 0:
            with socket.socket() as s:
                s.bind((host, 0))
                port = s.getsockname()[1]
        server = uvicorn.Server(uvicorn.Config(create_api(self), host=host, port=port, log_level="warning"))
        t = threading.Thread(target=server.run, name="ome-api", daemon=True)
        t.start()
        for _ in range(100):
            if server.started:
                break
            time.sleep(0.05)
        self._api_server = server
        self.api_url = f"http://{host}:{port}"
        if self.executor:
            self.executor.kubelet.api_url = self.api_url
        return self.api_url

    def wait_for(self, pred, timeout: float = 60.0, interval: float = 0.2, drive: bool = False) -> bool:
        end = time.time() + timeout
        while time.time() < end:
            if drive:
                self.step(1)
            if pred():
                return True
            time.sleep(interval)
        return False

    def shutdown(self) -> None:
        if getattr(self, "_api_server", None) is not None:
            self._api_server.should_exit = True
        if self._started:
            self.manager.stop()
        if self.agent:
            self.agent.stop()
        if self.executor:
            self.executor.shutdown()


# ------------------------------------------------------------------ REST API
def create_api(cluster: Cluster):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import JSONResponse, PlainTextResponse

    from ome_amd.store import store as S

    app = FastAPI(title="ome-amd manager")
    st = cluster.store

    @app.post("/admission")
    async def admission(review: dict):
        """admission.k8s.io/v1 AdmissionReview (mutating + validating) for a real API server."""
        from ome_amd.store.kube import admission_review

        return admission_review(st, review)

    def err(e: Exception):
        code = {S.NotFound: 404, S.AlreadyExists: 409, S.Conflict: 409, S.Invalid: 422}.get(type(e), 400)
        return JSONResponse({"kind": "Status", "status": "Failure", "message": str(e), "code": code}, status_code=code)

    def api_version(group: str, version: str) -> str:
        return f"{group}/{version}" if group else version

    def resolve(group: str, plural: str) -> str:
        kind = KIND_OF_PLURAL.get(plural)
        if kind is None:
            raise HTTPException(404, f"unknown resource {plural}")
        if plural == "services" and group == "serving.knative.dev":
            kind = "Service"
        return kind

    async def handle(request: Request, group: str, version: str, ns: str | None, plural: str, name: str | None,
                     sub: str | None):
        kind = resolve(group, plural)
        av = api_version(group, version)
        try:
            if request.method == "GET" and name is None:
                sel = request.query_params.get("labelSelector")
                items = st.list(av, kind, ns, selector=sel)
                return {"apiVersion": av, "kind": f"{kind}List", "items": items}
            if request.method == "GET" and sub == "log":
                if not cluster.executor:
                    raise HTTPException(404, "no executor")
                return PlainTextResponse(cluster.executor.kubelet.logs(ns, name, request.query_params.get("container")))
            if request.method == "GET":
                return st.get(av, kind, name, ns)
            body = await request.json() if request.method in ("POST", "PUT", "PATCH") else None
            if body is not None:
                body.setdefault("apiVersion", av)
                body.setdefault("kind", kind)
                if ns and (group, kind) not in CLUSTER_SCOPED:
                    body.setdefault("metadata", {}).setdefault("namespace", ns)
            if request.method == "POST":
                return st.create(body, dry_run=request.query_params.get("dryRun") == "All")
            if request.method == "PUT":
                return st.update_status(body) if sub == "status" else st.update(body)
            if request.method == "PATCH":
                return st.patch(av, kind, name, body, ns)
            if request.method == "DELETE":
                st.delete(av, kind, name, ns)
                return {"kind": "Status", "status": "Success"}
        except HTTPException:
            raise
        except Exception as e:  # noqa: BLE001
            return err(e)
        raise HTTPException(405)

    methods = ["GET", "POST", "PUT", "PATCH", "DELETE"]

    @app.api_route("/api/{version}/namespaces/{ns}/{plural}", methods=methods)
    async def core_ns_list(request: Request, version: str, ns: str, plural: str):
        return await handle(request, "", version, ns, plural, None, None)

    @app.api_route("/api/{version}/namespaces/{ns}/{plural}/{name}", methods=methods)
    async def core_ns_obj(request: Request, version: str, ns: str, plural: str, name: str):
        return await handle(request, "", version, ns, plural, name, None)

    @app.api_route("/api/{version}/namespaces/{ns}/{plural}/{name}/{sub}", methods=methods)
    async def core_ns_sub(request: Request, version: str, ns: str, plural: str, name: str, sub: str):
        return await handle(request, "", version, ns, plural, name, sub)

    @app.api_route("/api/{version}/{plural}", methods=methods)
    async def core_list(request: Request, version: str, plural: str):
        return await handle(request, "", version, None, plural, None, None)

    @app.api_route("/api/{version}/{plural}/{name}", methods=methods)
    async def core_obj(request: Request, version: str, plural: str, name: str):
        return await handle(request, "", version, None, plural, name, None)

    @app.api_route("/apis/{group}/{version}/namespaces/{ns}/{plural}", methods=methods)
    async def g_ns_list(request: Request, group: str, version: str, ns: str, plural: str):
        return await handle(request, group, version, ns, plural, None, None)

    @app.api_route("/apis/{group}/{version}/namespaces/{ns}/{plural}/{name}", methods=methods)
    async def g_ns_obj(request: Request, group: str, version: str, ns: str, plural: str, name: str):
        return await handle(request, group, version, ns, plural, name, None)

    @app.api_route("/apis/{group}/{version}/namespaces/{ns}/{plural}/{name}/{sub}", methods=methods)
    async def g_ns_sub(request: Request, group: str, version: str, ns: str, plural: str, name: str, sub: str):
        return await handle(request, group, version, ns, plural, name, sub)

    @app.api_route("/apis/{group}/{version}/{plural}", methods=methods)
    async def g_list(request: Request, group: str, version: str, plural: str):
        return await handle(request, group, version, None, plural, None, None)

    @app.api_route("/apis/{group}/{version}/{plural}/{name}", methods=methods)
    async def g_obj(request: Request, group: str, version: str, plural: str, name: str):
        return await handle(request, group, version, None, plural, name, None)

    @app.api_route("/apis/{group}/{version}/{plural}/{name}/{sub}", methods=methods)
    async def g_sub(request: Request, group: str, version: str, plural: str, name: str, sub: str):
        return await handle(request, group, version, None, plural, name, sub)

    # web console (H8): dashboard at /console/, its REST API at /console/api/v1
    from ome_amd.console import mount as mount_console

    mount_console(app, st, models_root=getattr(cluster.agent, "models_root", None))

    @app.post("/apply")
    async def apply(request: Request):
        try:
            return {"items": cluster.apply((await request.body()).decode())}
        except Exception as e:  # noqa: BLE001
            return err(e)

    @app.get("/openapi/v2")
    def openapi_v2():
        """Swagger 2.0 of the ome.io/v1beta1 API (the SDK's source document)."""
        from ome_amd.api.openapi import swagger

        return swagger()

    @app.get("/healthz")
    def healthz():
        return {"status": "ok"}

    @app.get("/readyz")
    def readyz():
        ok, msg = cluster.agent.healthz() if cluster.agent else (True, "ok")
        return JSONResponse({"status": "ok" if ok else msg}, status_code=200 if ok else 503)

    @app.get("/metrics")
    def metrics():
        from ome_amd.modelagent import metrics as MM

        lines = []
        for c in cluster.manager.controllers:
            lines.append(f'controller_runtime_reconcile_total{{controller="{c.name}"}} {c.reconciles}')
            lines.append(f'controller_runtime_reconcile_errors_total{{controller="{c.name}"}} {c.errors}')
            lines.append(f'workqueue_depth{{name="{c.name}"}} {len(c.queue)}')
        return PlainTextResponse("\n".join(lines) + "\n" + MM.render().decode())

    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="ome-amd manager (store + controllers + executor + model agent)")
    ap.add_argument("--catalog", action="append", default=[], help="YAML file/dir to apply at start (repeatable)")
    ap.add_argument("--state-dir", default=os.environ.get("OME_STATE_DIR", "/tmp/ome-state"))
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", "mi355x-node-0"))
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--models-root-dir", default=None)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9443)
    ap.add_argument("--simulate", action="store_true", help="do not launch pod processes (control-plane only)")
    ap.add_argument("--no-agent", action="store_true")
    ap.add_argument("--kubeconfig", default=None, help="reconcile a real cluster through this kubeconfig")
    ap.add_argument("--in-cluster", action="store_true", help="reconcile the cluster we run in (service account)")
    ap.add_argument("--tls-cert-dir", default=None,
                    help="serve HTTPS with tls.crt / tls.key from this dir (the API server calls /admission over TLS)")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    store = None
    if args.kubeconfig or args.in_cluster:
        from ome_amd.store import kube

        client = kube.KubeClient.in_cluster() if args.in_cluster else kube.KubeClient.from_kubeconfig(args.kubeconfig)
        store = kube.KubeStore(client, kube.MANAGER_KINDS)
    cl = Cluster(args.state_dir, args.node_name, args.gpus, simulate=args.simulate, models_root=args.models_root_dir,
                 with_agent=not args.no_agent and store is None, with_executor=store is None, store=store)
    for c in args.catalog:
        log.info("applied %d objects from %s", cl.load_catalog(c), c)
    cl.start()
    import uvicorn

    try:
        tls = {}
        if args.tls_cert_dir:
            tls = {"ssl_certfile": os.path.join(args.tls_cert_dir, "tls.crt"),
                   "ssl_keyfile": os.path.join(args.tls_cert_dir, "tls.key")}
        uvicorn.run(create_api(cl), host=args.host, port=args.port, log_level="warning", **tls)
    finally:
        cl.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

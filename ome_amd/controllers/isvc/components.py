"""Engine / Decoder / Router component builders (``pkg/controller/v1beta1/inferenceservice/components``).

Each component turns a merged component spec into object metadata + pod spec(s) and
reconciles the workload for its deployment mode.  Model plumbing follows the reference:
``MODEL_PATH`` env + read-only hostPath mount of ``storage.path``; node selector on the
node label ``models.ome.io/<...>=Ready`` that the model agent sets; runtime < AcceleratorClass
resource merge when the ISVC runner sets none; per-accelerator ``runtimeArgsOverride`` /
``environmentOverride`` / ``tensorParallelismOverride`` (TP/PP rewrite);
``PARALLELISM_SIZE = gpusPerPod * (1 + workers)``.  GPU resources default to ``amd.com/gpu``.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

from ome_amd.api import constants as C
from ome_amd.api import v1beta1 as V
from ome_amd.controllers.config import ControllerConfig
from ome_amd.controllers.isvc import merging as M
from ome_amd.controllers.isvc import workloads as W
from ome_amd.store.store import Store

POD_FIELDS = ("containers", "volumes", "nodeSelector", "affinity", "tolerations", "serviceAccountName", "hostIPC",
              "hostNetwork", "schedulerName", "imagePullSecrets", "dnsPolicy", "initContainers", "securityContext",
              "priorityClassName", "runtimeClassName", "hostPID", "shareProcessNamespace", "subdomain", "hostname",
              "terminationGracePeriodSeconds", "restartPolicy", "topologySpreadConstraints", "readinessGates")
EXT_FIELDS = ("minReplicas", "maxReplicas", "scaleTarget", "scaleMetric", "containerConcurrency", "timeoutSeconds",
              "canaryTrafficPercent", "minAvailable", "maxUnavailable", "deploymentStrategy", "kedaConfig")
DISALLOWED_ANNOTATIONS = ("kubectl.kubernetes.io/last-applied-configuration",)


def pod_part(spec: dict | None) -> dict:
    return {k: copy.deepcopy(v) for k, v in (spec or {}).items() if k in POD_FIELDS}


def ext_part(spec: dict | None) -> dict:
    return {k: copy.deepcopy(v) for k, v in (spec or {}).items() if k in EXT_FIELDS}


@dataclass
class ComponentContext:
    store: Store
    isvc: dict
    cfg: ControllerConfig
    mode: str
    base_model: dict | None            # (Cluster)BaseModel object
    runtime_name: str
    runtime_spec: dict                 # ServingRuntimeSpec (JSON form)
    supported_format: V.SupportedModelFormat | None = None
    ac_name: str = ""
    ac_spec: dict | None = None
    ft_weights: list[dict] = field(default_factory=list)

    @property
    def model_spec(self) -> dict:
        return (self.base_model or {}).get("spec") or {}

    @property
    def model_meta(self) -> dict:
        return (self.base_model or {}).get("metadata") or {}

    @property
    def is_cluster_model(self) -> bool:
        return (self.base_model or {}).get("kind") == "ClusterBaseModel"


class Component:
    kind = C.ENGINE

    def __init__(self, ctx: ComponentContext, spec: dict):
        self.ctx, self.spec = ctx, spec

    # ---------------------------------------------------------------- metadata
    def name(self) -> str:
        return C.component_name(self.ctx.isvc["metadata"]["name"], self.kind)

    def annotations(self) -> dict:
        ctx = self.ctx
        a = {k: v for k, v in (ctx.isvc["metadata"].get("annotations") or {}).items()
             if k not in DISALLOWED_ANNOTATIONS}
        a.update(self.spec.get("annotations") or {})
        if ctx.ft_weights:
            ft = ctx.ft_weights[0]
            a[C.FT_ADAPTER_INJECTION] = ft["metadata"]["name"]
            strategy = ((ft.get("spec") or {}).get("hyperParameters") or {}).get("strategy")
            if strategy:
                a[f"{C.GROUP}/fine-tuned-weight-ft-strategy"] = strategy
        mm = ctx.model_meta.get("annotations") or {}
        for k in (C.BASE_MODEL_DECRYPTION_KEY, C.BASE_MODEL_DECRYPTION_SECRET):
            if k in mm:
                a[k] = mm[k]
        if ctx.base_model is not None:
            a[C.BASE_MODEL_NAME_ANN] = ctx.model_meta["name"]
            if ctx.model_spec.get("vendor"):
                a[C.BASE_MODEL_VENDOR_ANN] = ctx.model_spec["vendor"]
            fmt = ctx.model_spec.get("modelFormat") or {}
            if fmt.get("name"):
                a[C.BASE_MODEL_FORMAT_ANN] = fmt["name"]
            if fmt.get("version"):
                a[C.BASE_MODEL_FORMAT_VERSION_ANN] = fmt["version"]
        if ctx.runtime_name:
            a[C.SERVING_RUNTIME_ANN] = ctx.runtime_name
        return a

    def labels(self) -> dict:
        ctx = self.ctx
        lab = dict(ctx.isvc["metadata"].get("labels") or {})
        lab.update(self.spec.get("labels") or {})
        lab.update({C.ISVC_LABEL: ctx.isvc["metadata"]["name"], C.COMPONENT_LABEL: self.kind,
                    C.SERVING_RUNTIME_LABEL: ctx.runtime_name, C.FT_SERVING_LABEL: str(bool(ctx.ft_weights)).lower()})
        if ctx.base_model is not None:
            lab[C.BASE_MODEL_NAME_LABEL] = ctx.model_meta["name"]
            lab[C.BASE_MODEL_SIZE_LABEL] = (ctx.model_meta.get("annotations") or {}).get(C.MODEL_CATEGORY, "SMALL")
            lab[C.BASE_MODEL_TYPE_LABEL] = "Serving"
            if ctx.model_spec.get("vendor"):
                lab[C.BASE_MODEL_VENDOR_LABEL] = ctx.model_spec["vendor"]
        return lab

    def meta(self) -> dict:
        return {"name": self.name(), "namespace": self.ctx.isvc["metadata"]["namespace"], "labels": self.labels(),
                "annotations": self.annotations()}

    # ---------------------------------------------------------------- pod spec
    def _accel_cfg(self) -> V.AcceleratorModelConfig | None:
        f = self.ctx.supported_format
        if f is None or not f.accelerator_config or not self.ctx.ac_name:
            return None
        return f.accelerator_config.get(self.ctx.ac_name)

    def _prepare_runner(self, runner: dict, worker_size: int, isvc_component: dict | None) -> None:
        ctx = self.ctx
        storage = ctx.model_spec.get("storage") or {}
        path = storage.get("path")
        if path and not ctx.ft_weights:
            M.set_env(runner, C.MODEL_PATH_ENV, path, overwrite=False)
        if path and ctx.base_model is not None:
            M.add_volume_mount(runner, {"name": ctx.model_meta["name"], "mountPath": path, "readOnly": True})
        if ctx.ft_weights:
            M.add_volume_mount(runner, {"name": "model-empty-dir", "mountPath": "/opt/ml/model"})
            M.set_env(runner, C.MODEL_PATH_ENV, "/opt/ml/model", overwrite=False)
            M.set_env(runner, C.SERVED_MODEL_NAME_ENV, f"/data/{ctx.ft_weights[0]['metadata']['name']}")
        acfg = self._accel_cfg()
        if acfg is not None:
            for k, v in (acfg.environment_override or {}).items():
                M.set_env(runner, k, v)
        # resources: only when the ISVC's own runner left them unspecified
        isvc_runner = (isvc_component or {}).get("runner") or {}
        if not isvc_runner.get("resources"):
            M.merge_resources(runner, ctx.ac_spec, ctx.runtime_spec)
        if acfg is not None:
            runner["args"] = M.merge_args(runner.get("args"), acfg.runtime_args_override)
            tpo = acfg.tensor_parallelism_override
            if tpo is not None:
                if tpo.tensor_parallel_size:
                    M.override_param(runner, M.TP_ALIASES, tpo.tensor_parallel_size)
                if tpo.pipeline_parallel_size:
                    M.override_param(runner, M.PP_ALIASES, tpo.pipeline_parallel_size)
                if tpo.data_parallel_size:  # applied here (the reference declares it but never applies it)
                    M.override_param(runner, M.DP_ALIASES, tpo.data_parallel_size)
        gpus = M.gpu_count(runner)
        if gpus > 0:
            M.set_env(runner, C.PARALLELISM_SIZE_ENV, str(gpus * (1 + worker_size)))

    def _pod_spec(self, base_pod: dict, runner: dict | None) -> dict:
        ps = copy.deepcopy(base_pod)
        ps.setdefault("containers", [])
        if runner is not None:
            runner = copy.deepcopy(runner)
            name = runner.get("name") or C.MAIN_CONTAINER
            runner["name"] = name
            idx = next((i for i, c in enumerate(ps["containers"]) if c.get("name") == name), None)
            if idx is None:
                ps["containers"].append({})
                idx = len(ps["containers"]) - 1
            merged = M.merge_runtime_container(ps["containers"][idx], runner)
            ps["containers"][idx] = M.replace_placeholders(merged, self.ctx.isvc["metadata"])
        elif ps["containers"]:
            ps["containers"][0] = M.replace_placeholders(ps["containers"][0], self.ctx.isvc["metadata"])
        else:
            raise ValueError(f"{self.kind}: no containers found in pod spec and no runner spec provided")
        return ps

    def _finish_pod(self, ps: dict) -> dict:
        ctx = self.ctx
        storage = ctx.model_spec.get("storage") or {}
        if storage.get("path") and ctx.base_model is not None:
            M.add_volume(ps, {"name": ctx.model_meta["name"], "hostPath": {"path": storage["path"]}})
        if ctx.ft_weights:
            M.add_volume(ps, {"name": "model-empty-dir", "emptyDir": {"medium": "Memory"}})
        if ctx.base_model is not None:
            ns = ps.setdefault("nodeSelector", {})
            ns[C.model_label(ctx.model_meta.get("namespace"), ctx.model_meta["name"], ctx.is_cluster_model)] = "Ready"
            for src in (ctx.runtime_spec.get("nodeSelector"), (ctx.ac_spec or {}).get("discovery", {}).get("nodeSelector"),
                        ((ctx.isvc.get("spec") or {}).get(self.kind) or {}).get("nodeSelector")):
                ns.update(src or {})
        isvc_comp = (ctx.isvc.get("spec") or {}).get(self.kind) or {}
        if not isvc_comp.get("affinity") and ctx.ac_spec and (ctx.ac_spec.get("discovery") or {}).get("affinity"):
            ps["affinity"] = copy.deepcopy(ctx.ac_spec["discovery"]["affinity"])
        return ps

    def worker_size(self) -> int:
        return int(((self.spec.get("worker") or {}).get("size")) or 0)

    def leader_pod_spec(self) -> dict:
        spec = self.spec
        isvc_comp = (self.ctx.isvc.get("spec") or {}).get(self.kind)
        if self.ctx.mode in (C.DeploymentMode.MULTINODE, C.DeploymentMode.MULTINODE_RAY_VLLM) and spec.get("leader"):
            base, runner = pod_part(spec["leader"]), copy.deepcopy(spec["leader"].get("runner"))
        else:
            base, runner = pod_part(spec), copy.deepcopy(spec.get("runner"))
        if runner is not None:
            self._prepare_runner(runner, self.worker_size(), isvc_comp)
        return self._finish_pod(self._pod_spec(base, runner))

    def worker_pod_spec(self) -> dict | None:
        w = self.spec.get("worker")
        if w is None:
            return None
        runner = copy.deepcopy(w.get("runner"))
        if runner is not None:
            self._prepare_runner(runner, self.worker_size(), (self.ctx.isvc.get("spec") or {}).get(self.kind))
        base = pod_part(w)
        if runner is None and not base.get("containers"):
            return None
        return self._finish_pod(self._pod_spec(base, runner))

    # ---------------------------------------------------------------- reconcile
    def reconcile(self) -> dict:
        """Create/update the workload; returns an info dict for status propagation."""
        ctx, meta = self.ctx, self.meta()
        ext = ext_part(self.spec)
        leader = self.leader_pod_spec()
        if ctx.mode == C.DeploymentMode.RAW:
            obj = W.reconcile_raw(ctx.store, ctx.isvc, meta, leader, ext, ctx.cfg)
            return {"mode": ctx.mode, "object": obj, "meta": meta}
        if ctx.mode == C.DeploymentMode.MULTINODE:
            obj = W.reconcile_multinode(ctx.store, ctx.isvc, meta, leader, self.worker_pod_spec(), self.worker_size(),
                                        ext)
            return {"mode": ctx.mode, "object": obj, "meta": meta}
        if ctx.mode == C.DeploymentMode.MULTINODE_RAY_VLLM:
            probers, requeue = W.reconcile_ray(ctx.store, ctx.isvc, meta, leader, ext, ctx.cfg)
            return {"mode": ctx.mode, "objects": probers, "meta": meta, "requeue_after": requeue}
        if ctx.mode == C.DeploymentMode.SERVERLESS:
            obj = W.ensure(ctx.store, W.build_ksvc(meta, leader, ext), ctx.isvc)
            return {"mode": ctx.mode, "object": obj, "meta": meta}
        raise ValueError(f"invalid deployment mode for {self.kind}: {ctx.mode}")


class Engine(Component):
    kind = C.ENGINE


class Decoder(Component):
    kind = C.DECODER

    def reconcile(self) -> dict:
        if self.ctx.mode == C.DeploymentMode.SERVERLESS:
            raise ValueError("decoder does not support serverless deployment")
        return super().reconcile()


class Router(Component):
    kind = C.ROUTER

    def annotations(self) -> dict:
        a = {k: v for k, v in (self.ctx.isvc["metadata"].get("annotations") or {}).items()
             if k not in DISALLOWED_ANNOTATIONS}
        a.update(self.spec.get("annotations") or {})
        if self.ctx.runtime_name:
            a[C.SERVING_RUNTIME_ANN] = self.ctx.runtime_name
        return a

    def leader_pod_spec(self) -> dict:
        spec = self.spec
        runner = copy.deepcopy(spec.get("runner"))
        if runner is not None:
            for k, v in (spec.get("config") or {}).items():
                M.set_env(runner, k, str(v))
            M.set_env(runner, "INFERENCESERVICE_NAME", self.ctx.isvc["metadata"]["name"], overwrite=False)
            M.set_env(runner, "NAMESPACE", self.ctx.isvc["metadata"]["namespace"], overwrite=False)
        ps = self._pod_spec(pod_part(spec), runner)
        sa = W.reconcile_router_rbac(self.ctx.store, self.ctx.isvc, self.meta())
        ps.setdefault("serviceAccountName", sa)
        return ps


def make_component(kind: str, ctx: ComponentContext, spec: dict) -> Component:
    return {C.ENGINE: Engine, C.DECODER: Decoder, C.ROUTER: Router}[kind](ctx, spec)

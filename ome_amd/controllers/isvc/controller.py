"""InferenceService controller: the central reconcile (``inferenceservice/controller.go:117-503``).

finalizer -> deployment mode (annotation / config default) -> VirtualDeployment shortcut ->
ModelConfig ConfigMap -> predictor->engine migration -> resolve (Cluster)BaseModel (reject
disabled) -> validate the user runtime or auto-select one (RuntimeSelector) -> merge runtime
component templates with the ISVC (strategic merge) -> per-component deployment modes ->
AcceleratorClass per engine/decoder (AcceleratorClassSelector) -> reconcile engine, decoder,
router workloads -> ingress + external Service + URL -> clean up removed components ->
status (component conditions, model status, Ready) + events.
"""
from __future__ import annotations

import copy
import logging

from ome_amd.api import constants as C
from ome_amd.api import v1beta1 as V
from ome_amd.controllers.config import ControllerConfig, resolve_ingress
from ome_amd.controllers.isvc import merging as M
from ome_amd.controllers.isvc import status as S
from ome_amd.controllers.isvc import workloads as W
from ome_amd.controllers.isvc.components import ComponentContext, make_component
from ome_amd.controllers.runtime import Controller, Result
from ome_amd.policy.accelerator_selector import AcceleratorClassSelector
from ome_amd.policy.runtime_selector import RuntimeSelector, SelectorError
from ome_amd.store.store import Conflict, NotFound, Store

log = logging.getLogger("ome_amd.isvc")
API = C.API_VERSION


# ------------------------------------------------------------------ deployment modes
def mode_from_annotations(ann: dict | None) -> str | None:
    m = (ann or {}).get(C.DEPLOYMENT_MODE)
    return m if m and C.DeploymentMode.is_valid(m) else None


def engine_mode(engine: dict | None) -> str:
    if engine is None:
        return C.DeploymentMode.RAW
    m = mode_from_annotations(engine.get("annotations"))
    if m:
        return m
    if engine.get("leader") is not None or engine.get("worker") is not None:
        return C.DeploymentMode.MULTINODE
    if engine.get("minReplicas") == 0:
        return C.DeploymentMode.SERVERLESS
    return C.DeploymentMode.RAW


def determine_modes(engine: dict | None, decoder: dict | None, router: dict | None) -> tuple[str, str, str]:
    e = engine_mode(engine)
    d = C.DeploymentMode.RAW
    r = C.DeploymentMode.RAW
    if decoder is not None:
        if e == C.DeploymentMode.SERVERLESS:
            e = C.DeploymentMode.RAW
        if decoder.get("leader") is not None or decoder.get("worker") is not None:
            d = C.DeploymentMode.MULTINODE
    if router is not None and router.get("minReplicas") == 0:
        r = C.DeploymentMode.SERVERLESS
    if engine is None:
        raise ValueError("engine component is required")
    return e, d, r


def migrate_predictor(isvc: dict) -> bool:
    """Deprecated ``spec.predictor`` -> ``spec.engine`` + ``spec.model`` + ``spec.runtime``."""
    sp = isvc.get("spec") or {}
    pred = sp.get("predictor")
    if not pred or sp.get("engine"):
        return False
    model = pred.get("model") or {}
    engine = {k: v for k, v in pred.items() if k not in ("model", "workerSpec")}
    if model:
        runner = {k: v for k, v in model.items() if k not in ("baseModel", "fineTunedWeights", "runtime",
                                                            "protocolVersion", "storageUri")}
        if runner:
            runner.setdefault("name", C.MAIN_CONTAINER)
            engine["runner"] = runner
    if pred.get("workerSpec"):
        w = copy.deepcopy(pred["workerSpec"])
        engine["worker"] = w
        engine.setdefault("leader", {})
    sp["engine"] = engine
    if model.get("baseModel") and not sp.get("model"):
        sp["model"] = {"name": model["baseModel"]}
        if model.get("fineTunedWeights"):
            sp["model"]["fineTunedWeights"] = model["fineTunedWeights"]
    if model.get("runtime") and not sp.get("runtime"):
        sp["runtime"] = {"name": model["runtime"]}
    sp.pop("predictor", None)
    isvc["spec"] = sp
    return True


class InferenceServiceReconciler:
    def __init__(self, store: Store):
        self.store = store
        self.runtime_selector = RuntimeSelector(store)
        self.ac_selector = AcceleratorClassSelector(store)

    def event(self, isvc, etype, reason, msg):
        try:
            self.store.record_event(isvc, etype, reason, msg)
        except Exception:  # noqa: BLE001
            pass

    def get_base_model(self, name: str, namespace: str) -> dict:
        o = self.store.try_get(API, "BaseModel", name, namespace)
        if o is None:
            o = self.store.try_get(API, "ClusterBaseModel", name)
        if o is None:
            raise LookupError(f"No BaseModel or ClusterBaseModel with the name: {name}")
        return o

    def reconcile(self, key) -> Result:
        ns, name = key
        isvc = self.store.try_get(API, "InferenceService", name, ns)
        if isvc is None:
            return Result()
        cfg = ControllerConfig.from_store(self.store)
        ann = isvc["metadata"].get("annotations") or {}
        mode = mode_from_annotations(ann) or cfg.deploy.defaultDeploymentMode
        # finalizer
        if isvc["metadata"].get("deletionTimestamp"):
            self.store.remove_finalizer(isvc, C.ISVC_FINALIZER)
            return Result()
        if C.ISVC_FINALIZER not in (isvc["metadata"].get("finalizers") or []):
            isvc = self.store.add_finalizer(isvc, C.ISVC_FINALIZER)
        status = copy.deepcopy(isvc.get("status") or {})
        status.setdefault("components", {})
        try:
            res = self._reconcile(isvc, status, cfg, mode)
        except Exception as e:
            set_failed = not isinstance(e, (Conflict,))
            if set_failed:
                S.set_condition(status, "Ready", "False", type(e).__name__, str(e)[:1000])
                self._write_status(isvc, status)
            raise
        self._write_status(isvc, status)
        return res

    def _write_status(self, isvc, status):
        cur = self.store.try_get(API, "InferenceService", isvc["metadata"]["name"], isvc["metadata"]["namespace"])
        if cur is None:
            return
        was_ready = S.is_ready(cur)
        if cur.get("status") != status:
            cur["status"] = status
            self.store.update_status(cur)
        now_ready = S.is_ready({"status": status})
        if now_ready and not was_ready:
            self.event(cur, "Normal", "InferenceServiceReady", "InferenceService is Ready")
        elif was_ready and not now_ready:
            self.event(cur, "Warning", "InferenceServiceNotReady", "InferenceService became not ready")

    def _reconcile(self, isvc: dict, status: dict, cfg: ControllerConfig, mode: str) -> Result:
        meta = isvc["metadata"]
        if mode == C.DeploymentMode.VIRTUAL:
            S.set_condition(status, "IngressReady", "True", "VirtualDeployment")
            S.set_condition(status, "EngineReady", "True", "VirtualDeployment")
            S.finalize_ready(status, [])
            return Result()
        work = copy.deepcopy(isvc)
        migrate_predictor(work)
        spec = work.get("spec") or {}
        model_ref = spec.get("model") or {}
        if not model_ref.get("name"):
            raise ValueError("model reference is required")
        try:
            base_model = self.get_base_model(model_ref["name"], meta["namespace"])
        except LookupError as e:
            self.event(isvc, "Warning", "ModelReconcileError", str(e))
            status["modelStatus"] = {"transitionStatus": "InvalidSpec",
                                     "lastFailureInfo": {"reason": "BaseModelNotFound", "message": str(e)}}
            raise
        bm_spec = V.spec_of(base_model)
        if bm_spec.disabled:
            raise ValueError(f"specified base model {model_ref['name']} is disabled")
        ft_weights = []
        for ftn in model_ref.get("fineTunedWeights") or []:
            ft = self.store.try_get(API, "FineTunedWeight", ftn)
            if ft is None:
                raise LookupError(f"No FineTunedWeight with the name: {ftn}")
            ft_weights.append(ft)
        if len(ft_weights) > 1:
            raise ValueError("stacked fine-tuned serving is not supported yet")
        W.reconcile_modelconfig(self.store, isvc, base_model["metadata"]["name"], base_model.get("spec") or {},
                                [f.get("spec") for f in ft_weights])
        # runtime
        rt_ref = spec.get("runtime") or {}
        try:
            if rt_ref.get("name"):
                user_rt = True
                rt_name = rt_ref["name"]
                rt_spec = self.runtime_selector.validate(rt_name, bm_spec, work, meta["namespace"])
            else:
                user_rt = False
                sel = self.runtime_selector.select(bm_spec, work, meta["namespace"])
                rt_name, rt_spec = sel.name, sel.spec
        except SelectorError as e:
            self.event(isvc, "Warning", "RuntimeSelectionError", str(e))
            status["modelStatus"] = {"transitionStatus": "InvalidSpec",
                                     "lastFailureInfo": {"reason": "NoSupportingRuntime", "message": str(e)[:1000]}}
            raise
        rt_json = rt_spec.dump()
        engine = M.merge_spec(rt_json.get("engineConfig"), spec.get("engine"))
        decoder = M.merge_spec(rt_json.get("decoderConfig"), spec.get("decoder"))
        router = M.merge_spec(rt_json.get("routerConfig"), spec.get("router")) if spec.get("router") is not None else None
        e_mode, d_mode, r_mode = determine_modes(engine, decoder, router)
        if engine is not None and not mode_from_annotations(engine.get("annotations")) and \
                mode_from_annotations(meta.get("annotations")) in (C.DeploymentMode.MULTINODE_RAY_VLLM,
                                                                  C.DeploymentMode.SERVERLESS) and decoder is None:
            e_mode = mode_from_annotations(meta.get("annotations"))
        fmt = self.runtime_selector.supported_format(rt_spec, bm_spec, user_rt)
        infos: dict[str, dict] = {}
        requeue = None
        for kind, cspec, cmode in ((C.ENGINE, engine, e_mode), (C.DECODER, decoder, d_mode),
                                   (C.ROUTER, router, r_mode)):
            if cspec is None:
                continue
            ac_obj, ac_name = (None, "")
            if kind in (C.ENGINE, C.DECODER):
                ac_obj, ac_name = self.ac_selector.get_accelerator_class(work, rt_spec, kind)
            ctx = ComponentContext(self.store, work, cfg, cmode, base_model, rt_name, rt_json, fmt, ac_name,
                                   (ac_obj or {}).get("spec"), ft_weights)
            info = make_component(kind, ctx, cspec).reconcile()
            infos[kind] = info
            comp_status = status["components"].setdefault(kind, {})
            if ac_name:
                comp_status["selectedAccelerator"] = {
                    "acceleratorClass": ac_name,
                    "reason": "explicit" if self.ac_selector.class_by_name(work, kind) else
                    f"policy:{self.ac_selector.policy(work, kind)}",
                    "nodeSelector": ((ac_obj or {}).get("spec") or {}).get("discovery", {}).get("nodeSelector") or {}}
            if info.get("requeue_after"):
                requeue = min(requeue or 1e9, info["requeue_after"])
        # ingress / external service / URL
        ingress_mode = r_mode if router is not None else (d_mode if decoder is not None else e_mode)
        entry = C.ROUTER if router is not None else (C.DECODER if decoder is not None else C.ENGINE)
        ic = resolve_ingress(cfg.ingress, meta.get("annotations"))
        entry_svc = C.component_name(meta["name"], entry)
        ing = W.reconcile_ingress(self.store, isvc, ic, ingress_mode, entry_svc)
        S.set_condition(status, "IngressReady", ing["status"], ing.get("reason", ""), ing.get("message", ""))
        W.reconcile_external_service(self.store, isvc, entry, ic)
        if ic.disableIngressCreation:
            url = f"http://{meta['name']}.{meta['namespace']}.svc.cluster.local:{C.DEFAULT_HTTP_PORT}"
        else:
            url = f"{ic.urlScheme}://{W.domain_name(meta['name'], meta, ic)}{W.url_path(isvc, ic)}"
        status["url"] = url
        status["address"] = {"url": url}
        # cleanup components removed from the spec
        present = set(infos)
        for kind in (C.ENGINE, C.DECODER, C.ROUTER):
            if kind not in present:
                self._cleanup_component(isvc, kind)
                status["components"].pop(kind, None)
                for c in list(status.get("conditions") or []):
                    if c["type"] == S.READY_CONDITION[kind]:
                        status["conditions"].remove(c)
        # component status
        for kind, info in infos.items():
            st, reason, msg = S.workload_ready(info)
            S.set_condition(status, S.READY_CONDITION[kind], st, reason, msg)
            cs = status["components"].setdefault(kind, {})
            obj = info.get("object") or {}
            cs["latestCreatedRevision"] = str(obj.get("metadata", {}).get("generation", ""))
            if st == "True":
                cs["url"] = f"http://{C.component_name(meta['name'], kind)}.{meta['namespace']}.svc.cluster.local"
                cs["latestReadyRevision"] = cs["latestCreatedRevision"]
        pods = S.component_pods(self.store, isvc, entry if entry != C.ROUTER else C.ENGINE)
        status["modelStatus"] = S.model_status_from_pods(pods)
        status["observedGeneration"] = meta.get("generation", 1)
        S.finalize_ready(status, sorted(infos))
        if not S.is_ready({"status": status}):
            requeue = min(requeue or 5.0, 5.0)
        return Result(requeue_after=requeue)

    def _cleanup_component(self, isvc: dict, kind: str) -> None:
        m = isvc["metadata"]
        uid = m.get("uid")
        sel = {C.ISVC_LABEL: m["name"], C.COMPONENT_LABEL: kind}
        for api, k in (("apps/v1", "Deployment"), ("v1", "Service"), ("leaderworkerset.x-k8s.io/v1", "LeaderWorkerSet"),
                       ("autoscaling/v2", "HorizontalPodAutoscaler"), ("keda.sh/v1alpha1", "ScaledObject"),
                       ("policy/v1", "PodDisruptionBudget"), ("serving.knative.dev/v1", "Service"),
                       ("ray.io/v1", "RayCluster")):
            for o in self.store.list(api, k, m["namespace"], selector=sel):
                if any(r.get("uid") == uid for r in o["metadata"].get("ownerReferences") or []):
                    try:
                        self.store.delete(api, k, o["metadata"]["name"], m["namespace"])
                    except NotFound:
                        pass


def setup(store: Store) -> Controller:
    r = InferenceServiceReconciler(store)

    def runtime_changed(obj):  # a (Cluster)ServingRuntime change may re-select runtimes
        return [Controller.key_of(o) for o in store.list(API, "InferenceService")]

    def model_changed(obj):
        name = obj["metadata"]["name"]
        return [Controller.key_of(o) for o in store.list(API, "InferenceService")
                if ((o.get("spec") or {}).get("model") or {}).get("name") == name]

    def pod_changed(obj):
        lab = obj["metadata"].get("labels") or {}
        if C.ISVC_LABEL in lab:
            return [(obj["metadata"].get("namespace", ""), lab[C.ISVC_LABEL])]
        return []

    c = Controller("inferenceservice", store, r.reconcile, (API, "InferenceService"),
                   owns=[("apps/v1", "Deployment"), ("v1", "Service"), ("v1", "ConfigMap"),
                         ("autoscaling/v2", "HorizontalPodAutoscaler"), ("policy/v1", "PodDisruptionBudget"),
                         ("leaderworkerset.x-k8s.io/v1", "LeaderWorkerSet"), ("ray.io/v1", "RayCluster"),
                         ("keda.sh/v1alpha1", "ScaledObject")],
                   watches=[("ServingRuntime", runtime_changed), ("ClusterServingRuntime", runtime_changed),
                            ("BaseModel", model_changed), ("ClusterBaseModel", model_changed),
                            ("Pod", pod_changed)])
    c.reconciler = r
    return c

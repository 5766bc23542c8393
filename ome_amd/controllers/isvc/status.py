"""InferenceService status propagation (``status/status_reconciler.go``, ``inference_service_status.go``).

Component readiness comes from the workload: Deployment ``Available`` (Raw), LeaderWorkerSet
``Available`` (MultiNode), every prober Deployment available (MultiNodeRayVLLM), KSVC ``Ready``
(Serverless).  The top-level ``Ready`` condition is the living set IngressReady ∧ EngineReady,
plus DecoderReady / RouterReady when those components exist (a PD service without decoders
cannot serve; the reference only gates on engine + ingress).  Model status is derived from the
component pods: Loaded / Loading / Pending / FailedToLoad with the container termination
message + exit code as ``lastFailureInfo``.
"""
from __future__ import annotations

from ome_amd.api import constants as C
from ome_amd.store.store import Store, now_iso

READY_CONDITION = {C.ENGINE: "EngineReady", C.DECODER: "DecoderReady", C.ROUTER: "RouterReady",
                   C.PREDICTOR: "PredictorReady"}


def get_condition(status: dict, ctype: str) -> dict | None:
    for c in status.get("conditions") or []:
        if c.get("type") == ctype:
            return c
    return None


def set_condition(status: dict, ctype: str, state: str, reason: str = "", message: str = "") -> None:
    conds = status.setdefault("conditions", [])
    for c in conds:
        if c["type"] == ctype:
            if c.get("status") != state:
                c["lastTransitionTime"] = now_iso()
            c.update({"status": state, "reason": reason, "message": message})
            return
    conds.append({"type": ctype, "status": state, "reason": reason, "message": message,
                  "lastTransitionTime": now_iso()})
    conds.sort(key=lambda c: c["type"])


def _cond(obj: dict | None, ctype: str) -> dict | None:
    for c in ((obj or {}).get("status") or {}).get("conditions") or []:
        if c.get("type") == ctype:
            return c
    return None


def workload_ready(info: dict) -> tuple[str, str, str]:
    mode = info["mode"]
    if mode == C.DeploymentMode.RAW:
        c = _cond(info.get("object"), "Available")
        if c is None:
            return "Unknown", "DeploymentPending", "deployment has no Available condition yet"
        return c.get("status", "Unknown"), c.get("reason", ""), c.get("message", "")
    if mode == C.DeploymentMode.MULTINODE:
        c = _cond(info.get("object"), "Available")
        if c is None:
            return "Unknown", "LeaderWorkerSetPending", "leaderworkerset has no Available condition yet"
        return c.get("status", "Unknown"), c.get("reason", ""), c.get("message", "")
    if mode == C.DeploymentMode.MULTINODE_RAY_VLLM:
        objs = info.get("objects") or []
        if not objs:
            return "False", "NoDeployments", "No deployments available"
        for o in objs:
            c = _cond(o, "Available")
            if c is None or c.get("status") != "True":
                return "False", "ProberUnavailable", f"multinode prober {o['metadata']['name']} not available"
        return "True", "", ""
    if mode == C.DeploymentMode.SERVERLESS:
        c = _cond(info.get("object"), "Ready")
        if c is None:
            return "Unknown", "KnativePending", "knative service not ready"
        return c.get("status", "Unknown"), c.get("reason", ""), c.get("message", "")
    return "Unknown", "", ""


def model_status_from_pods(pods: list[dict]) -> dict:
    if not pods:
        return {"transitionStatus": "InProgress", "modelRevisionStates": {"activeModelState": "Pending",
                                                                         "targetModelState": "Pending"}}
    ready = 0
    failure = None
    for p in pods:
        st = p.get("status") or {}
        if any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or []):
            ready += 1
        for cs in st.get("containerStatuses") or []:
            term = (cs.get("state") or {}).get("terminated") or (cs.get("lastState") or {}).get("terminated")
            if term and int(term.get("exitCode", 0)) != 0:
                failure = {"location": p["metadata"]["name"], "reason": "ModelLoadFailed",
                           "message": term.get("message") or term.get("reason", ""),
                           "exitCode": int(term.get("exitCode", 1)), "time": now_iso()}
    if ready:
        out = {"transitionStatus": "UpToDate", "modelRevisionStates": {"activeModelState": "Loaded",
                                                                      "targetModelState": "Loaded"}}
    elif failure:
        out = {"transitionStatus": "BlockedByFailedLoad",
               "modelRevisionStates": {"activeModelState": "FailedToLoad", "targetModelState": "FailedToLoad"},
               "lastFailureInfo": failure}
    else:
        out = {"transitionStatus": "InProgress", "modelRevisionStates": {"activeModelState": "Loading",
                                                                        "targetModelState": "Loaded"}}
    out["modelCopies"] = {"failedCopies": sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Failed"),
                          "totalCopies": len(pods)}
    return out


def component_pods(store: Store, isvc: dict, component: str) -> list[dict]:
    m = isvc["metadata"]
    return store.list("v1", "Pod", m["namespace"], selector={C.ISVC_LABEL: m["name"], C.COMPONENT_LABEL: component})


def finalize_ready(status: dict, components: list[str]) -> None:
    need = ["IngressReady"] + [READY_CONDITION[c] for c in components]
    bad = [n for n in need if (get_condition(status, n) or {}).get("status") != "True"]
    if not bad:
        set_condition(status, "Ready", "True")
    else:
        first = get_condition(status, bad[0]) or {}
        st = "False" if first.get("status") == "False" else "Unknown"
        set_condition(status, "Ready", st, first.get("reason") or "NotReady",
                      first.get("message") or f"waiting for {', '.join(bad)}")


def is_ready(isvc: dict) -> bool:
    return (get_condition(isvc.get("status") or {}, "Ready") or {}).get("status") == "True"

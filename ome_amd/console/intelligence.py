"""Runtime intelligence for the web console: which ServingRuntimes can serve a model, a
recommendation, and pre-creation validation of a runtime manifest.

Reference behaviour: ``web-console/backend/internal/services/runtime_intelligence.go:47-309``
(FindCompatibleRuntimes / CheckCompatibility / GetRecommendation / ValidateRuntimeConfiguration).
The reference console scores runtimes with its own ad-hoc heuristic (format name match +50,
multi-model +10, HTTP protocol +5, framework substring in the image +20) that can disagree with
what the controller will actually pick.  Here the console asks the same RuntimeSelector the
InferenceService controller uses (``ome_amd.policy.runtime_selector``, reference
``pkg/runtimeselector``), so "recommended" is by construction the runtime an InferenceService
without ``spec.runtime`` would get; the score breakdown and human-readable reasons are derived
from that selector's compatibility checks.
"""
from __future__ import annotations

from ome_amd.api import v1beta1 as V
from ome_amd.policy import runtime_selector as RS

API = "ome.io/v1beta1"

# common format-name aliases (the reference console's alias table, runtime_intelligence.go:218-223)
_ALIASES = {"pytorch": {"torch", "pt", "pth"}, "tensorflow": {"tf", "savedmodel"}, "onnx": set(),
            "safetensors": {"safetensor", "st"}}


def canonical_format(name: str | None) -> str:
    n = (name or "").strip().lower()
    for canon, al in _ALIASES.items():
        if n == canon or n in al:
            return canon
    return n


def model_spec_from_query(model_format: str, framework: str | None = None, architecture: str | None = None,
                          size: str | None = None, quantization: str | None = None,
                          format_version: str | None = None) -> V.BaseModelSpec:
    """A minimal BaseModelSpec from console query parameters (``?modelFormat=&modelFramework=``)."""
    spec: dict = {"modelFormat": {"name": canonical_format(model_format)}}
    if format_version:
        spec["modelFormat"]["version"] = format_version
    if framework:
        spec["modelFramework"] = {"name": framework}
    if architecture:
        spec["modelArchitecture"] = architecture
    if size:
        spec["modelParameterSize"] = size
    if quantization:
        spec["quantization"] = quantization
    return V.BaseModelSpec.model_validate(spec)


def model_spec_of(store, name: str, namespace: str | None) -> V.BaseModelSpec:
    obj = store.try_get(API, "BaseModel", name, namespace) if namespace else None
    if obj is None:
        obj = store.get(API, "ClusterBaseModel", name)
    return V.spec_of(obj)


def _reasons(spec: V.ServingRuntimeSpec, model: V.BaseModelSpec) -> list[str]:
    out = []
    for f in spec.supported_model_formats or []:
        if not RS.format_mismatch(model, f):
            out.append(f"supports model format {f.model_format.name if f.model_format else f.name}"
                       + (f" / architecture {f.model_architecture}" if f.model_architecture else "")
                       + (f" (priority {f.priority})" if f.priority else ""))
    if spec.model_size_range:
        out.append(f"model size within [{spec.model_size_range.min}, {spec.model_size_range.max}]")
    return out


def evaluate(store, name: str, spec: V.ServingRuntimeSpec, model: V.BaseModelSpec, isvc: dict | None = None,
             is_cluster: bool = True) -> dict:
    """Compatibility verdict of one runtime for one model (the CheckCompatibility response)."""
    warnings: list[str] = []
    if spec.is_disabled():
        return {"runtime": name, "compatible": False, "score": 0, "reasons": [], "warnings": ["runtime is disabled"],
                "clusterScoped": is_cluster}
    ok, why = RS.compatibility(spec, model, isvc)
    score = RS.runtime_score(spec, model) if ok else 0
    if ok and not any(f.auto_select for f in spec.supported_model_formats or []):
        warnings.append("autoSelect is off: only used when an InferenceService names it explicitly")
    return {"runtime": name, "compatible": bool(ok and score > 0), "score": int(score),
            "reasons": _reasons(spec, model) if ok else [], "warnings": warnings + ([] if ok else list(why)),
            "clusterScoped": is_cluster}


def find_compatible(store, model: V.BaseModelSpec, namespace: str = "default", isvc: dict | None = None) -> list[dict]:
    """Every compatible runtime, best first, in the RuntimeSelector's order (namespace runtimes
    before cluster runtimes at equal score, then closest size range, then name)."""
    sel = RS.RuntimeSelector(store)
    ranked = sel.compatible_runtimes(model, isvc, namespace)
    out = []
    for m in ranked:
        d = evaluate(store, m.name, m.spec, model, isvc, m.is_cluster)
        d["score"] = m.score
        out.append(d)
    return out


def recommend(store, model: V.BaseModelSpec, namespace: str = "default", isvc: dict | None = None) -> dict:
    sel = RS.RuntimeSelector(store)
    try:
        m = sel.select(model, isvc, namespace)
    except RS.NoRuntimeFoundError as e:
        return {"runtime": None, "error": str(e)}
    d = evaluate(store, m.name, m.spec, model, isvc, m.is_cluster)
    d["score"] = m.score
    d["recommendation"] = "the runtime the InferenceService controller selects for this model"
    return d


def validate_runtime(obj: dict) -> tuple[list[str], list[str]]:
    """(errors, warnings) for a (Cluster)ServingRuntime manifest before it is created
    (reference ValidateRuntimeConfiguration + schema validation through the pydantic model)."""
    errors: list[str] = []
    warnings: list[str] = []
    spec = obj.get("spec")
    if not isinstance(spec, dict):
        return ["Runtime spec is required"], warnings
    fmts = spec.get("supportedModelFormats")
    if fmts is None:
        warnings.append("No supported model formats specified")
    elif not fmts:
        warnings.append("Supported model formats list is empty")
    containers = spec.get("containers")
    engine = (spec.get("engineConfig") or {}).get("runner") or {}
    if not containers and not engine:
        errors.append("At least one container (spec.containers or spec.engineConfig.runner) is required")
    for i, c in enumerate(containers or []):
        if not isinstance(c, dict):
            errors.append(f"Container {i} is invalid")
            continue
        for key in ("name", "image"):
            if key not in c:
                errors.append(f"Container {i} is missing '{key}' field")
    if not spec.get("protocolVersions"):
        warnings.append("No protocol versions specified")
    try:
        V.ServingRuntimeSpec.model_validate(spec)
    except Exception as e:  # noqa: BLE001 — pydantic ValidationError text is the message
        errors.append(f"schema: {e}")
    return errors, warnings

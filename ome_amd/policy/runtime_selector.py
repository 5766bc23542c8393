"""RuntimeSelector: auto-select / validate a (Cluster)ServingRuntime for a base model.

Semantics follow the reference (``pkg/runtimeselector/{matcher,scorer,selector,fetcher}.go``):

* compatibility = not disabled ∧ accelerator-class requirements of the ISVC are all supported
  by the runtime ∧ some supportedModelFormat matches (diffusion pipeline, architecture,
  quantization, format name+version, framework name+version — each "both set and equal, or
  both unset") ∧ model size within ``modelSizeRange``;
* only runtimes with at least one ``autoSelect: true`` format take part in auto-selection;
* score = max over auto-select formats of Σ weight × priority (format weight default 10,
  framework weight default 5, priority default 1);
* ordering: score desc → size proximity (|min-size| + |max-size|, smaller first) →
  namespace-scoped before cluster-scoped → name asc; namespace-scoped matches always precede
  cluster-scoped ones in the final list.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from ome_amd.api import v1beta1 as V
from ome_amd.policy import version as ver
from ome_amd.store.store import NotFound, Store


class SelectorError(Exception):
    pass


class RuntimeNotFoundError(SelectorError):
    def __init__(self, name: str, namespace: str):
        super().__init__(f"runtime {name} not found in namespace {namespace} or cluster scope")
        self.name, self.namespace = name, namespace


class RuntimeDisabledError(SelectorError):
    def __init__(self, name: str, is_cluster: bool = False):
        super().__init__(f"runtime {name} is disabled")
        self.name = name


class RuntimeCompatibilityError(SelectorError):
    def __init__(self, runtime: str, model_format: str, reason: str):
        super().__init__(f"runtime {runtime} does not support model format {model_format}: {reason}")
        self.runtime, self.reason = runtime, reason


class NoRuntimeFoundError(SelectorError):
    def __init__(self, model_format: str, namespace: str, excluded: dict[str, str], n_ns: int, n_cluster: int):
        lines = [f"no runtime found to support model format {model_format!r} in namespace {namespace!r} "
                 f"({n_ns} namespace-scoped, {n_cluster} cluster-scoped runtimes considered)"]
        for k, v in sorted(excluded.items()):
            lines.append(f"  - {k}: {v}")
        super().__init__("\n".join(lines))
        self.excluded = excluded


class ModelValidationError(SelectorError):
    pass


@dataclass
class RuntimeMatch:
    name: str
    spec: V.ServingRuntimeSpec
    score: int
    is_cluster: bool
    details: dict = field(default_factory=dict)


DEFAULT_PRIORITY = 1
FORMAT_WEIGHT = 10
FRAMEWORK_WEIGHT = 5


def parse_model_size(s: str | None) -> float:
    if not s:
        return 0.0
    mult = 1.0
    for suf, m in (("T", 1e12), ("B", 1e9), ("M", 1e6), ("K", 1e3)):
        if s.endswith(suf):
            s, mult = s[:-1], m
            break
    try:
        return float(s) * mult
    except ValueError:
        return 0.0


def _both_or_neither(a, b) -> bool:
    return (a is None) == (b is None)


def _cmp_component(name, model: V.DiffusionComponentSpec | None, rt: V.DiffusionComponentSpec | None):
    if rt is None:
        return True, ""
    if model is None:
        return False, f"component {name} required by runtime but not specified in model"
    if rt.library and rt.library != model.library:
        return False, f"{name} library mismatch (model={model.library}, runtime={rt.library})"
    if rt.type and rt.type != model.type:
        return False, f"{name} type mismatch (model={model.type}, runtime={rt.type})"
    return True, ""


def compare_diffusion(model: V.DiffusionPipelineSpec | None, fmt: V.DiffusionPipelineSpec | None):
    if fmt is None:
        return True, ""
    if model is None:
        return False, "diffusion pipeline required by runtime but not specified in model"
    if fmt.class_name is not None and model.class_name != fmt.class_name:
        return False, f"pipeline class mismatch (model={model.class_name}, runtime={fmt.class_name})"
    for n in ("scheduler", "text_encoder", "tokenizer", "transformer", "vae"):
        ok, r = _cmp_component(n, getattr(model, n), getattr(fmt, n))
        if not ok:
            return ok, r
    if fmt.additional_components:
        if not model.additional_components:
            return False, "diffusion pipeline missing required additional components"
        for k, c in fmt.additional_components.items():
            if k not in model.additional_components:
                return False, f"diffusion component {k} missing in model"
            ok, r = _cmp_component(k, model.additional_components[k], c)
            if not ok:
                return ok, r
    return True, ""


def _versioned_match(fmt: V.ModelFormat | None, model: V.ModelFormat | None) -> tuple[bool, str]:
    """name + version compatibility of a format/framework pair (both present)."""
    if fmt.name != model.name:
        return False, f"name mismatch (model={model.name}, runtime={fmt.name})"
    if fmt.version is not None and model.version is not None:
        if not ver.satisfies(fmt.version, model.version, fmt.operator):
            return False, f"version mismatch (model={model.version}, runtime={fmt.version})"
    elif not _both_or_neither(fmt.version, model.version):
        return False, "version requirement mismatch"
    return True, ""


def format_mismatch(model: V.BaseModelSpec, f: V.SupportedModelFormat) -> list[str]:
    """Every reason a supported format does not match a model (empty list == compatible)."""
    reasons = []
    ok, r = compare_diffusion(model.diffusion_pipeline, f.diffusion_pipeline)
    if not ok:
        reasons.append(r or "diffusion pipeline mismatch")
    if model.model_architecture is not None and f.model_architecture is not None:
        if model.model_architecture != f.model_architecture:
            reasons.append(f"architecture mismatch (model={model.model_architecture}, runtime={f.model_architecture})")
    elif not _both_or_neither(model.model_architecture, f.model_architecture):
        reasons.append("architecture requirement mismatch")
    if model.quantization is not None and f.quantization is not None:
        if model.quantization != f.quantization:
            reasons.append(f"quantization mismatch (model={model.quantization}, runtime={f.quantization})")
    elif not _both_or_neither(model.quantization, f.quantization):
        reasons.append("quantization requirement mismatch")
    mf = model.model_format
    if f.model_format is not None and mf is not None:
        ok, r = _versioned_match(f.model_format, mf)
        if not ok:
            reasons.append("format " + r)
    elif not _both_or_neither(f.model_format, mf):
        reasons.append("format requirement mismatch")
    if f.model_framework is not None and model.model_framework is not None:
        ok, r = _versioned_match(f.model_framework, model.model_framework)
        if not ok:
            reasons.append("framework " + r)
    elif not _both_or_neither(f.model_framework, model.model_framework):
        reasons.append("framework requirement mismatch")
    return reasons


def isvc_accelerator_classes(isvc: dict | None) -> set[str]:
    if not isvc:
        return set()
    req = set()
    ann = isvc.get("metadata", {}).get("annotations") or {}
    if "ome.io/accelerator-class" in ann:
        req.add(ann["ome.io/accelerator-class"])
    sp = isvc.get("spec") or {}
    ac = (sp.get("acceleratorSelector") or {}).get("acceleratorClass")
    if ac:
        req.add(ac)
    for comp in ("engine", "decoder"):
        c = ((sp.get(comp) or {}).get("acceleratorOverride") or {}).get("acceleratorClass")
        if c:
            req.add(c)
    return req


def accelerator_compatible(rt: V.ServingRuntimeSpec, isvc: dict | None) -> bool:
    req = isvc_accelerator_classes(isvc)
    if not req:
        return True
    sup = (rt.accelerator_requirements.accelerator_classes if rt.accelerator_requirements else None) or []
    return bool(sup) and req.issubset(set(sup))


def size_ok(rt: V.ServingRuntimeSpec, model: V.BaseModelSpec) -> bool:
    if not model.model_parameter_size or rt.model_size_range is None:
        return True
    s = parse_model_size(model.model_parameter_size)
    return parse_model_size(rt.model_size_range.min) <= s <= parse_model_size(rt.model_size_range.max)


def compatibility(rt: V.ServingRuntimeSpec, model: V.BaseModelSpec, isvc: dict | None) -> tuple[bool, list[str]]:
    if rt.is_disabled():
        return False, ["runtime is disabled"]
    if not accelerator_compatible(rt, isvc):
        return False, ["runtime does not support the required accelerator class"]
    mismatches = []
    for f in rt.supported_model_formats or []:
        r = format_mismatch(model, f)
        if not r:
            if size_ok(rt, model):
                return True, []
            return False, [f"model size {model.model_parameter_size} is outside supported range "
                           f"[{rt.model_size_range.min}, {rt.model_size_range.max}]"]
        mismatches.append(", ".join(r))
    label = model.model_format.name if model.model_format else "?"
    return False, [f"model format '{label}' not in supported formats: " + ("; ".join(mismatches) or "none defined")]


def format_score(model: V.BaseModelSpec, f: V.SupportedModelFormat, priority: int) -> int:
    mf, fmt_ok, fw_ok = model.model_format, False, False
    if f.model_format is not None and mf is not None:
        if f.model_format.name != mf.name:
            return 0
        if f.model_format.version is not None and mf.version is not None:
            if not ver.satisfies(f.model_format.version, mf.version, f.model_format.operator):
                return 0
        fmt_ok = True
    if f.model_framework is not None and model.model_framework is not None:
        if f.model_framework.name != model.model_framework.name:
            return 0
        fv, mv = f.model_framework.version, model.model_framework.version
        if fv is not None and mv is not None and not ver.satisfies(fv, mv, f.model_framework.operator):
            return 0
        fw_ok = True
    if not (fmt_ok or (f.model_format is None and mf is None)):
        return 0
    if not (fw_ok or (f.model_framework is None and model.model_framework is None)):
        return 0
    score = 0
    if fmt_ok:
        score += (f.model_format.weight or FORMAT_WEIGHT) * priority
    if fw_ok:
        score += (f.model_framework.weight or FRAMEWORK_WEIGHT) * priority
    return score


def runtime_score(rt: V.ServingRuntimeSpec, model: V.BaseModelSpec) -> int:
    best = 0
    for f in rt.supported_model_formats or []:
        if f.auto_select is False:
            continue
        pr = f.priority if f.priority is not None else DEFAULT_PRIORITY
        best = max(best, format_score(model, f, pr))
    return best


def _size_distance(m: RuntimeMatch, model: V.BaseModelSpec) -> float:
    r = m.spec.model_size_range
    if r is None or not model.model_parameter_size:
        return 0.0
    s = parse_model_size(model.model_parameter_size)
    return abs(parse_model_size(r.min) - s) + abs(parse_model_size(r.max) - s)


def _sort(matches: list[RuntimeMatch], model: V.BaseModelSpec) -> list[RuntimeMatch]:
    return sorted(matches, key=lambda m: (-m.score, _size_distance(m, model) if model.model_parameter_size else 0,
                                          m.is_cluster, m.name))


class RuntimeSelector:
    def __init__(self, store: Store):
        self.store = store

    def fetch(self, namespace: str) -> tuple[list[dict], list[dict]]:
        def order(objs):
            return sorted(objs, key=lambda o: o["metadata"]["name"])
        ns = order(self.store.list("ome.io/v1beta1", "ServingRuntime", namespace=namespace))
        cl = order(self.store.list("ome.io/v1beta1", "ClusterServingRuntime"))
        return ns, cl

    def get_runtime(self, name: str, namespace: str) -> tuple[V.ServingRuntimeSpec, bool]:
        o = self.store.try_get("ome.io/v1beta1", "ServingRuntime", name, namespace)
        if o is not None:
            return V.spec_of(o), False
        o = self.store.try_get("ome.io/v1beta1", "ClusterServingRuntime", name)
        if o is not None:
            return V.spec_of(o), True
        raise RuntimeNotFoundError(name, namespace)

    @staticmethod
    def _validate(model: V.BaseModelSpec) -> None:
        if model is None:
            raise ModelValidationError("model specification is nil")
        if model.model_format is None or not model.model_format.name:
            raise ModelValidationError("model format name is required")

    def compatible_runtimes(self, model: V.BaseModelSpec, isvc: dict | None, namespace: str) -> list[RuntimeMatch]:
        self._validate(model)
        ns, cl = self.fetch(namespace)
        out = {False: [], True: []}
        for is_cluster, objs in ((False, ns), (True, cl)):
            for o in objs:
                spec = V.spec_of(o)
                if spec.is_disabled():
                    continue
                ok, _ = compatibility(spec, model, isvc)
                if not ok or not any(f.auto_select for f in spec.supported_model_formats or []):
                    continue
                sc = runtime_score(spec, model)
                if sc <= 0:
                    continue
                out[is_cluster].append(RuntimeMatch(o["metadata"]["name"], spec, sc, is_cluster))
        return _sort(out[False], model) + _sort(out[True], model)

    def select(self, model: V.BaseModelSpec, isvc: dict | None, namespace: str) -> RuntimeMatch:
        matches = self.compatible_runtimes(model, isvc, namespace)
        if matches:
            return matches[0]
        ns, cl = self.fetch(namespace)
        excluded = {}
        for o in ns + cl:
            ok, reasons = compatibility(V.spec_of(o), model, isvc)
            if not ok and reasons:
                excluded[o["metadata"]["name"]] = reasons[0]
            elif ok:
                excluded[o["metadata"]["name"]] = "auto-select disabled or zero score"
        raise NoRuntimeFoundError(model.model_format.name, namespace, excluded, len(ns), len(cl))

    def validate(self, name: str, model: V.BaseModelSpec, isvc: dict | None, namespace: str) -> V.ServingRuntimeSpec:
        self._validate(model)
        spec, is_cluster = self.get_runtime(name, namespace)
        if spec.is_disabled():
            raise RuntimeDisabledError(name, is_cluster)
        ok, reasons = compatibility(spec, model, isvc)
        if not ok:
            raise RuntimeCompatibilityError(name, model.model_format.name, reasons[0] if reasons else "incompatible")
        return spec

    def supported_format(self, rt: V.ServingRuntimeSpec, model: V.BaseModelSpec,
                         user_specified: bool) -> V.SupportedModelFormat | None:
        best, best_score = None, 0
        for f in rt.supported_model_formats or []:
            if not user_specified and not f.auto_select:
                continue
            s = format_score(model, f, DEFAULT_PRIORITY)
            if s > best_score:
                best, best_score = f, s
        return best


__all__ = ["RuntimeSelector", "RuntimeMatch", "NoRuntimeFoundError", "RuntimeNotFoundError",
           "RuntimeDisabledError", "RuntimeCompatibilityError", "ModelValidationError", "parse_model_size",
           "compatibility", "runtime_score", "NotFound"]

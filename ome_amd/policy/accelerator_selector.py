"""AcceleratorClassSelector: choose the AcceleratorClass for an ISVC component.

Decision order (``pkg/acceleratorclassselector/selector.go:46-85``): only when the runtime
declares ``acceleratorRequirements.acceleratorClasses``; explicit name first (component
``acceleratorOverride.acceleratorClass`` -> ISVC ``acceleratorSelector.acceleratorClass``),
else a policy (component override policy -> ISVC selector policy) over the runtime's
candidate list filtered by the ISVC constraints.

Policies (scores as in ``policy_helpers.go``):
* BestFit      0.70 * memory-fit (1 / over-provision ratio) + 0.30 * compute score, where the
               compute score walks the preferred precisions with a 1, 0.5, 0.25, ... penalty and
               falls back to fp16 at the accumulated penalty;
* Cheapest     spot/hour > hour > per-million-tokens > tier (low=1, medium=2, high=3);
* MostCapable  0.5 * mem + 0.3 * bandwidth + 0.2 * TFLOPS, each normalised to the candidate max;
* FirstAvailable  first candidate in runtime-declared order.
Fixes vs the reference: candidate order is the runtime's declared order (the reference
iterates a Go map, so "FirstAvailable" was effectively random), and a policy with no
constraints scores instead of dereferencing a nil constraint block.
"""
from __future__ import annotations

from ome_amd.api import v1beta1 as V
from ome_amd.store.store import Store
from ome_amd.utils.quantity import to_float, to_gib

BEST_FIT, CHEAPEST, MOST_CAPABLE, FIRST_AVAILABLE = "BestFit", "Cheapest", "MostCapable", "FirstAvailable"
POLICIES = (BEST_FIT, CHEAPEST, MOST_CAPABLE, FIRST_AVAILABLE)


def _spec(ac: dict) -> V.AcceleratorClassSpec:
    return V.AcceleratorClassSpec.model_validate(ac.get("spec") or {})


def tflops_for(perf: V.AcceleratorPerformance | None, precision: str) -> int:
    if perf is None:
        return 0
    p = precision.lower()
    val = {"fp32": perf.fp32_tflops, "fp16": perf.fp16_tflops, "bf16": perf.fp16_tflops, "int8": perf.int8_tops,
           "fp8": perf.int8_tops, "int4": perf.int4_tops, "fp4": perf.int4_tops}.get(p)
    return int(val or 0)


def max_tflops(perf: V.AcceleratorPerformance | None) -> int:
    if perf is None:
        return 0
    return max(int(x or 0) for x in (perf.fp32_tflops, perf.fp16_tflops, perf.int8_tops, perf.int4_tops))


def meets_requirements(ac: dict, c: V.AcceleratorConstraints | None) -> tuple[bool, str]:
    if c is None:
        return True, ""
    s = _spec(ac)
    name = ac["metadata"]["name"]
    if name in (c.excluded_classes or []):
        return False, "explicitly excluded"
    if c.architecture_families:
        vf = f"{(s.vendor or '').lower()}-{(s.family or '').lower()}"
        fam = (s.family or "").lower()
        if not any((f.lower() == vf) if "-" in f else (f.lower() == fam) for f in c.architecture_families):
            return False, f"architecture family {fam} not in allowed list"
    if c.min_memory is not None or c.max_memory is not None:
        if s.capabilities.memory_gb is None:
            return False, "missing memory specification for memory check"
        mem = int(to_gib(s.capabilities.memory_gb))
        if c.min_memory is not None and mem < c.min_memory:
            return False, f"memory {mem}GB < required {c.min_memory}GB"
        if c.max_memory is not None and mem > c.max_memory:
            return False, f"memory {mem}GB > max allowed {c.max_memory}GB"
    if c.required_features:
        have = {f.lower() for f in s.capabilities.features or []}
        for f in c.required_features:
            if f.lower() not in have:
                return False, f"missing required feature: {f}"
    if c.min_architecture_version is not None:
        cc = s.capabilities.compute_capability
        if not cc:
            return False, "missing compute capability for architecture version check"
        if cc < c.min_architecture_version:
            return False, f"compute capability {cc} < required {c.min_architecture_version}"
    return True, ""


def _tflops_score(tf: int, required: int) -> float:
    if tf == 0:
        return 0.0
    if required == 0:
        return 1.0
    return min(1.0, tf / required)


def memory_fit_score(ac: dict, c: V.AcceleratorConstraints | None) -> float:
    if c is None or c.min_memory is None:
        return 1.0
    s = _spec(ac)
    if s.capabilities.memory_gb is None:
        return 0.0
    have, need = to_gib(s.capabilities.memory_gb), float(c.min_memory)
    if have < need:
        return 0.0
    if need <= 0 or have == need:
        return 1.0
    return need / have


def compute_score(ac: dict, c: V.AcceleratorConstraints | None) -> float:
    perf = _spec(ac).capabilities.performance
    if perf is None:
        return 0.0
    req = (c.min_compute_performance_tflops if c else None) or 0
    prefs = (c.preferred_precisions if c else None) or []
    if not prefs:
        return _tflops_score(max_tflops(perf), req)
    penalty = 1.0
    for p in prefs:
        tf = tflops_for(perf, p)
        if tf > 0:
            return _tflops_score(tf, req) * penalty
        penalty *= 0.5
    if "fp16" not in [p.lower() for p in prefs]:
        tf = tflops_for(perf, "fp16")
        if tf > 0:
            return _tflops_score(tf, req) * penalty
    return 0.0


def best_fit_score(ac: dict, c: V.AcceleratorConstraints | None) -> float:
    return 0.70 * memory_fit_score(ac, c) + 0.30 * compute_score(ac, c)


def candidate_cost(ac: dict) -> tuple[float, str] | None:
    cost = _spec(ac).cost
    if cost is None:
        return None
    if cost.spot_per_hour is not None:
        return to_float(cost.spot_per_hour), "spot-hourly"
    if cost.per_hour is not None:
        return to_float(cost.per_hour), "hourly"
    if cost.per_million_tokens is not None:
        return to_float(cost.per_million_tokens), "per-million-tokens"
    if cost.tier:
        return float({"low": 1, "medium": 2, "high": 3}.get(cost.tier.lower(), 2)), "tier"
    return None


def _raw(ac: dict, prefs: list[str]) -> tuple[float, float, float]:
    s = _spec(ac)
    primary = prefs[0].lower() if prefs else "fp16"
    tf = float(tflops_for(s.capabilities.performance, primary))
    if tf == 0.0:
        for p in prefs[1:]:
            v = tflops_for(s.capabilities.performance, p)
            if v > 0:
                tf = float(v)
                break
    mem = to_gib(s.capabilities.memory_gb) if s.capabilities.memory_gb is not None else 0.0
    bw = to_float(s.capabilities.memory_bandwidth_gbps) if s.capabilities.memory_bandwidth_gbps is not None else 0.0
    return tf, mem, bw


def capability_scores(cands: list[dict], prefs: list[str]) -> list[float]:
    raws = [_raw(a, prefs) for a in cands]
    mt = max((r[0] for r in raws), default=0) or 0
    mm = max((r[1] for r in raws), default=0) or 0
    mb = max((r[2] for r in raws), default=0) or 0
    return [0.5 * (m / mm if mm else 0) + 0.3 * (b / mb if mb else 0) + 0.2 * (t / mt if mt else 0)
            for t, m, b in raws]


class AcceleratorClassSelector:
    def __init__(self, store: Store):
        self.store = store

    def _get(self, name: str) -> dict | None:
        return self.store.try_get("ome.io/v1beta1", "AcceleratorClass", name)

    @staticmethod
    def _override(isvc: dict, component: str) -> dict:
        sp = isvc.get("spec") or {}
        return (sp.get(component) or {}).get("acceleratorOverride") or {} if component in ("engine", "decoder") else {}

    def class_by_name(self, isvc: dict, component: str) -> str | None:
        ov = self._override(isvc, component)
        if ov.get("acceleratorClass"):
            return ov["acceleratorClass"]
        return ((isvc.get("spec") or {}).get("acceleratorSelector") or {}).get("acceleratorClass")

    def policy(self, isvc: dict, component: str) -> str:
        ov = self._override(isvc, component)
        if ov.get("policy"):
            return ov["policy"]
        return ((isvc.get("spec") or {}).get("acceleratorSelector") or {}).get("policy") or ""

    def candidates(self, rt: V.ServingRuntimeSpec) -> list[dict]:
        names = (rt.accelerator_requirements.accelerator_classes if rt.accelerator_requirements else None) or []
        seen, out = set(), []
        for n in names:
            if n in seen:
                continue
            seen.add(n)
            ac = self._get(n)
            if ac is not None:
                out.append(ac)
        return out

    def select_by_policy(self, isvc: dict, rt: V.ServingRuntimeSpec, policy: str) -> str | None:
        cands = self.candidates(rt)
        sel = (isvc.get("spec") or {}).get("acceleratorSelector") or {}
        cons = V.AcceleratorConstraints.model_validate(sel["constraints"]) if sel.get("constraints") else None
        valid = [a for a in cands if meets_requirements(a, cons)[0]]
        if not valid:
            return None
        names = [a["metadata"]["name"] for a in valid]
        if policy == FIRST_AVAILABLE or len(valid) == 1:
            return names[0]
        if policy == BEST_FIT:
            scores = [best_fit_score(a, cons) for a in valid]
        elif policy == MOST_CAPABLE:
            scores = capability_scores(valid, (cons.preferred_precisions if cons else None) or [])
        elif policy == CHEAPEST:
            costs = [(candidate_cost(a), n) for a, n in zip(valid, names)]
            costs = [(c[0], n) for c, n in costs if c is not None]
            if not costs:
                return None
            return min(costs, key=lambda x: x[0])[1]
        else:
            return None
        best = max(range(len(valid)), key=lambda i: (scores[i], -i))
        return names[best]

    def get_accelerator_class(self, isvc: dict, rt: V.ServingRuntimeSpec | None, component: str) -> tuple[dict | None, str]:
        """-> (AcceleratorClass object or None, name or '')."""
        if rt is None or rt.accelerator_requirements is None or not rt.accelerator_requirements.accelerator_classes:
            return None, ""
        name = self.class_by_name(isvc, component)
        if not name:
            pol = self.policy(isvc, component)
            if not pol:
                return None, ""
            name = self.select_by_policy(isvc, rt, pol)
        if not name:
            return None, ""
        ac = self._get(name)
        if ac is None:
            raise LookupError(f"AcceleratorClass {name} not found")
        return ac, name

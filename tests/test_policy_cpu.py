"""Runtime selection (``pkg/runtimeselector``), accelerator-class selection
(``pkg/acceleratorclassselector``) and model-version semantics (``pkg/modelver``)."""
import pytest

from ome_amd.api import v1beta1 as V
from ome_amd.policy import accelerator_selector as A
from ome_amd.policy import version as ver
from ome_amd.policy.runtime_selector import (ModelValidationError, NoRuntimeFoundError, RuntimeCompatibilityError,
                                             RuntimeDisabledError, RuntimeNotFoundError, RuntimeSelector,
                                             parse_model_size)
from ome_amd.store.store import Store

API = "ome.io/v1beta1"


# ------------------------------------------------------------------ versions
@pytest.mark.parametrize("a,b,eq,gt", [
    ("1.8.0", "1.8.0", True, False), ("2.0.0", "1.9.0", False, True), ("1.9.0", "1.8.0", False, True),
    ("1.8.5", "1.8.0", False, True), ("1.0.0", "2.0.0", False, False), ("1.8.0-alpha", "1.8.0-alpha", True, False),
    ("1.8.0-beta", "1.8.0-alpha", False, True), ("1.8.0+20240707", "1.8.0+20240707", True, False),
    ("1.8.0+20240708", "1.8.0+20240707", False, True), ("v0.8.0", "v0.8.0", True, False), ("v1", "v1", True, False),
    ("1", "1", True, False), ("1.12", "1.12", True, False), ("1", "2", False, False),
    ("v1.9.0", "v2.9.0", False, False), ("v0.9.0", "v0.8.0", False, True),
])
def test_version_ordering(a, b, eq, gt):
    c = ver.compare(ver.parse(a), ver.parse(b))
    assert (c == 0) == eq and (c > 0) == gt


@pytest.mark.parametrize("bad", ["", "01.2", "1.x", "V1.0", "1.0.0-", "1..0"])
def test_version_rejects(bad):
    with pytest.raises(ver.VersionError):
        ver.parse(bad)


@pytest.mark.parametrize("sup,model,op,want", [
    ("4.46.0", "4.46.0", None, True), ("4.47.0", "4.46.0", "GreaterThan", True),
    ("4.46.0", "4.46.0", "GreaterThan", False), ("4.46.0", "4.46.0", "GreaterThanOrEqual", True),
    ("4.46", "4.46.0", "GreaterThanOrEqual", False),           # precision must agree
    ("v4.47.0", "4.46.0", "GreaterThan", False),               # so must the major prefix
    ("4.47.0", "4.46.0-rc1", "GreaterThan", False),            # unofficial only matches Equal
    ("4.46.0-rc1", "4.46.0-rc1", "GreaterThan", True),
])
def test_version_satisfies(sup, model, op, want):
    assert ver.satisfies(sup, model, op) == want


# ------------------------------------------------------------------ runtime selection
def _rt(name, arch="LlamaForCausalLM", fmt="safetensors", fmt_ver="1.0.0", fw="transformers", fw_ver="4.46.0",
        op=None, size=("1B", "10B"), priority=1, auto=True, disabled=False, accel=None, kind="ClusterServingRuntime",
        ns=None):
    f = {"modelFormat": {"name": fmt, "version": fmt_ver}, "modelFramework": {"name": fw, "version": fw_ver},
         "modelArchitecture": arch, "autoSelect": auto, "priority": priority}
    if op:
        f["modelFramework"]["operator"] = op
    spec = {"supportedModelFormats": [f], "disabled": disabled}
    if size:
        spec["modelSizeRange"] = {"min": size[0], "max": size[1]}
    if accel:
        spec["acceleratorRequirements"] = {"acceleratorClasses": accel}
    meta = {"name": name, **({"namespace": ns} if ns else {})}
    return {"apiVersion": API, "kind": kind, "metadata": meta, "spec": spec}


def _model(arch="LlamaForCausalLM", size="8B", fw_ver="4.46.0", fmt="safetensors"):
    return V.BaseModelSpec.model_validate({
        "modelFormat": {"name": fmt, "version": "1.0.0"}, "modelFramework": {"name": "transformers", "version": fw_ver},
        "modelArchitecture": arch, "modelParameterSize": size, "storage": {"storageUri": "hf://x/y"}})


def _store(*objs):
    s = Store()
    for o in objs:
        s.create(o)
    return s


def test_parse_model_size():
    assert parse_model_size("8B") == 8e9 and parse_model_size("70.6B") == 70.6e9
    assert parse_model_size("500M") == 5e8 and parse_model_size("1.5T") == 1.5e12 and parse_model_size("x") == 0


def test_select_prefers_priority_then_namespace_then_size_fit():
    s = _store(_rt("wide", size=("1B", "100B")), _rt("snug", size=("7B", "9B")), _rt("hi", priority=3, size=("1B", "100B")))
    sel = RuntimeSelector(s)
    assert sel.select(_model(), None, "default").name == "hi"
    s.delete(API, "ClusterServingRuntime", "hi")
    assert sel.select(_model(), None, "default").name == "snug"  # closer size range wins ties
    s.create(_rt("ns-rt", kind="ServingRuntime", ns="default", size=("1B", "100B")))
    m = sel.select(_model(), None, "default")
    assert m.name == "ns-rt" and not m.is_cluster  # namespace-scoped runtimes come first


def test_incompatible_runtimes_are_excluded_with_reasons():
    s = _store(_rt("other-arch", arch="MixtralForCausalLM"), _rt("too-small", size=("1B", "3B")),
               _rt("disabled", disabled=True), _rt("manual-only", auto=False), _rt("old-fw", fw_ver="4.40.0"))
    sel = RuntimeSelector(s)
    with pytest.raises(NoRuntimeFoundError) as e:
        sel.select(_model(), None, "default")
    msg = str(e.value)
    assert "other-arch" in msg and "too-small" in msg
    # explicit runtime: validated, not scored
    with pytest.raises(RuntimeDisabledError):
        sel.validate("disabled", _model(), None, "default")
    with pytest.raises(RuntimeCompatibilityError):
        sel.validate("too-small", _model(), None, "default")
    with pytest.raises(RuntimeNotFoundError):
        sel.validate("nope", _model(), None, "default")
    assert sel.validate("manual-only", _model(), None, "default") is not None  # autoSelect only gates auto pick
    with pytest.raises(ModelValidationError):
        sel.select(V.BaseModelSpec.model_validate({"storage": {"storageUri": "hf://x"}}), None, "default")


def test_framework_version_operator():
    s = _store(_rt("ge", fw_ver="4.46.0", op="GreaterThanOrEqual"))
    sel = RuntimeSelector(s)
    assert sel.select(_model(fw_ver="4.45.1"), None, "default").name == "ge"
    with pytest.raises(NoRuntimeFoundError):
        sel.select(_model(fw_ver="4.47.0"), None, "default")


def test_accelerator_class_requirement_filters_runtimes():
    s = _store(_rt("nv", accel=["nvidia-h100"]), _rt("amd", accel=["amd-mi355x", "amd-mi300x"]))
    isvc = {"spec": {"acceleratorSelector": {"acceleratorClass": "amd-mi355x"}}}
    assert RuntimeSelector(s).select(_model(), isvc, "default").name == "amd"


# ------------------------------------------------------------------ accelerator classes
def _ac(name, mem, fp16=None, int8=None, bw=None, cost=None, family="cdna4", vendor="amd", features=None, cc=None):
    caps = {"memoryGB": mem, "features": features or []}
    perf = {k: v for k, v in (("fp16Tflops", fp16), ("int8Tops", int8)) if v is not None}
    if perf:
        caps["performance"] = perf
    if bw:
        caps["memoryBandwidthGBps"] = bw
    if cc:
        caps["computeCapability"] = cc
    spec = {"vendor": vendor, "family": family, "capabilities": caps}
    if cost:
        spec["cost"] = cost
    return {"apiVersion": API, "kind": "AcceleratorClass", "metadata": {"name": name}, "spec": spec}


MI355X = _ac("amd-mi355x", "288Gi", fp16=2500, int8=5000, bw="8000", cost={"perHour": "6.0"}, features=["fp8", "xgmi"])
MI300X = _ac("amd-mi300x", "192Gi", fp16=1300, int8=2600, bw="5300", cost={"perHour": "4.0"}, family="cdna3",
             features=["fp8", "xgmi"])
SMALL = _ac("small", "48Gi", fp16=360, bw="864", cost={"spotPerHour": "1.0"}, family="ada", vendor="nvidia")


def _sel_store():
    return _store(MI355X, MI300X, SMALL)


def _rt_spec(classes):
    return V.ServingRuntimeSpec.model_validate({"acceleratorRequirements": {"acceleratorClasses": classes}})


@pytest.mark.parametrize("policy,constraints,want", [
    ("FirstAvailable", None, "amd-mi300x"),
    ("MostCapable", None, "amd-mi355x"),
    ("Cheapest", None, "small"),
    ("BestFit", {"minMemory": 150}, "amd-mi300x"),            # tightest memory fit
    ("BestFit", {"minMemory": 200}, "amd-mi355x"),
    ("Cheapest", {"minMemory": 100}, "amd-mi300x"),
    ("MostCapable", {"architectureFamilies": ["cdna3"]}, "amd-mi300x"),
    ("Cheapest", {"requiredFeatures": ["xgmi"], "excludedClasses": ["amd-mi300x"]}, "amd-mi355x"),
])
def test_accelerator_policies(policy, constraints, want):
    sel = A.AcceleratorClassSelector(_sel_store())
    sel_spec = {"policy": policy, **({"constraints": constraints} if constraints else {})}
    isvc = {"spec": {"acceleratorSelector": sel_spec}}
    ac, name = sel.get_accelerator_class(isvc, _rt_spec(["amd-mi300x", "amd-mi355x", "small"]), "engine")
    assert name == want and ac["metadata"]["name"] == want


def test_accelerator_explicit_and_component_override():
    sel = A.AcceleratorClassSelector(_sel_store())
    rt = _rt_spec(["amd-mi300x", "amd-mi355x"])
    isvc = {"spec": {"acceleratorSelector": {"acceleratorClass": "amd-mi300x"},
                     "engine": {"acceleratorOverride": {"acceleratorClass": "amd-mi355x"}}}}
    assert sel.get_accelerator_class(isvc, rt, "engine")[1] == "amd-mi355x"
    assert sel.get_accelerator_class(isvc, rt, "decoder")[1] == "amd-mi300x"
    # runtime without accelerator requirements: no class
    assert sel.get_accelerator_class(isvc, V.ServingRuntimeSpec(), "engine") == (None, "")
    with pytest.raises(LookupError):
        sel.get_accelerator_class({"spec": {"acceleratorSelector": {"acceleratorClass": "ghost"}}}, rt, "engine")


def test_requirement_checks():
    c = V.AcceleratorConstraints.model_validate({"minMemory": 200, "architectureFamilies": ["amd-cdna4"],
                                                 "requiredFeatures": ["FP8"]})
    assert A.meets_requirements(MI355X, c) == (True, "")
    ok, why = A.meets_requirements(MI300X, c)
    assert not ok and "family" in why
    assert A.memory_fit_score(MI355X, V.AcceleratorConstraints(min_memory=144)) == pytest.approx(0.5)
    assert A.compute_score(MI355X, V.AcceleratorConstraints(preferred_precisions=["fp4", "int8"],
                                                            min_compute_performance_tflops=2500)) == pytest.approx(0.5)

"""Table-driven policy cases ported (behaviour, not code) from the reference's Go tests:

* version operators: ``pkg/runtimeselector/matcher_test.go`` TestCompareModelFormatVersions /
  TestCompareModelFrameworkVersions (supported OP model semantics, unofficial versions only match
  Equal, precision and ``v`` major-prefix must agree);
* model size parsing / ranges: ``matcher_test.go`` (boundaries, nil sizes);
* accelerator scoring: ``pkg/acceleratorclassselector/policy_helpers_test.go``
  (TestScoreFromTFLOPS, TestGetTFLOPSForPrecision, TestGetMaxTFLOPS, TestCalculateMemoryFitScore,
  TestCalculateComputePerformanceTFLOPSScore, TestCalculateBestFitScore, TestGetCandidateCost,
  TestMeetsRequirements)."""
import pytest

from ome_amd.api import v1beta1 as V
from ome_amd.policy import accelerator_selector as A
from ome_amd.policy import runtime_selector as R
from ome_amd.policy import version as ver

# ---------------------------------------------------------------- versions
VERSION_CASES = [
    ("Equal versions with Equal operator", "1.0.0", "Equal", "1.0.0", True),
    ("Equal versions with GreaterThan operator", "1.0.0", "GreaterThan", "1.0.0", False),
    ("GreaterThan - supported version is greater", "1.8.0", "GreaterThan", "1.7.0", True),
    ("GreaterThan - supported version is not greater", "1.7.0", "GreaterThan", "1.8.0", False),
    ("GreaterThanOrEqual - equal versions", "1.8.0", "GreaterThanOrEqual", "1.8.0", True),
    ("GreaterThanOrEqual - supported version is greater", "1.9.0", "GreaterThanOrEqual", "1.8.0", True),
    ("GreaterThanOrEqual - supported version is less", "1.7.0", "GreaterThanOrEqual", "1.8.0", False),
    ("Unofficial version forces equality check", "1.8.0-dev", "GreaterThan", "1.8.0-dev", True),
    ("Unofficial version not equal", "1.8.0-dev", "GreaterThan", "1.8.0-alpha", False),
    ("Equal versions with precision 1", "1", None, "1", True),
    ("Precision mismatch", "1.0", "GreaterThan", "1.0.0", False),
    ("Major prefix mismatch", "v1.0.0", "GreaterThan", "1.0.0", False),
    ("Nil operator defaults to Equal", "v2.0.0", None, "v2.0.0", True),
    ("GreaterThan across minor", "2.1", "GreaterThan", "2.0", True),
    ("GreaterThan across major with prefix", "v3.0.0", "GreaterThan", "v2.9.9", True),
    ("Build metadata is unofficial", "1.0.0+b1", "GreaterThanOrEqual", "1.0.0+b1", True),
    ("Leading zero is invalid", "01.0.0", "Equal", "01.0.0", False),
    ("Uppercase V prefix is invalid", "V1.0.0", "Equal", "V1.0.0", False),
]


@pytest.mark.parametrize("name,supported,op,model,want", VERSION_CASES, ids=[c[0] for c in VERSION_CASES])
def test_version_operator_table(name, supported, op, model, want):
    assert ver.satisfies(supported, model, op) is want


@pytest.mark.parametrize("name,supported,op,model,want", VERSION_CASES, ids=[c[0] for c in VERSION_CASES])
def test_format_and_framework_version_matching(name, supported, op, model, want):
    """The same table through the format / framework matchers of the runtime selector."""
    base = V.BaseModelSpec.model_validate({"modelFormat": {"name": "safetensors", "version": model},
                                           "modelFramework": {"name": "transformers", "version": "4.0"}})
    f = V.SupportedModelFormat.model_validate({"modelFormat": {"name": "safetensors", "version": supported,
                                                               "operator": op},
                                               "modelFramework": {"name": "transformers", "version": "4.0"},
                                               "autoSelect": True})
    assert (not R.format_mismatch(base, f)) is want
    fw = V.BaseModelSpec.model_validate({"modelFormat": {"name": "safetensors", "version": "1"},
                                         "modelFramework": {"name": "transformers", "version": model}})
    ff = V.SupportedModelFormat.model_validate({"modelFormat": {"name": "safetensors", "version": "1"},
                                                "modelFramework": {"name": "transformers", "version": supported,
                                                                   "operator": op}, "autoSelect": True})
    assert (not R.format_mismatch(fw, ff)) is want


# ---------------------------------------------------------------- sizes / compatibility
SIZE_CASES = [
    ("8B", 8e9), ("70B", 70e9), ("1.5B", 1.5e9), ("405B", 405e9), ("1T", 1e12), ("125M", 125e6), ("7K", 7e3),
    ("", 0.0), (None, 0.0), ("abc", 0.0), ("12", 12.0),
]


@pytest.mark.parametrize("s,want", SIZE_CASES)
def test_parse_model_size(s, want):
    assert R.parse_model_size(s) == want


def _rt(min_s=None, max_s=None, fmt="safetensors", arch=None, quant=None, disabled=False, auto=True):
    spec = {"supportedModelFormats": [{"modelFormat": {"name": fmt}, "autoSelect": auto,
                                       **({"modelArchitecture": arch} if arch else {}),
                                       **({"quantization": quant} if quant else {})}],
            "disabled": disabled}
    if min_s or max_s:
        spec["modelSizeRange"] = {"min": min_s, "max": max_s}
    return V.ServingRuntimeSpec.model_validate(spec)


def _model(size="8B", fmt="safetensors", arch=None, quant=None):
    d = {"modelFormat": {"name": fmt}}
    if size is not None:
        d["modelParameterSize"] = size
    if arch:
        d["modelArchitecture"] = arch
    if quant:
        d["quantization"] = quant
    return V.BaseModelSpec.model_validate(d)


COMPAT_CASES = [
    ("supported model format", _rt(), _model(), True),
    ("unsupported model format", _rt(fmt="onnx"), _model(), False),
    ("model size out of range", _rt("1B", "7B"), _model("8B"), False),
    ("model size at minimum boundary", _rt("8B", "70B"), _model("8B"), True),
    ("model size at maximum boundary", _rt("1B", "8B"), _model("8B"), True),
    ("model with nil parameter size", _rt("1B", "7B"), _model(None), True),
    ("runtime with nil size range", _rt(), _model("405B"), True),
    ("architecture and quantization match", _rt(arch="LlamaForCausalLM", quant="fp8"),
     _model(arch="LlamaForCausalLM", quant="fp8"), True),
    ("architecture mismatch", _rt(arch="MistralForCausalLM"), _model(arch="LlamaForCausalLM"), False),
    ("quantization mismatch", _rt(quant="int4"), _model(quant="fp8"), False),
    ("quantization required by runtime only", _rt(quant="fp8"), _model(), False),
    ("disabled runtime", _rt(disabled=True), _model(), False),
]


@pytest.mark.parametrize("name,rt,model,want", COMPAT_CASES, ids=[c[0] for c in COMPAT_CASES])
def test_runtime_compatibility_table(name, rt, model, want):
    ok, reasons = R.compatibility(rt, model, None)
    assert ok is want
    assert bool(reasons) is (not want)


# ---------------------------------------------------------------- accelerator scoring
@pytest.mark.parametrize("tf,req,want", [(0, 100, 0.0), (100, 0, 1.0), (100, 100, 1.0), (200, 100, 1.0),
                                         (50, 100, 0.5), (25, 100, 0.25), (95, 100, 0.95)])
def test_score_from_tflops(tf, req, want):
    assert A._tflops_score(tf, req) == pytest.approx(want)


PERF = V.AcceleratorPerformance.model_validate({"fp32Tflops": 100, "fp16Tflops": 200, "int8Tops": 400,
                                                "int4Tops": 800})


@pytest.mark.parametrize("perf,prec,want", [(PERF, "fp32", 100), (PERF, "fp16", 200), (PERF, "int8", 400),
                                            (PERF, "fp8", 400), (PERF, "int4", 800), (PERF, "FP16", 200),
                                            (None, "fp16", 0),
                                            (V.AcceleratorPerformance.model_validate({"fp32Tflops": 100}), "fp16", 0),
                                            (PERF, "unknown", 0)])
def test_tflops_for_precision(perf, prec, want):
    assert A.tflops_for(perf, prec) == want


@pytest.mark.parametrize("perf,want", [
    ({"fp32Tflops": 100, "fp16Tflops": 200, "int8Tops": 400, "int4Tops": 800}, 800),
    ({"fp32Tflops": 500, "fp16Tflops": 200}, 500), ({"fp16Tflops": 200}, 200), (None, 0), ({}, 0),
    ({"fp32Tflops": 0, "fp16Tflops": 0}, 0)])
def test_max_tflops(perf, want):
    assert A.max_tflops(None if perf is None else V.AcceleratorPerformance.model_validate(perf)) == want


def _ac(mem_gib=None, perf=None, cost=None, features=None, vendor=None, family=None, name="test-accelerator",
        bw=None):
    caps = {}
    if mem_gib is not None:
        caps["memoryGB"] = f"{mem_gib}Gi"
    if perf is not None:
        caps["performance"] = perf
    if features is not None:
        caps["features"] = features
    if bw is not None:
        caps["memoryBandwidthGBps"] = bw
    spec = {"capabilities": caps}
    if cost is not None:
        spec["cost"] = cost
    if vendor:
        spec["vendor"] = vendor
    if family:
        spec["family"] = family
    return {"metadata": {"name": name}, "spec": spec}


def _cons(**kw):
    return V.AcceleratorConstraints.model_validate(kw)


@pytest.mark.parametrize("have,need,want", [(40, None, 1.0), (40, 40, 1.0), (80, 40, 0.5), (400, 40, 0.1),
                                            (160, 40, 0.25), (50, 40, 0.8)])
def test_memory_fit_score(have, need, want):
    assert A.memory_fit_score(_ac(have), _cons(minMemory=need)) == pytest.approx(want, abs=0.01)


COMPUTE_CASES = [
    ("No requirement - perfect score", {"fp16Tflops": 100}, None, ["fp16"], 1.0),
    ("First precision exact match", {"fp16Tflops": 100}, 100, ["fp16"], 1.0),
    ("First precision exceeds requirement", {"fp16Tflops": 200}, 100, ["fp16"], 1.0),
    ("First precision half of requirement", {"fp16Tflops": 50}, 100, ["fp16"], 0.5),
    ("Second precision fallback with penalty", {"fp16Tflops": 100}, 100, ["fp8", "fp16"], 0.5),
    ("Third precision fallback with penalty", {"fp16Tflops": 100}, 100, ["int4", "int8", "fp16"], 0.25),
    ("No preferred precisions - use max", {"fp32Tflops": 50, "fp16Tflops": 100, "int8Tops": 200}, 200, [], 1.0),
    ("No precision has TFLOPS data", {}, 100, ["fp16"], 0.0),
    ("Nil performance struct", None, 100, ["fp16"], 0.0),
]


@pytest.mark.parametrize("name,perf,req,prefs,want", COMPUTE_CASES, ids=[c[0] for c in COMPUTE_CASES])
def test_compute_performance_score(name, perf, req, prefs, want):
    c = _cons(minComputePerformanceTFLOPS=req, preferredPrecisions=prefs)
    assert A.compute_score(_ac(perf=perf), c) == pytest.approx(want, abs=0.01)


@pytest.mark.parametrize("mem,tf,need,prefs,want", [(40, 100, 40, ["fp16"], 1.0), (80, 100, 40, ["fp16"], 0.65),
                                                    (40, 100, 40, ["fp8", "fp16"], 0.85)])
def test_best_fit_score(mem, tf, need, prefs, want):
    ac = _ac(mem, {"fp16Tflops": tf})
    assert A.best_fit_score(ac, _cons(minMemory=need, preferredPrecisions=prefs)) == pytest.approx(want, abs=0.02)


@pytest.mark.parametrize("cost,want", [({"spotPerHour": "1", "perHour": "2", "perMillionTokens": "3"}, "spot-hourly"),
                                       ({"perHour": "2", "perMillionTokens": "3"}, "hourly"),
                                       ({"perMillionTokens": "3"}, "per-million-tokens"), ({"tier": "low"}, "tier"),
                                       (None, None), ({}, None)])
def test_candidate_cost(cost, want):
    got = A.candidate_cost(_ac(cost=cost))
    assert (got[1] if got else None) == want


MEETS_CASES = [
    ("No constraints - always eligible", _ac(), None, True, ""),
    ("Explicitly excluded", _ac(name="excluded-gpu"), _cons(excludedClasses=["excluded-gpu", "other-gpu"]), False,
     "explicitly excluded"),
    ("Below MinMemory", _ac(16), _cons(minMemory=32), False, "memory 16GB < required 32GB"),
    ("Meets MinMemory", _ac(40), _cons(minMemory=32), True, ""),
    ("Exceeds MaxMemory", _ac(80), _cons(maxMemory=64), False, "memory 80GB > max allowed 64GB"),
    ("Missing required feature", _ac(features=["cuda", "tensor-cores"]), _cons(requiredFeatures=["nvlink"]), False,
     "missing required feature: nvlink"),
    ("Has all required features", _ac(features=["cuda", "tensor-cores", "nvlink"]),
     _cons(requiredFeatures=["tensor-cores", "nvlink"]), True, ""),
    ("Architecture family mismatch", _ac(vendor="AMD", family="RDNA"),
     _cons(architectureFamilies=["nvidia-ampere", "nvidia-hopper"]), False,
     "architecture family rdna not in allowed list"),
    ("Architecture family match", _ac(vendor="NVIDIA", family="Ampere"),
     _cons(architectureFamilies=["nvidia-ampere", "nvidia-hopper"]), True, ""),
    ("CDNA4 family match (MI355X)", _ac(vendor="AMD", family="CDNA4"), _cons(architectureFamilies=["amd-cdna4"]),
     True, ""),
    ("Missing memory specification when MinMemory required", _ac(), _cons(minMemory=40), False,
     "missing memory specification for memory check"),
    ("MinComputePerformanceTFLOPS not a hard filter (soft constraint)", _ac(),
     _cons(minComputePerformanceTFLOPS=1000), True, ""),
]


@pytest.mark.parametrize("name,ac,c,want,reason", MEETS_CASES, ids=[m[0] for m in MEETS_CASES])
def test_meets_requirements(name, ac, c, want, reason):
    ok, why = A.meets_requirements(ac, c)
    assert ok is want
    if not want:
        assert why == reason


def test_capability_scores_nonzero_and_normalised():
    cands = [_ac(288, {"fp16Tflops": 2500}, bw="8000", name="mi355x"), _ac(192, {"fp16Tflops": 1300}, bw="5300",
                                                                           name="mi300x"),
             _ac(80, None, bw="2000", name="nodata")]
    s = A.capability_scores(cands, ["fp16"])
    assert s[0] == pytest.approx(1.0) and 0 < s[1] < s[0] and s[2] > 0   # memory fallback keeps it non-zero

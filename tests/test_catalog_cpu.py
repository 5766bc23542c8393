"""Generated MI355X model/runtime catalog (``ome_amd/catalog.py``, checked in under
``config/runtimes/ome-amd`` and ``config/models/<vendor>``): every runtime parses into the v1beta1
types with no unknown fields, serves an architecture the first-party runtime implements, passes
the runtime server's own flag parser, sizes tensor parallelism for 288 GB HBM, and is what the
RuntimeSelector auto-picks for its base model."""
from pathlib import Path

import pytest

from ome_amd import catalog
from ome_amd.api import v1beta1 as V
from ome_amd.models import supported
from ome_amd.policy.runtime_selector import RuntimeSelector
from ome_amd.runtime.server import build_parser
from ome_amd.store.store import Store

ROOT = Path(__file__).resolve().parent.parent


def _all_runtimes():
    rts, _ = catalog.generate()
    return [d for docs in rts.values() for d in docs]


def _containers(spec: dict):
    e = spec["engineConfig"]
    for part in (e.get("runner"), (e.get("leader") or {}).get("runner"), (e.get("worker") or {}).get("runner"),
                 (spec.get("decoderConfig") or {}).get("runner")):
        if part:
            yield part


def test_checked_in_catalog_is_current(tmp_path):
    catalog.write(tmp_path)
    for p in sorted(tmp_path.rglob("*.yaml")):
        rel = p.relative_to(tmp_path)
        assert (ROOT / "config" / rel).read_text() == p.read_text(), f"regenerate config/{rel}"


@pytest.mark.parametrize("rt", _all_runtimes(), ids=lambda r: r["metadata"]["name"])
def test_runtime_entry(rt):
    spec = V.ServingRuntimeSpec.model_validate(rt["spec"])
    assert not spec.model_extra and not spec.engine_config.model_extra
    fmt = spec.supported_model_formats[0]
    assert supported(fmt.model_architecture), fmt.model_architecture
    for c in _containers(rt["spec"]):
        args = [a.replace("$(MODEL_PATH)", "/m").replace("$(LWS_LEADER_ADDRESS)", "10.0.0.1")
                .replace("$(LWS_WORKER_INDEX)", "1") for a in c["args"]]
        if "ome_amd.diffusion.server" in c["command"]:
            from ome_amd.diffusion.server import build_parser as diffusion_parser

            ns = diffusion_parser().parse_args(args)
            assert ns.tp_size == 1 and c["resources"]["limits"]["amd.com/gpu"] == 1
            continue
        ns = build_parser().parse_args(args)
        gpus = c["resources"]["limits"]["amd.com/gpu"]
        assert ns.tp_size in (gpus, gpus * getattr(ns, "nnodes", 1))


def test_tp_sizing_for_288gb():
    by = {f.name: catalog.tp_for(f) for f in catalog.FAMILIES}
    assert by["llama-3-70b-instruct"] == 1          # 141 GB bf16 on one MI355X
    assert by["llama-4-scout-17b-16e-instruct"] == 2
    assert by["deepseek-v3"] == 8 and by["llama-3-1-405b-instruct-fp8"] == 4


def test_selector_picks_catalog_runtime_for_each_base_model():
    rts, models = catalog.generate()
    s = Store()
    for docs in rts.values():
        for d in docs:
            s.create(d)
    sel = RuntimeSelector(s)
    for docs in models.values():
        for m in docs:
            spec = V.BaseModelSpec.model_validate(m["spec"])
            f = next(f for f in catalog.FAMILIES if f.name == m["metadata"]["name"])
            if catalog._pooled_twin(f):
                # embedding / reward checkpoint of a generative architecture: its pooling runtime is
                # opt-in (validated for the model by name), and the catalog's ISVC sample names it
                own = f"ome-amd-{f.name}-tp{catalog.tp_for(f)}"
                assert catalog.isvc_samples(f)[f.name]["spec"]["runtime"]["name"] == own
                sel.validate(own, spec, None, "default")
                continue
            got = sel.select(spec, None, "default").name
            if not f.runtime:
                # model-only entry: served by a runtime family of the same architecture / quantisation
                # whose size class covers it
                hosts = {f"ome-amd-{g.name}-tp{catalog.tp_for(g)}" for g in catalog.FAMILIES
                         if g.runtime and catalog._covers(g, f)}
                assert got in hosts, (m["metadata"]["name"], got)
                continue
            # the family's own single-pod runtime, or an interchangeable one (same architecture, size
            # class and parallelism: e.g. Llama-3 / Llama-3.1 8B)
            twins = {f"ome-amd-{g.name}-tp{catalog.tp_for(g)}" for g in catalog.FAMILIES
                     if g.runtime and g.arch == f.arch and g.quantization == f.quantization
                     and catalog.tp_for(g) == catalog.tp_for(f) and abs(g.params_b - f.params_b) / f.params_b < 0.16}
            assert got in twins, (m["metadata"]["name"], got)

"""Deployment packaging (reference H5-H7: charts/, config/default kustomize, dockerfiles/): the
CRD chart carries exactly the generated CRDs, kustomize overlays reference existing files, every
static manifest parses, and the image entrypoints exist as modules."""
import glob
import importlib.util
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_crd_chart_matches_generated_crds():
    chart = sorted(os.path.basename(p) for p in glob.glob(f"{ROOT}/charts/ome-amd-crd/templates/*.yaml"))
    gen = sorted(os.path.basename(p) for p in glob.glob(f"{ROOT}/config/crd/ome.io_*.yaml"))
    assert chart == gen and len(gen) == 8
    for n in gen:
        assert open(f"{ROOT}/charts/ome-amd-crd/templates/{n}").read() == open(f"{ROOT}/config/crd/{n}").read()


def test_kustomizations_reference_existing_files():
    for k in glob.glob(f"{ROOT}/config/**/kustomization.yaml", recursive=True):
        d = os.path.dirname(k)
        doc = yaml.safe_load(open(k))
        for r in doc.get("resources", []):
            assert os.path.exists(os.path.join(d, r)), (k, r)
        for g in doc.get("configMapGenerator", []):
            for f in g.get("files", []):
                assert os.path.exists(os.path.join(d, f)), (k, f)


def test_static_manifests_parse():
    for f in glob.glob(f"{ROOT}/config/**/*.yaml", recursive=True):
        list(yaml.safe_load_all(open(f)))
    for chart in glob.glob(f"{ROOT}/charts/*/"):
        meta = yaml.safe_load(open(os.path.join(chart, "Chart.yaml")))
        assert meta["apiVersion"] == "v2" and meta["name"] == os.path.basename(chart.rstrip("/"))
        yaml.safe_load(open(os.path.join(chart, "values.yaml")))


def test_image_entrypoints_exist():
    for mod in ("ome_amd.manager", "ome_amd.cli", "ome_amd.agent", "ome_amd.prober", "ome_amd.metrics_aggregator",
                "ome_amd.runtime.server", "ome_amd.router", "ome_amd.build"):
        assert importlib.util.find_spec(mod) is not None, mod

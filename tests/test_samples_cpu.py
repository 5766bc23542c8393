"""Every generated sample (config/samples) passes admission against the generated catalog:
each InferenceService resolves its model and runtime, each BenchmarkJob's scenarios and task
validate (the reference ships 147 ISVC + 4 BenchmarkJob samples, ``config/samples/**``)."""
import os
import sys
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def test_samples_admit_against_catalog(tmp_path):
    from ome_amd.manager import Cluster

    cl = Cluster(str(tmp_path / "state"), simulate=True, with_agent=False, with_executor=False)
    try:
        for d in ("config/acceleratorclasses", "config/runtimes/ome-amd", "config/models"):
            cl.load_catalog(str(ROOT / d))
        isvcs = sorted((ROOT / "config/samples/isvc").rglob("*.yaml"))
        assert len(isvcs) >= 85
        for p in isvcs:
            for doc in yaml.safe_load_all(p.read_text()):
                ns = doc["metadata"]["namespace"]
                cl.apply([{"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}}])
                out = cl.apply([doc])[0]
                if "runtime" in doc["spec"]:
                    assert out["spec"]["runtime"]["name"] == doc["spec"]["runtime"]["name"], p
        for p in sorted((ROOT / "config/samples/benchmark").glob("*.yaml")):
            for doc in yaml.safe_load_all(p.read_text()):
                ns = doc["metadata"]["namespace"]
                cl.apply([{"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}}])
                cl.apply([doc])
    finally:
        cl.shutdown()

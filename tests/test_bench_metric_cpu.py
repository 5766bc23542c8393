"""bench.py's JSON carries BASELINE.json's metric string only for the headline config
(verdict r05, weak item 13: the DeepSeek exploration JSON carried the Llama-3-8B metric)."""
import argparse
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_metric_string_is_the_baseline_one_only_for_the_headline():
    b = _bench()
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    ns = lambda **kw: argparse.Namespace(**{"model": "llama-3-8b", "layers": None, "quantization": None,
                                             "kv_cache_dtype": "auto", **kw})
    assert b._metric(ns()) == base
    for kw in ({"model": "deepseek-v3"}, {"layers": 4}, {"quantization": "fp8"}, {"kv_cache_dtype": "fp8_e4m3"}):
        m = b._metric(ns(**kw))
        assert m != base and "not the headline" in m, (kw, m)
    assert "deepseek-v3" in b._metric(ns(model="deepseek-v3"))

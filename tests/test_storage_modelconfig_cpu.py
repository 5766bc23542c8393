"""Storage-URI grammar (``pkg/utils/storage/storage.go``; valid / invalid cases of its
``storage_test.go``) and HF config introspection over the reference's golden ``config.json``
fixtures (``pkg/hfutil/modelconfig/testdata``)."""
import os

import pytest

from ome_amd.io.safetensors import count_params_in_dir
from ome_amd.modelagent import modelconfig as mc
from ome_amd.storage import uri as U

FIX = "/root/reference/pkg/hfutil/modelconfig/testdata"


@pytest.mark.parametrize("uri,typ,parts", [
    ("oci://n/myns/b/mybucket/o/mypath", "OCI", {"namespace": "myns", "bucket": "mybucket", "prefix": "mypath"}),
    ("oci://n/myns/b/mybucket/o/path/to/my/object", "OCI", {"prefix": "path/to/my/object"}),
    ("oci://n/my-ns.123/b/my_bucket-123/o/path.with.dots/and-dashes", "OCI", {"bucket": "my_bucket-123"}),
    ("pvc://my-pvc/results", "PVC", {"namespace": "", "pvc": "my-pvc", "subpath": "results"}),
    ("pvc://my-namespace:my-pvc/path/to/results", "PVC", {"namespace": "my-namespace", "subpath": "path/to/results"}),
    ("pvc://model-storage:shared-pvc/path/to/models/llama2-7b", "PVC", {"pvc": "shared-pvc"}),
    ("hf://meta-llama/Meta-Llama-3-8B-Instruct", "HUGGINGFACE", {"model_id": "meta-llama/Meta-Llama-3-8B-Instruct",
                                                                "branch": "main"}),
    ("hf://org/model@v2", "HUGGINGFACE", {"branch": "v2"}),
    ("s3://bucket@us-east-1/prefix/x", "S3", {"bucket": "bucket", "region": "us-east-1", "prefix": "prefix/x"}),
    ("s3://bucket/prefix", "S3", {"region": "", "prefix": "prefix"}),
    ("az://acct.blob.core.windows.net/cont/a/b", "AZURE", {"account": "acct", "container": "cont", "blob_path": "a/b"}),
    ("az://acct/cont", "AZURE", {"blob_path": ""}),
    ("gs://bucket/obj/path", "GCS", {"bucket": "bucket", "object": "obj/path"}),
    ("github://owner/repo@v1.2", "GITHUB", {"owner": "owner", "repository": "repo", "tag": "v1.2"}),
    ("vendor://nvidia/models/llama", "VENDOR", {"vendor": "nvidia", "resource_type": "models"}),
    ("local:///raid/models/x", "LOCAL", {"path": "/raid/models/x"}),
    ("random://llama-3-8b?layers=2", "RANDOM", {"preset": "llama-3-8b", "layers": "2"}),
])
def test_uri_parse(uri, typ, parts):
    u = U.parse(uri)
    assert u.type == typ
    for k, v in parts.items():
        assert u.parts[k] == v, k


@pytest.mark.parametrize("uri", [
    "n/myns/b/mybucket/o/mypath", "oci://myns/b/mybucket/o/mypath", "oci://n/myns/mybucket/o/mypath",
    "oci://n/myns/b/mybucket/mypath", "", "oci://", "oci://n/myns/b/mybucket/o", "oci://b/mybucket/n/myns/o/mypath",
    "invalid://uri", "pvc://MyNamespace:my-pvc/models", "pvc://my_namespace:my-pvc/models",
    "pvc://-namespace:my-pvc/models", "pvc://namespace-:my-pvc/models",
    "pvc://a123456789012345678901234567890123456789012345678901234567890123:my-pvc/models", "pvc://:my-pvc/models",
    "pvc://default:/models", "my-pvc/results", "pvc://", "pvc:///results", "pvc://my-pvc/", "pvc://default:my-pvc/",
    "pvc://my-pvc", "pvc://default:my-pvc", "hf://", "s3://", "gs://", "github://owner", "vendor://a/b",
])
def test_uri_rejects(uri):
    with pytest.raises(U.StorageURIError):
        U.parse(uri)


# ------------------------------------------------------------------ model config introspection
# published parameter counts (model cards) — the reference returns rounded nominal values from a
# lookup table when no safetensors are present; we compute exact counts from the config.
PUBLISHED = {
    "llama3.json": (70.55e9, "llama"), "llama3_1_405b.json": (405.85e9, "llama"), "llama3_2_1b.json": (1.24e9, "llama"),
    "llama3_2_3b.json": (3.21e9, "llama"), "mixtral.json": (46.70e9, "mixtral"),
    "deepseek_v3.json": (671.0e9, "deepseek_v3"), "qwen2.5_7b.json": (7.62e9, "qwen2"),
    "qwen2.5_72b.json": (72.71e9, "qwen2"), "qwen3_30b.json": (30.53e9, "qwen3_moe"),
    "gpt_oss_120b.json": (116.83e9, "gpt_oss"), "gpt_oss_20b.json": (20.91e9, "gpt_oss"),
    "mistral_7b_instruct.json": (7.24e9, "mistral"), "gemma_2_9b.json": (9.24e9, "gemma2"),
    "kimi_k2_instruct.json": (1.03e12, "kimi_k2"), "phi3.json": (3.82e9, "phi3"),
}


@pytest.mark.skipif(not os.path.isdir(FIX), reason="reference fixtures not present")
@pytest.mark.parametrize("name", sorted(PUBLISHED))
def test_param_counts_match_published(name):
    want, mt = PUBLISHED[name]
    info = mc.load_model_config(os.path.join(FIX, name))
    assert info.model_type == mt
    assert abs(info.param_count - want) / want < 0.01, (info.param_count, want)
    assert info.context_length > 0 and info.size_bytes > 0


@pytest.mark.skipif(not os.path.isdir(FIX), reason="reference fixtures not present")
def test_every_fixture_parses_with_capabilities():
    names = sorted(f for f in os.listdir(FIX) if f.endswith(".json"))
    caps = {}
    for n in names:
        info = mc.load_model_config(os.path.join(FIX, n))
        caps[n] = mc.capabilities(info)
        md = mc.model_metadata(info)
        assert md["modelFormat"]["name"] == "safetensors"
    assert caps["llama3_2_11b_vision.json"] == ["IMAGE_TEXT_TO_TEXT"]
    assert caps["bge_large.json"] == ["EMBEDDING"] and caps["e5_mistral_7b.json"] == ["EMBEDDING"]
    assert caps["llama3.json"] == ["TEXT_TO_TEXT"] and caps["qwen2_vl_7b.json"] == ["IMAGE_TEXT_TO_TEXT"]
    assert mc.load_model_config(os.path.join(FIX, "qwen3_8b_fp8.json")).quantization == "fp8"


@pytest.mark.skipif(not os.path.isdir(FIX), reason="reference fixtures not present")
def test_safetensors_count_wins_over_config_estimate():
    d = os.path.join(FIX, "tiny-random-PhiModel")
    info = mc.load_model_config(d)
    assert info.param_count == count_params_in_dir(d) > 0
    assert mc.format_param_count(info.param_count).endswith("K")


def test_format_helpers():
    assert mc.format_param_count(8_030_261_248) == "8.03B"
    assert mc.format_param_count(494_032_768) == "494.03M"
    assert mc.format_param_count(1_026_000_000_000).endswith("T")

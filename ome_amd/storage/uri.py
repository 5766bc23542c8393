"""Storage URI grammar (``pkg/utils/storage/storage.go``) plus ``random://`` for synthetic weights.

  oci://n/{namespace}/b/{bucket}/o/{prefix}      pvc://[{ns}:]{pvc}/{subpath}
  hf://{org}/{model}[@{branch}]                  s3://{bucket}[@{region}]/{prefix}
  az://{account}/{container}/{path} | az://{account}.blob.core.windows.net/{container}/{path}
  gs://{bucket}/{object}                          github://{owner}/{repo}[@{tag}]
  vendor://{vendor}/{type}/{path}                 local://{path}
  random://{preset}[?layers=N]                    (MI355X-native addition: random-init weights of a
                                                   named architecture, the BASELINE benchmark rule)
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from urllib.parse import parse_qs


class StorageURIError(ValueError):
    pass


PREFIXES = {
    "oci://": "OCI", "pvc://": "PVC", "vendor://": "VENDOR", "hf://": "HUGGINGFACE", "s3://": "S3",
    "az://": "AZURE", "gs://": "GCS", "github://": "GITHUB", "local://": "LOCAL", "random://": "RANDOM",
}


def storage_type(uri: str) -> str:
    for p, t in PREFIXES.items():
        if uri.startswith(p):
            return t
    raise StorageURIError(f"unknown storage type for URI: {uri}")


@dataclass
class StorageURI:
    type: str
    raw: str
    parts: dict = field(default_factory=dict)


_NS_RE = re.compile(r"^[a-z0-9]([a-z0-9-]{0,61}[a-z0-9])?$")


def parse(uri: str) -> StorageURI:
    t = storage_type(uri)
    body = uri.split("://", 1)[1]
    if not body:
        raise StorageURIError(f"invalid {t} storage URI: missing content after prefix")
    p: dict = {}
    if t == "OCI":
        s = body.split("/")
        if len(s) < 6 or s[0] != "n" or s[2] != "b" or s[4] != "o":
            raise StorageURIError("invalid OCI storage URI format. Expected: oci://n/{namespace}/b/{bucket}/o/{object_path}")
        p = {"namespace": s[1], "bucket": s[3], "prefix": "/".join(s[5:])}
    elif t == "PVC":
        if "/" not in body:
            raise StorageURIError("invalid PVC storage URI format: missing subpath")
        first, sub = body.split("/", 1)
        ns = ""
        if ":" in first:
            ns, name = first.split(":", 1)
            if not ns or not name or ":" in name:
                raise StorageURIError("invalid PVC storage URI format: bad namespace:pvc-name")
            if not _NS_RE.match(ns):
                raise StorageURIError(f"invalid PVC storage URI format: invalid namespace {ns!r}")
        else:
            name = first
        if not name or not sub:
            raise StorageURIError("invalid PVC storage URI format: missing PVC name or subpath")
        p = {"namespace": ns, "pvc": name, "subpath": sub}
    elif t == "VENDOR":
        s = body.split("/", 2)
        if len(s) < 3 or not all(s):
            raise StorageURIError("invalid vendor storage URI format. Expected: vendor://{vendor}/{type}/{path}")
        p = {"vendor": s[0], "resource_type": s[1], "resource_path": s[2]}
    elif t == "HUGGINGFACE":
        model, _, branch = body.partition("@")
        if not model:
            raise StorageURIError("invalid Hugging Face storage URI format: model ID cannot be empty")
        p = {"model_id": model, "branch": branch or "main"}
    elif t == "S3":
        if "@" in body:
            bucket, rest = body.split("@", 1)
            region, _, prefix = rest.partition("/")
        else:
            bucket, _, prefix = body.partition("/")
            region = ""
        if not bucket:
            raise StorageURIError("invalid S3 storage URI format: bucket name cannot be empty")
        p = {"bucket": bucket, "prefix": prefix, "region": region}
    elif t == "AZURE":
        if ".blob.core.windows.net/" in body:
            acct, rest = body.split(".blob.core.windows.net/", 1)
            cont, _, path = rest.partition("/")
        else:
            s = body.split("/", 2)
            if len(s) < 2:
                raise StorageURIError("invalid Azure storage URI format: missing container name")
            acct, cont = s[0], s[1]
            path = s[2] if len(s) > 2 else ""
        if not acct or not cont:
            raise StorageURIError("invalid Azure storage URI format: account and container are required")
        p = {"account": acct, "container": cont, "blob_path": path}
    elif t == "GCS":
        bucket, _, obj = body.partition("/")
        if not bucket:
            raise StorageURIError("invalid GCS storage URI format: bucket name cannot be empty")
        p = {"bucket": bucket, "object": obj}
    elif t == "GITHUB":
        repo, _, tag = body.partition("@")
        s = repo.split("/", 1)
        if len(s) != 2 or not all(s):
            raise StorageURIError("invalid GitHub storage URI format: expected owner/repository")
        p = {"owner": s[0], "repository": s[1], "tag": tag or "latest"}
    elif t == "LOCAL":
        p = {"path": body}
    elif t == "RANDOM":
        name, _, q = body.partition("?")
        p = {"preset": name, **{k: v[0] for k, v in parse_qs(q).items()}}
    return StorageURI(t, uri, p)


def validate(uri: str) -> None:
    parse(uri)

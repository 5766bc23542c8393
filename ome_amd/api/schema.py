"""CRD / OpenAPI generation from the pydantic v1beta1 models (the reference generates
``config/crd/full/*.yaml`` with controller-gen from Go types, ``hack/`` + ``pkg/openapi``).

    python -m ome_amd.api.schema config/crd        # one CustomResourceDefinition per kind

Schemas are OpenAPI v3 as Kubernetes structural schemas require: ``$ref``s inlined, ``anyOf``
with ``null`` collapsed to ``nullable``, and ``x-kubernetes-preserve-unknown-fields`` on every
object (the models accept unknown fields, like the reference's ``runtime.RawExtension`` /
embedded PodSpec parts).
"""
from __future__ import annotations

import sys
from pathlib import Path

import yaml

from ome_amd.api import constants as C
from ome_amd.api.v1beta1 import KINDS, SHORT_NAMES

PRINTER_COLUMNS = {
    "InferenceService": [{"name": "URL", "type": "string", "jsonPath": ".status.url"},
                         {"name": "Ready", "type": "string", "jsonPath": ".status.conditions[?(@.type=='Ready')].status"},
                         {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"}],
    "BaseModel": [{"name": "Vendor", "type": "string", "jsonPath": ".spec.vendor"},
                  {"name": "Architecture", "type": "string", "jsonPath": ".spec.modelArchitecture"},
                  {"name": "Size", "type": "string", "jsonPath": ".spec.modelParameterSize"},
                  {"name": "State", "type": "string", "jsonPath": ".status.state"}],
    "BenchmarkJob": [{"name": "State", "type": "string", "jsonPath": ".status.state"},
                     {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"}],
}
PRINTER_COLUMNS["ClusterBaseModel"] = PRINTER_COLUMNS["BaseModel"]


def _inline(node, defs: dict, depth: int = 0):
    if depth > 40:
        return {"type": "object", "x-kubernetes-preserve-unknown-fields": True}
    if isinstance(node, list):
        return [_inline(x, defs, depth) for x in node]
    if not isinstance(node, dict):
        return node
    if "$ref" in node:
        target = defs[node["$ref"].split("/")[-1]]
        return _inline({**target, **{k: v for k, v in node.items() if k != "$ref"}}, defs, depth + 1)
    out = {}
    for k, v in node.items():
        if k in ("title", "$defs", "default", "examples"):
            continue
        out[k] = _inline(v, defs, depth)
    for key in ("anyOf", "oneOf"):
        alts = out.get(key)
        if alts:
            non_null = [a for a in alts if a.get("type") != "null"]
            nullable = len(non_null) != len(alts)
            if len(non_null) == 1:
                out.pop(key)
                out.update(non_null[0])
            elif all(set(a) <= {"type"} for a in non_null) and non_null:
                # scalar unions (e.g. int | str quantities): int-or-string in Kubernetes terms
                out.pop(key)
                out["x-kubernetes-int-or-string"] = True
            else:
                out.pop(key)
                out["x-kubernetes-preserve-unknown-fields"] = True
            if nullable:
                out["nullable"] = True
    if out.get("type") == "object" or "properties" in out:
        out["type"] = "object"
        out["x-kubernetes-preserve-unknown-fields"] = True
        ap = out.get("additionalProperties")
        if isinstance(ap, bool):
            out.pop("additionalProperties")
    return out


def spec_schema(model_cls) -> dict:
    js = model_cls.model_json_schema(by_alias=True)
    defs = js.get("$defs", {})
    return _inline(js, defs)


def crd(kind: str) -> dict:
    plural, namespaced, spec_cls = KINDS[kind]
    shorts = [s for s, k in SHORT_NAMES.items() if k == kind]
    version = {"name": C.VERSION, "served": True, "storage": True, "subresources": {"status": {}},
               "schema": {"openAPIV3Schema": {"type": "object", "properties": {
                   "apiVersion": {"type": "string"}, "kind": {"type": "string"},
                   "metadata": {"type": "object"}, "spec": spec_schema(spec_cls),
                   "status": {"type": "object", "x-kubernetes-preserve-unknown-fields": True}}}}}
    if kind in PRINTER_COLUMNS:
        version["additionalPrinterColumns"] = PRINTER_COLUMNS[kind]
    return {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
            "metadata": {"name": f"{plural}.{C.GROUP}"},
            "spec": {"group": C.GROUP, "scope": "Namespaced" if namespaced else "Cluster",
                     "names": {"kind": kind, "plural": plural, "singular": kind.lower(), "listKind": f"{kind}List",
                               **({"shortNames": shorts} if shorts else {})},
                     "versions": [version]}}


def write_all(out_dir: str | Path) -> list[Path]:
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    paths = []
    for kind in KINDS:
        p = out / f"{C.GROUP}_{KINDS[kind][0]}.yaml"
        p.write_text(yaml.safe_dump(crd(kind), sort_keys=False))
        paths.append(p)
    return paths


if __name__ == "__main__":
    for p in write_all(sys.argv[1] if len(sys.argv) > 1 else "config/crd"):
        print(p)

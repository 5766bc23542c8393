"""Swagger 2.0 document of the ``ome.io/v1beta1`` API (the reference's ``pkg/openapi/swagger.json``,
produced there by ``hack/update-openapigen.sh`` from the Go types, and the input of its
``hack/python-sdk/client-gen.sh``).

Here the source of truth is the pydantic models (:mod:`ome_amd.api.v1beta1` specs,
:mod:`ome_amd.api.objects` statuses and envelopes); definitions are named ``v1beta1.<Type>``
like the reference's, and ``paths`` describe the manager's Kubernetes-style REST routes
(``/apis/ome.io/v1beta1/[namespaces/{namespace}/]<plural>[/{name}[/status]]``) that
:mod:`ome_amd.sdk` calls.

    python -m ome_amd.api.openapi config/openapi/swagger.json
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

from ome_amd.api import constants as C
from ome_amd.api import objects as O
from ome_amd.api import v1beta1 as V

PREFIX = "v1beta1."
VERSION = "0.1"
_DROP = {"title", "discriminator"}


def _swaggerize(node):
    """JSON-schema (pydantic) -> Swagger 2.0 schema: ``anyOf [X, null]`` -> X, ``const`` -> enum,
    ``$defs`` refs already point at ``#/definitions/v1beta1.*``."""
    if isinstance(node, list):
        return [_swaggerize(x) for x in node]
    if not isinstance(node, dict):
        return node
    if "anyOf" in node:
        alts = [a for a in node["anyOf"] if a.get("type") != "null"]
        rest = {k: v for k, v in node.items() if k != "anyOf"}
        if len(alts) == 1:
            return _swaggerize({**alts[0], **{k: v for k, v in rest.items() if k in ("description", "default")}})
        # int | str (intstr) and other unions: Kubernetes' int-or-string convention
        if {a.get("type") for a in alts} <= {"integer", "string"}:
            return {"type": "string", "format": "int-or-string", **{k: v for k, v in rest.items() if k == "description"}}
        return {"type": "object", **{k: v for k, v in rest.items() if k == "description"}}
    out = {}
    for k, v in node.items():
        if k in _DROP:
            continue
        if k == "const":
            out["enum"] = [v]
            continue
        if k == "default" and v is None:
            continue
        out[k] = _swaggerize(v)
    return out


def definitions() -> dict:
    models = [*O.OBJECTS.values(), *O.LISTS.values(), V.ComponentExtensionSpec, O.AcceleratorSelection,
              O.ScalerAuthenticationRef, O.SupportedRuntime, O.ModelSpec, O.ModelExtensionSpec, O.PredictorExtensionSpec, O.PodSpec,
              O.ServingRuntimePodSpec, V.TensorParallelismConfig, V.AcceleratorModelConfig, V.AcceleratorConstraints,
              V.AcceleratorSelector, V.InferenceServiceReference, V.Endpoint, V.EndpointSpec, V.ServiceMetadata,
              V.PodOverride, V.HuggingFaceSecretReference]
    defs: dict = {}
    for m in models:
        sch = m.model_json_schema(by_alias=True, ref_template="#/definitions/" + PREFIX + "{model}", mode="serialization")
        for name, d in (sch.pop("$defs", None) or {}).items():
            defs.setdefault(PREFIX + name, _swaggerize(d))
        defs[PREFIX + m.__name__] = _swaggerize(sch)
    for k in list(defs):
        defs[k].setdefault("type", "object")
    return dict(sorted(defs.items()))


def _ops(kind: str, plural: str, namespaced: bool) -> dict:
    ref = {"$ref": f"#/definitions/{PREFIX}{kind}"}
    lref = {"$ref": f"#/definitions/{PREFIX}{kind}List"}
    scope = "Namespaced" if namespaced else ""
    base = f"/apis/{C.API_VERSION}/" + ("namespaces/{namespace}/" if namespaced else "") + plural
    ns_param = [{"name": "namespace", "in": "path", "required": True, "type": "string"}] if namespaced else []
    name_param = [{"name": "name", "in": "path", "required": True, "type": "string"}]
    body = [{"name": "body", "in": "body", "required": True, "schema": ref}]
    ok = lambda s: {"200": {"description": "OK", "schema": s}}  # noqa: E731
    tag = [kind]
    return {
        base: {
            "get": {"operationId": f"list{scope}{kind}", "tags": tag, "parameters": ns_param + [
                {"name": "labelSelector", "in": "query", "type": "string"}], "responses": ok(lref)},
            "post": {"operationId": f"create{scope}{kind}", "tags": tag, "parameters": ns_param + body + [
                {"name": "dryRun", "in": "query", "type": "string", "enum": ["All"]}],
                "responses": {"200": {"description": "OK", "schema": ref}, "409": {"description": "AlreadyExists"},
                              "422": {"description": "Invalid (admission)"}}},
        },
        base + "/{name}": {
            "get": {"operationId": f"read{scope}{kind}", "tags": tag, "parameters": ns_param + name_param,
                    "responses": {**ok(ref), "404": {"description": "NotFound"}}},
            "put": {"operationId": f"replace{scope}{kind}", "tags": tag, "parameters": ns_param + name_param + body,
                    "responses": {**ok(ref), "409": {"description": "Conflict"}}},
            "patch": {"operationId": f"patch{scope}{kind}", "tags": tag, "consumes": ["application/merge-patch+json"],
                      "parameters": ns_param + name_param + [{"name": "body", "in": "body", "required": True,
                                                              "schema": {"type": "object"}}], "responses": ok(ref)},
            "delete": {"operationId": f"delete{scope}{kind}", "tags": tag, "parameters": ns_param + name_param,
                       "responses": {"200": {"description": "OK"}}},
        },
        base + "/{name}/status": {
            "put": {"operationId": f"replace{scope}{kind}Status", "tags": tag, "parameters": ns_param + name_param + body,
                    "responses": ok(ref)},
        },
    }


def swagger() -> dict:
    paths: dict = {}
    for kind, (plural, namespaced, _spec) in V.KINDS.items():
        paths.update(_ops(kind, plural, namespaced))
    return {"swagger": "2.0",
            "info": {"title": "ome-amd", "description": f"{C.API_VERSION} API of the MI355X-native OME", "version": VERSION},
            "consumes": ["application/json"], "produces": ["application/json"],
            "paths": dict(sorted(paths.items())), "definitions": definitions()}


def write(path: str | Path) -> Path:
    p = Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(json.dumps(swagger(), indent=2, sort_keys=False) + "\n")
    return p


if __name__ == "__main__":
    print(write(sys.argv[1] if len(sys.argv) > 1 else "config/openapi/swagger.json"))

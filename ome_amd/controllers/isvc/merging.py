"""Spec merging for ServingRuntime templates and InferenceService overrides.

* ``strategic_merge``: Kubernetes strategic-merge semantics for the PodSpec fields the specs
  use — maps merge recursively, lists of named objects (containers, volumes, env,
  volumeMounts, ports, imagePullSecrets) merge by ``name``, other lists are replaced;
  ``None`` in the override deletes (``utils/merging.go:59-144``).
* ``merge_runtime_container``: strategic merge of a runtime container with a runner, then
  **args concatenated** runtime-first (``MergeRuntimeContainers``, :20-57).
* ``merge_args`` / ``override_arg``: key-based CLI arg merge for ``runtimeArgsOverride`` and the
  TP/PP rewrite of ``--tp-size|--tp|--tensor-parallel-size`` and
  ``--pp-size|--pp|--pipeline-parallel-size``, preserving the single-string multi-line form.
* ``replace_placeholders``: ``{{.Name}}``-style Go templates over the ISVC metadata.
"""
from __future__ import annotations

import copy
import json
import re

from ome_amd.controllers.config import render_template

_MERGE_KEYS = {"containers": "name", "initContainers": "name", "volumes": "name", "env": "name",
               "volumeMounts": "mountPath", "ports": "containerPort", "imagePullSecrets": "name",
               "tolerations": None, "envFrom": None}


def strategic_merge(base, override, field: str | None = None):
    if override is None:
        return copy.deepcopy(base)
    if isinstance(base, dict) and isinstance(override, dict):
        out = copy.deepcopy(base)
        for k, v in override.items():
            if v is None:
                out.pop(k, None)
            else:
                out[k] = strategic_merge(out.get(k), v, k)
        return out
    if isinstance(base, list) and isinstance(override, list):
        key = _MERGE_KEYS.get(field or "")
        if key and all(isinstance(x, dict) for x in base + override):
            out = copy.deepcopy(base)
            for item in override:
                k = item.get(key)
                for i, b in enumerate(out):
                    if k is not None and b.get(key) == k:
                        out[i] = strategic_merge(b, item, None)
                        break
                else:
                    out.append(copy.deepcopy(item))
            return out
        return copy.deepcopy(override)
    return copy.deepcopy(override)


def merge_spec(runtime_spec: dict | None, isvc_spec: dict | None) -> dict | None:
    """ISVC component spec over the runtime's component template.  No ISVC spec -> None."""
    if isvc_spec is None:
        return None
    if runtime_spec is None:
        return copy.deepcopy(isvc_spec)
    return strategic_merge(runtime_spec, isvc_spec)


def merge_runtime_container(runtime_c: dict, runner: dict) -> dict:
    merged = strategic_merge(runtime_c, {k: v for k, v in runner.items() if k != "args"})
    if not merged.get("name"):
        merged["name"] = runtime_c.get("name")
    args = list(runtime_c.get("args") or []) + list(runner.get("args") or [])
    if args:
        merged["args"] = args
    return merged


def replace_placeholders(container: dict, meta: dict) -> dict:
    vals = {"Name": meta.get("name", ""), "Namespace": meta.get("namespace", ""),
            "Labels": meta.get("labels") or {}, "Annotations": meta.get("annotations") or {}}
    s = json.dumps(container)
    if "{{" not in s:
        return container
    return json.loads(render_template(s, vals))


# ------------------------------------------------------------------ args
def _key(arg: str) -> str:
    a = arg.strip()
    if not a:
        return ""
    if not a.startswith("-"):
        return a
    if "=" in a:
        return a.split("=", 1)[0]
    return a.split()[0]


def is_multiline(args: list[str]) -> bool:
    return bool(args) and ("\n" in args[0] or "\\" in args[0])


def normalize_args(args: list[str]) -> list[str]:
    out = []
    for a in args:
        if is_multiline([a]):
            for line in a.split("\n"):
                t = line.strip().rstrip("\\").strip()
                if t:
                    out.extend(_split_flag_line(t))
        elif a.strip():
            out.append(a.strip())
    return out


def _split_flag_line(line: str) -> list[str]:
    # "--tp-size 4" on one line -> ["--tp-size", "4"] so groups parse uniformly
    parts = line.split()
    if len(parts) == 2 and parts[0].startswith("-") and not parts[1].startswith("-"):
        return parts
    return [line]


def to_multiline(args: list[str]) -> list[str]:
    if not args:
        return args
    lines, i = [], 0
    while i < len(args):
        a = args[i]
        if a.startswith("-") and "=" not in a and i + 1 < len(args) and not args[i + 1].startswith("-"):
            lines.append(f"{a} {args[i + 1]}")
            i += 2
        else:
            lines.append(a)
            i += 1
    return ["\n".join(line + (" \\" if j < len(lines) - 1 else "") for j, line in enumerate(lines))]


def _groups(args: list[str]) -> list[tuple[str, list[str]]]:
    out, i = [], 0
    while i < len(args):
        a = args[i]
        k = _key(a)
        if not k or "=" in a:
            out.append((k or a, [a]))
            i += 1
        elif i + 1 < len(args) and not args[i + 1].startswith("-"):
            out.append((k, [a, args[i + 1]]))
            i += 2
        else:
            out.append((k, [a]))
            i += 1
    return out


def merge_args(base: list[str] | None, override: list[str] | None) -> list[str]:
    base, override = list(base or []), list(override or [])
    if not override:
        return base
    if not base:
        return override
    multiline = is_multiline(base)
    order: list[str] = []
    m: dict[str, list[str]] = {}
    for k, v in _groups(normalize_args(base)) + _groups(normalize_args(override)):
        if k not in m:
            order.append(k)
        m[k] = v
    merged = [x for k in order for x in m[k]]
    return to_multiline(merged) if multiline else merged


def override_arg(args: list[str] | None, key: str, value: int) -> tuple[list[str], bool]:
    args = list(args or [])
    if not args:
        return args, False
    if is_multiline(args):
        pat = re.compile(re.escape(key) + r"(?:=|\s+)\d+")
        if not pat.search(args[0]):
            return args, False
        args[0] = pat.sub(f"{key}={value}", args[0])
        return args, True
    for i, a in enumerate(args):
        if a == key and i + 1 < len(args):
            args[i + 1] = str(value)
            return args, True
        if a.startswith(key + "="):
            args[i] = f"{key}={value}"
            return args, True
        # single-string command lines: "python -m x --tp-size 4 ..."
        if " " in a:
            pat = re.compile(r"(?<!\S)" + re.escape(key) + r"(?:=|\s+)\d+")
            if pat.search(a):
                args[i] = pat.sub(f"{key} {value}", a, count=1)
                return args, True
    return args, False


TP_ALIASES = ("--tp-size", "--tp", "--tensor-parallel-size")
PP_ALIASES = ("--pp-size", "--pp", "--pipeline-parallel-size")
DP_ALIASES = ("--dp-size", "--dp", "--data-parallel-size")


def override_param(container: dict, aliases, value: int) -> bool:
    for a in aliases:
        args, ok = override_arg(container.get("args"), a, value)
        if ok:
            container["args"] = args
            return True
    for a in aliases:
        cmd, ok = override_arg(container.get("command"), a, value)
        if ok:
            container["command"] = cmd
            return True
    return False


# ------------------------------------------------------------------ env / volumes helpers
def set_env(container: dict, name: str, value: str, overwrite: bool = True) -> None:
    env = container.setdefault("env", [])
    for e in env:
        if e.get("name") == name:
            if overwrite:
                e.clear()
                e.update({"name": name, "value": value})
            return
    env.append({"name": name, "value": value})


def get_env(container: dict, name: str) -> str | None:
    for e in container.get("env") or []:
        if e.get("name") == name:
            return e.get("value")
    return None


def add_volume_mount(container: dict, vm: dict) -> None:
    vms = container.setdefault("volumeMounts", [])
    if not any(v.get("mountPath") == vm["mountPath"] or v.get("name") == vm["name"] for v in vms):
        vms.append(vm)


def add_volume(pod_spec: dict, vol: dict) -> None:
    vols = pod_spec.setdefault("volumes", [])
    if not any(v.get("name") == vol["name"] for v in vols):
        vols.append(vol)


def gpu_count(container: dict, resource_names=None) -> int:
    from ome_amd.api import constants as C

    names = resource_names or C.GPU_RESOURCE_NAMES
    res = container.get("resources") or {}
    for section in ("limits", "requests"):
        for n in names:
            v = (res.get(section) or {}).get(n)
            if v is not None:
                try:
                    return int(str(v))
                except ValueError:
                    return 0
    return 0


def merge_resources(container: dict, ac_spec: dict | None, runtime_spec: dict | None) -> None:
    """runtime container resources fill gaps; AcceleratorClass resources override (``MergeResource``)."""
    res = container.setdefault("resources", {})
    for section in ("requests", "limits"):
        cur = res.setdefault(section, {})
        for rc in (runtime_spec or {}).get("containers") or []:
            if rc.get("name") == container.get("name"):
                for k, v in ((rc.get("resources") or {}).get(section) or {}).items():
                    cur.setdefault(k, v)
                break
        for r in (ac_spec or {}).get("resources") or []:
            cur[r["name"]] = r.get("quantity")
        if not cur:
            res.pop(section)
    if not res:
        container.pop("resources")

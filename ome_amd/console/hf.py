"""Offline Hugging Face lookups for the web console.

The reference console proxies ``huggingface.co/api/models`` (``web-console/backend/internal/
handlers/huggingface.go:27-160``: search, model info, config.json).  A serving node here has no
egress, so the same three questions are answered from what is on the node:

* the local Hugging Face hub cache (``$HF_HUB_CACHE`` / ``$HF_HOME/hub``, ``models--org--name``
  snapshot directories, scanned with ``huggingface_hub`` when present);
* the models root the model-agent downloads into (``<root>/<org>/<name>/config.json``);
* the BaseModels / ClusterBaseModels already in the store (their ``hf://`` storage URIs).

Results carry the reference's field names (``id``, ``author``, ``downloads``, ``likes``, ``tags``,
``pipeline_tag``, ``library_name``) where they are knowable offline.
"""
from __future__ import annotations

import json
import os
from pathlib import Path


def _hub_cache() -> Path:
    p = os.environ.get("HF_HUB_CACHE") or os.environ.get("HUGGINGFACE_HUB_CACHE")
    if p:
        return Path(p)
    home = os.environ.get("HF_HOME") or os.path.join(os.path.expanduser("~"), ".cache", "huggingface")
    return Path(home) / "hub"


def _cached_repos() -> dict[str, Path]:
    """repo id -> newest snapshot directory in the local hub cache."""
    out: dict[str, Path] = {}
    root = _hub_cache()
    if not root.is_dir():
        return out
    for d in root.glob("models--*"):
        rid = d.name[len("models--"):].replace("--", "/")
        snaps = sorted((d / "snapshots").glob("*"), key=lambda p: p.stat().st_mtime, reverse=True)
        if snaps:
            out[rid] = snaps[0]
    return out


def _models_root_repos(models_root: str | None) -> dict[str, Path]:
    out: dict[str, Path] = {}
    if not models_root or not os.path.isdir(models_root):
        return out
    for cfg in Path(models_root).glob("*/*/config.json"):
        out[f"{cfg.parent.parent.name}/{cfg.parent.name}"] = cfg.parent
    for cfg in Path(models_root).glob("*/config.json"):
        out.setdefault(cfg.parent.name, cfg.parent)
    return out


def _store_repos(store) -> dict[str, dict]:
    out: dict[str, dict] = {}
    if store is None:
        return out
    for kind in ("ClusterBaseModel", "BaseModel"):
        for o in store.list("ome.io/v1beta1", kind):
            uri = ((o.get("spec") or {}).get("storage") or {}).get("storageUri") or ""
            if uri.startswith("hf://"):
                rid = uri[len("hf://"):].split("@")[0].strip("/")
                out.setdefault(rid, o)
    return out


def _describe(rid: str, path: Path | None, obj: dict | None) -> dict:
    cfg = {}
    if path is not None and (path / "config.json").is_file():
        try:
            cfg = json.loads((path / "config.json").read_text())
        except ValueError:
            cfg = {}
    spec = (obj or {}).get("spec") or {}
    arch = (cfg.get("architectures") or [spec.get("modelArchitecture")] or [None])[0]
    tags = [t for t in (cfg.get("model_type"), arch, "safetensors" if path and any(path.glob("*.safetensors")) else None)
            if t]
    return {"id": rid, "modelId": rid, "author": rid.split("/")[0] if "/" in rid else None,
            "downloads": 0, "likes": 0, "tags": tags,
            "pipeline_tag": "feature-extraction" if "embed" in rid.lower() else "text-generation",
            "library_name": "transformers", "local_path": str(path) if path else None,
            "in_cluster": obj is not None, "architecture": arch,
            "model_type": cfg.get("model_type")}


def search(q: str = "", limit: int = 20, author: str | None = None, store=None,
           models_root: str | None = None) -> list[dict]:
    ql = (q or "").lower()
    cached = {**_models_root_repos(models_root), **_cached_repos()}
    known = _store_repos(store)
    ids = sorted(set(cached) | set(known))
    out = []
    for rid in ids:
        if ql and ql not in rid.lower():
            continue
        if author and not rid.lower().startswith(author.lower() + "/"):
            continue
        out.append(_describe(rid, cached.get(rid), known.get(rid)))
        if len(out) >= max(1, int(limit)):
            break
    return out


def _locate(model_id: str, models_root: str | None) -> Path | None:
    cached = {**_models_root_repos(models_root), **_cached_repos()}
    if model_id in cached:
        return cached[model_id]
    if models_root:
        p = Path(models_root) / model_id
        if (p / "config.json").is_file():
            return p
    return None


def info(model_id: str, models_root: str | None = None) -> dict | None:
    p = _locate(model_id, models_root)
    if p is None:
        return None
    d = _describe(model_id, p, None)
    d["siblings"] = [{"rfilename": str(f.relative_to(p))} for f in sorted(p.rglob("*")) if f.is_file()]
    try:
        from ome_amd.modelagent.modelconfig import load_model_config, model_metadata

        d["ome"] = model_metadata(load_model_config(str(p)))
    except Exception:  # noqa: BLE001 — optional enrichment (parameter count, capabilities)
        pass
    return d


def config(model_id: str, models_root: str | None = None) -> dict | None:
    p = _locate(model_id, models_root)
    if p is None or not (p / "config.json").is_file():
        return None
    try:
        return json.loads((p / "config.json").read_text())
    except ValueError:
        return None

"""Checkpoint loading: SafeTensors shards -> (name, tensor) stream.

Fast path (``ome_amd.io.native`` / ``csrc/omeio``): the C++ loader parses shard headers,
``pread``s tensor byte ranges with a thread pool into pinned host buffers and issues
``hipMemcpyAsync`` straight into HBM, double-buffered (SURVEY.md §7.1 "Native artifact
I/O").  Fallback: ``safetensors.safe_open`` (no code execution; BASELINE loading rules).
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Iterator

import torch


def shard_files(model_path: str | Path) -> list[Path]:
    p = Path(model_path)
    idx = p / "model.safetensors.index.json"
    if idx.exists():
        wm = json.loads(idx.read_text())["weight_map"]
        return sorted({p / f for f in wm.values()})
    return sorted(p.glob("*.safetensors"))


def nested_components(model_path: str | Path) -> list[str]:
    """VILA / NVILA layout: component sub-directories holding safetensors (none at the top)."""
    from ome_amd.models.config import NESTED_COMPONENTS

    p = Path(model_path)
    if shard_files(p):
        return []
    return [c for c in NESTED_COMPONENTS if shard_files(p / c)]


def has_checkpoint(model_path: str | Path) -> bool:
    return bool(shard_files(model_path)) or bool(nested_components(model_path))


def iter_safetensors(model_path: str | Path, device="cpu", plan=None) -> Iterator[tuple[str, torch.Tensor]]:
    """``plan(name, shape) -> None | ("rows"|"cols", start, n)``: read only this tensor-parallel
    rank's shard of each tensor (``LlamaForCausalLM.shard_plan``); None = whole tensors.
    Component sub-directories (``nested_components``) are read in turn, names prefixed with the
    directory (``llm.``, ``vision_tower.``, ``mm_projector.``)."""
    comps = nested_components(model_path)
    if comps:
        for c in comps:
            sub = None if plan is None else (lambda name, shape, c=c: plan(f"{c}.{name}", shape))
            for name, t in iter_safetensors(Path(model_path) / c, device, sub):
                yield f"{c}.{name}", t
        return
    files = shard_files(model_path)
    if not files:
        raise FileNotFoundError(f"no safetensors shards under {model_path}")
    try:
        from ome_amd.io import native as nio

        if nio.available():
            ex = nio.ShardExchange.for_state(device) if plan is not None else None
            if torch.device(device).type == "cuda":
                yield from nio.iter_tensors_to_device(files, device, plan, ex)
            else:
                yield from nio.iter_tensors_host(files, plan, ex)
            return
    except ImportError:
        pass
    if plan is not None:
        raise RuntimeError("sharded checkpoint loading needs libomeio (python -m ome_amd.build)")
    from safetensors import safe_open

    for f in files:
        with safe_open(str(f), framework="pt", device="cpu") as fh:
            for name in fh.keys():
                yield name, fh.get_tensor(name)

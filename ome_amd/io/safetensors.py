"""SafeTensors header parsing and parameter counting (parity with
``pkg/hfutil/modelconfig/safetensors.go:16-195``: 8-byte little-endian header length, JSON
header (bounded), parameter count = sum of shape products excluding ``__metadata__``,
sharded checkpoints walked through ``model.safetensors.index.json``).

Uses the native ``omeio_st_header`` when ``libomeio.so`` is present, else pure Python.
Never executes anything from the file.
"""
from __future__ import annotations

import json
import os
import struct
from pathlib import Path

import torch

MAX_HEADER = 100 << 20
DTYPES = {"F64": torch.float64, "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16,
          "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
          "BOOL": torch.bool, "F8_E4M3": torch.float8_e4m3fn, "F8_E5M2": torch.float8_e5m2}
DTYPE_SIZE = {"F64": 8, "F32": 4, "F16": 2, "BF16": 2, "I64": 8, "I32": 4, "I16": 2, "I8": 1, "U8": 1, "BOOL": 1,
              "F8_E4M3": 1, "F8_E5M2": 1, "U16": 2, "U32": 4, "U64": 8}


def read_header(path: str | os.PathLike) -> tuple[dict, int]:
    """(header dict, data offset)."""
    try:
        from ome_amd.io import native

        if native.available():
            raw, off = native.st_header(path)
            return json.loads(raw), off
    except ImportError:
        pass
    with open(path, "rb") as f:
        pre = f.read(8)
        if len(pre) != 8:
            raise ValueError(f"{path}: truncated safetensors file")
        (n,) = struct.unpack("<Q", pre)
        size = os.fstat(f.fileno()).st_size
        if n == 0 or n > MAX_HEADER or 8 + n > size:
            raise ValueError(f"{path}: invalid safetensors header length {n}")
        hdr = json.loads(f.read(n))
    if not isinstance(hdr, dict):
        raise ValueError(f"{path}: header is not a JSON object")
    return hdr, 8 + n


def count_params(path: str | os.PathLike) -> int:
    hdr, _ = read_header(path)
    total = 0
    for k, v in hdr.items():
        if k == "__metadata__" or not isinstance(v, dict):
            continue
        n = 1
        for d in v.get("shape") or []:
            n *= int(d)
        total += n
    return total


def shard_list(model_dir: str | os.PathLike) -> list[Path]:
    p = Path(model_dir)
    idx = p / "model.safetensors.index.json"
    if idx.exists():
        wm = json.loads(idx.read_text()).get("weight_map") or {}
        return sorted({p / f for f in wm.values() if (p / f).exists()})
    return sorted(p.glob("*.safetensors"))


def count_params_in_dir(model_dir: str | os.PathLike, recursive: bool = False) -> int:
    files = shard_list(model_dir)
    if recursive:
        files = sorted(Path(model_dir).rglob("*.safetensors"))
    total = 0
    for f in files:
        try:
            total += count_params(f)
        except (ValueError, OSError):
            continue
    return total


def save_file(tensors: dict[str, torch.Tensor], path: str | os.PathLike, metadata: dict | None = None) -> None:
    """Minimal writer (tests / random:// checkpoints)."""
    rev = {v: k for k, v in DTYPES.items()}
    hdr, off, blobs = {}, 0, []
    for name, t in tensors.items():
        t = t.detach().contiguous().cpu()
        b = t.reshape(-1).view(torch.uint8).numpy().tobytes() if t.numel() else b""
        hdr[name] = {"dtype": rev[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + len(b)]}
        off += len(b)
        blobs.append(b)
    if metadata:
        hdr["__metadata__"] = {str(k): str(v) for k, v in metadata.items()}
    h = json.dumps(hdr, separators=(",", ":")).encode()
    h += b" " * ((8 - len(h) % 8) % 8)
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(h)))
        f.write(h)
        for b in blobs:
            f.write(b)

"""Shared runtime structures for model forward passes: attention metadata and the paged KV cache."""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch

from ome_amd import ops


@dataclass
class AttnMeta:
    """Per-step attention metadata (all int32, on the model device).

    decode:  one query token per sequence, ``seq_lens`` includes the new token.
    prefill: any mix of prompt chunks / single-token rows; sequence ``s`` owns query rows
             ``cu_q[s]:cu_q[s+1]`` at absolute positions ``kv_lens[s]-q_len .. kv_lens[s]-1``.
    mixed:   rows ``[0, num_prefill)`` are prefill chunks (``cu_q``/``kv_lens``/``items``/
             ``block_tables``), rows ``[num_prefill, T)`` are single-token decode rows run by the
             GQA-sharing decode kernel (``seq_lens``/``dec_block_tables``/``order``/``decode_ws``)
             — so decodes riding along a prefill step cost decode-kernel KV traffic, not G x it.
    """

    mode: str
    positions: torch.Tensor
    slots: torch.Tensor
    block_tables: torch.Tensor
    seq_lens: torch.Tensor | None = None
    cu_q: torch.Tensor | None = None
    kv_lens: torch.Tensor | None = None
    items: torch.Tensor | None = None
    logits_idx: torch.Tensor | None = None
    decode_ws: ops.DecodeWorkspace | None = None
    order: torch.Tensor | None = None      # decode: sequences longest-first (workgroup dispatch order)
    num_prefill: int = 0                   # mixed: rows before this index are prefill rows
    dec_block_tables: torch.Tensor | None = None
    extra: dict = field(default_factory=dict)

    @property
    def is_decode(self) -> bool:
        return self.mode == "decode"

    @property
    def num_tokens(self) -> int:
        return self.positions.shape[0]


#: ``--kv-cache-dtype`` values (SGLang / vLLM spelling) -> cache element dtype (None = model dtype)
KV_CACHE_DTYPES = {"auto": None, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
                   "fp8": torch.float8_e4m3fn, "fp8_e4m3": torch.float8_e4m3fn, "fp8_e5m2": torch.float8_e5m2}


def kv_cache_dtype(name: str | None, model_dtype=torch.bfloat16):
    key = (name or "auto").lower()
    if key not in KV_CACHE_DTYPES:
        raise ValueError(f"unsupported --kv-cache-dtype {name!r} (choose from {sorted(KV_CACHE_DTYPES)})")
    return KV_CACHE_DTYPES[key] or model_dtype


class PagedKVCache:
    """Per-layer paged K/V tensors: K ``[pages, Hkv, P, D]``, V ``[pages, Hkv, D, P]``.

    Elements are the model dtype (bf16), or OCP fp8 e4m3 / e5m2 (``--kv-cache-dtype fp8*``, K15)
    holding ``x / scale`` with one dequantisation scale per layer for K and for V
    (``k_scale`` / ``v_scale``, 1.0 unless the checkpoint provides them).
    Zero-initialised so that masked (never-written) slots can never inject NaN/Inf into the
    P*V product of the attention kernels.
    """

    def __init__(self, num_layers: int, num_pages: int, num_kv_heads: int, head_dim: int, page_size: int = 16,
                 dtype=torch.bfloat16, device="cuda", v_dim: int | None = None, layers: list[int] | None = None):
        """``v_dim`` = 0: key-only cache (MLA keeps one latent row per token, the values are a
        slice of it); ``None``: same width as the keys.  ``layers``: the global layer ids held
        here (a pipeline stage's slice); other entries of ``k`` / ``v`` are None."""
        self.num_layers, self.num_pages, self.page_size = num_layers, num_pages, page_size
        # ``num_kv_heads``: one count, or a {layer: heads} map (DeciLM / Nemotron-NAS: per-layer GQA)
        per = num_kv_heads if isinstance(num_kv_heads, dict) else None
        self.num_kv_heads = max(per.values()) if per else num_kv_heads
        self.head_dim, self.dtype = head_dim, dtype
        self.v_dim = head_dim if v_dim is None else v_dim
        self.local_layers = list(range(num_layers)) if layers is None else list(layers)
        own = set(self.local_layers)
        hk = (lambda i: per[i]) if per else (lambda i: num_kv_heads)  # noqa: E731
        self.k = [torch.zeros(num_pages, hk(i), page_size, head_dim, dtype=dtype, device=device)
                  if i in own else None for i in range(num_layers)]
        self.v = [torch.zeros(num_pages, hk(i), self.v_dim, page_size, dtype=dtype, device=device)
                  if i in own else None for i in range(num_layers)]
        self.k_scale = [1.0] * num_layers
        self.v_scale = [1.0] * num_layers

    @property
    def is_fp8(self) -> bool:
        return self.dtype in (torch.float8_e4m3fn, torch.float8_e5m2)

    def scales(self, i: int) -> tuple[float, float]:
        return self.k_scale[i], self.v_scale[i]

    def set_scales(self, scales: dict[int, tuple[float, float]]) -> None:
        """Per-layer (k_scale, v_scale) from a checkpoint (``*.k_scale`` / ``*.v_scale``)."""
        for i, (ks, vs) in scales.items():
            if 0 <= i < self.num_layers:
                self.k_scale[i], self.v_scale[i] = float(ks), float(vs)

    @staticmethod
    def bytes_per_page(num_layers: int, num_kv_heads: int, head_dim: int, page_size: int, dtype=torch.bfloat16,
                       v_dim: int | None = None) -> int:
        v = head_dim if v_dim is None else v_dim
        heads = sum(num_kv_heads.values()) if isinstance(num_kv_heads, dict) else num_layers * num_kv_heads
        return heads * (head_dim + v) * page_size * torch.tensor([], dtype=dtype).element_size()

    def layer(self, i: int) -> tuple[torch.Tensor, torch.Tensor]:
        return self.k[i], self.v[i]


# ---------------------------------------------------------------------------------------------
# Mixed steps: the prefill rows' attention and the decode rows' attention are independent
# kernels over disjoint output rows.  Decode attention streams the whole KV of every running
# sequence (HBM-bound, thousands of workgroups); prefill attention over a few short prompts is a
# latency-bound grid of a few hundred workgroups.  Issuing the prefill kernel on a side stream
# lets it run inside the decode kernel's wave instead of after it.  Opt-in: measured NEGATIVE on
# the headline (16.06k / 16.06k tok/s off vs 15.86k / 15.84k on, interleaved runs on one box,
# profiles/r03_mixed_attention_overlap.txt) -- the prefill grid steals CUs the HBM-bound decode
# kernel needs and the per-layer stream hand-offs add host work to every eager mixed step.
_MIXED_OVERLAP = os.environ.get("OME_MIXED_OVERLAP", "0") == "1"
_SIDE: dict = {}


def _side_stream(device: torch.device):
    s = _SIDE.get(device.index)
    if s is None:
        s = _SIDE[device.index] = torch.cuda.Stream(device)
    return s


def mixed_attention(q: torch.Tensor, n_prefill: int, prefill, decode) -> torch.Tensor:
    """``prefill(q_rows, out_rows)`` / ``decode(q_rows, out_rows)``: the two halves of a mixed
    step's attention, overlapped on two streams on the GPU (eager steps only: never inside a
    graph capture) and run back to back otherwise."""
    out = torch.empty_like(q)
    n = n_prefill
    if q.is_cuda and _MIXED_OVERLAP and not torch.cuda.is_current_stream_capturing():
        main = torch.cuda.current_stream(q.device)
        side = _side_stream(q.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            prefill(q[:n], out[:n])
        decode(q[n:], out[n:])
        main.wait_stream(side)
        q.record_stream(side)
        out.record_stream(side)
        return out
    prefill(q[:n], out[:n])
    decode(q[n:], out[n:])
    return out

"""Qwen-VL / Qwen-VL-Chat (``QWenLMHeadModel`` checkpoints with a ``visual`` config block).

Reference catalog entries: ``config/models/Qwen/Qwen-VL.yaml`` and ``Qwen-VL-Chat.yaml``.  The
language model is Qwen (v1), served by the ``QWenLMHeadModel`` spec of ``models/decoder.py``; this
adds the image side of the remote code (``visual.py``, not importable offline -- parity with it is
unpinned; ``tests/test_qwen_vl_cpu.py`` checks the tower against an fp32 restatement):

* ViT-bigG/14 at 448 px (``width`` 1664, 48 pre-norm blocks, 16 heads of 104 dims, GELU MLP of
  ``mlp_ratio`` x width): the patch conv as one GEMM, a learned 16 x 16 position table resized
  bicubically to the 32 x 32 patch grid, ``ln_pre``; the fused per-head [q | k | v] ``in_proj``
  rows are regrouped at load so the bidirectional varlen MFMA attention kernel reads q / k / v in
  place;
* a Resampler: 256 learned queries (+ 2-D sin-cos positions) cross-attend, 32 heads, to the
  LayerNormed ``kv_proj`` of the patch tokens (+ the resized sin-cos table); ``ln_post`` and the
  ``proj`` matrix give 256 language-model embeddings per image;
* prompts carry ``<img>`` (``image_start_id``), 256 placeholder rows and ``</img>``; the rows
  between the two markers take the image embeddings (what ``QWenModel.forward`` does after
  decoding the image path the remote tokenizer put there).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.decoder import DecoderForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import CLIP_MEAN, CLIP_STD, MMInput, load_image
from ome_amd.parallel import state as pstate


def sincos_2d(dim: int, grid: int) -> np.ndarray:
    """[grid * grid, dim] 2-D sin-cos table (the MAE layout the Resampler uses): the first half of
    the dims encodes each cell's column (w) coordinate, the second half its row (h) coordinate;
    each half is [sin | cos] over dim / 4 frequencies."""
    col, row = np.meshgrid(np.arange(grid, dtype=np.float32), np.arange(grid, dtype=np.float32), indexing="xy")
    grid_wh = np.stack([col, row], 0).reshape(2, 1, grid, grid)

    def one(d, pos):
        omega = 1.0 / 10000 ** (np.arange(d // 2, dtype=np.float32) / (d / 2.0))
        out = np.einsum("m,d->md", pos.reshape(-1), omega)
        return np.concatenate([np.sin(out), np.cos(out)], 1)

    return np.concatenate([one(dim // 2, grid_wh[0]), one(dim // 2, grid_wh[1])], 1)


def resize_pos(table: torch.Tensor, n: int) -> torch.Tensor:
    """[s*s, C] position table -> [n, C] (bicubic, as ``get_abs_pos``), identity when s*s == n."""
    s, t = int(math.isqrt(table.shape[0])), int(math.isqrt(n))
    if s == t:
        return table
    x = table.float().reshape(1, s, s, -1).permute(0, 3, 1, 2)
    x = F.interpolate(x, size=(t, t), mode="bicubic", align_corners=False)
    return x.permute(0, 2, 3, 1).reshape(t * t, -1).to(table.dtype)


def preprocess_qwen_vl(img, size: int) -> torch.Tensor:
    """PIL image -> [1, 3, size, size] fp32: bicubic resize to a square (no aspect preservation),
    CLIP mean / std normalisation (the remote code's torchvision pipeline)."""
    from PIL import Image

    img = load_image(img).resize((size, size), Image.BICUBIC)
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = (a - np.asarray(CLIP_MEAN, np.float32)) / np.asarray(CLIP_STD, np.float32)
    return torch.from_numpy(a).permute(2, 0, 1)[None].contiguous()


class QwenVLVisual:
    def __init__(self, vc: dict, device, dtype):
        self.device, self.dtype = device, dtype
        self.image = int(vc.get("image_size", 448))
        self.patch = int(vc.get("patch_size", 14))
        self.E = int(vc.get("width", 1664))
        self.L = int(vc.get("layers", 48))
        self.heads = int(vc.get("heads", 16))
        self.hd = self.E // self.heads
        self.mlp = int(self.E * float(vc.get("mlp_ratio", 4.9231)))
        self.out = int(vc.get("output_dim", 4096))
        self.nq = int(vc.get("n_queries", 256))
        self.rheads = self.out // 128
        self.side = self.image // self.patch
        self.w: dict[str, torch.Tensor] = {}

    @property
    def tokens(self) -> int:
        return self.nq

    def _put(self, t):
        return t.to(device=self.device, dtype=self.dtype).contiguous()

    def load(self, name: str, w: torch.Tensor) -> None:
        if name == "conv1.weight":
            w = w.reshape(w.shape[0], -1)
        elif name.endswith("attn.in_proj.weight") or name.endswith("attn.in_proj.bias"):
            # per-head [q | k | v] rows -> [all q; all k; all v] (head-contiguous q, k, v views)
            tail = w.shape[1:]
            w = w.reshape(self.heads, 3, self.hd, *tail).transpose(0, 1).reshape(3 * self.E, *tail)
        if name == "attn_pool.pos_embed":
            self.w[name] = w.float().to(self.device)
            return
        self.w[name] = self._put(w)

    def init_random(self, gen, std: float) -> None:
        E, M, O = self.E, self.mlp, self.out
        mk = lambda *s, sd=std: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, sd, generator=gen)  # noqa
        ones = lambda n: torch.ones(n, dtype=self.dtype, device=self.device)  # noqa: E731
        zeros = lambda n: torch.zeros(n, dtype=self.dtype, device=self.device)  # noqa: E731
        w = {"conv1.weight": mk(E, 3 * self.patch * self.patch), "positional_embedding": mk(256, E),
             "ln_pre.weight": ones(E), "ln_pre.bias": zeros(E), "ln_post.weight": ones(O), "ln_post.bias": zeros(O),
             "proj": mk(O, O), "attn_pool.query": mk(self.nq, O), "attn_pool.kv_proj.weight": mk(O, E),
             "attn_pool.attn.in_proj_weight": mk(3 * O, O), "attn_pool.attn.in_proj_bias": zeros(3 * O),
             "attn_pool.attn.out_proj.weight": mk(O, O), "attn_pool.attn.out_proj.bias": zeros(O),
             "attn_pool.ln_q.weight": ones(O), "attn_pool.ln_q.bias": zeros(O),
             "attn_pool.ln_kv.weight": ones(O), "attn_pool.ln_kv.bias": zeros(O)}
        for i in range(self.L):
            p = f"transformer.resblocks.{i}."
            w.update({p + "ln_1.weight": ones(E), p + "ln_1.bias": zeros(E), p + "ln_2.weight": ones(E),
                      p + "ln_2.bias": zeros(E), p + "attn.in_proj.weight": mk(3 * E, E),
                      p + "attn.in_proj.bias": zeros(3 * E), p + "attn.out_proj.weight": mk(E, E),
                      p + "attn.out_proj.bias": zeros(E), p + "mlp.c_fc.weight": mk(M, E), p + "mlp.c_fc.bias": zeros(M),
                      p + "mlp.c_proj.weight": mk(E, M), p + "mlp.c_proj.bias": zeros(E)})
        self.w = w
        self.w["attn_pool.pos_embed"] = torch.from_numpy(sincos_2d(O, int(math.isqrt(self.nq)))).to(self.device)

    def forward(self, px: torch.Tensor) -> torch.Tensor:
        """[n, 3, image, image] -> [n * n_queries, output_dim]."""
        w, E, ps, s = self.w, self.E, self.patch, self.side
        n = px.shape[0]
        T = s * s
        p = px.to(self.device, torch.float32).reshape(n, 3, s, ps, s, ps).permute(0, 2, 4, 1, 3, 5)
        x = linear(p.reshape(n * T, 3 * ps * ps).to(self.dtype), w["conv1.weight"])
        x = (x.view(n, T, E) + resize_pos(w["positional_embedding"], T)[None]).reshape(n * T, E)
        x = ops.layernorm(x.contiguous(), w["ln_pre.weight"], w["ln_pre.bias"], 1e-6)
        for i in range(self.L):
            q = f"transformer.resblocks.{i}."
            h = ops.layernorm(x, w[q + "ln_1.weight"], w[q + "ln_1.bias"], 1e-6)
            qkv = linear(h, w[q + "attn.in_proj.weight"], w[q + "attn.in_proj.bias"]).view(n * T, 3, self.heads, self.hd)
            a = ops.varlen_attention(qkv[:, 0], qkv[:, 1], qkv[:, 2], [T] * n, self.hd ** -0.5)
            x = x + linear(a.reshape(n * T, E), w[q + "attn.out_proj.weight"], w[q + "attn.out_proj.bias"])
            h = ops.layernorm(x, w[q + "ln_2.weight"], w[q + "ln_2.bias"], 1e-6)
            h = linear(h, w[q + "mlp.c_fc.weight"], w[q + "mlp.c_fc.bias"])
            x = x + linear(ops.act(h, 3) if h.is_cuda else F.gelu(h), w[q + "mlp.c_proj.weight"],
                           w[q + "mlp.c_proj.bias"])
        return self._resample(x.view(n, T, E))

    def _resample(self, x: torch.Tensor) -> torch.Tensor:
        """Resampler: learned queries cross-attend to the patch tokens (small: plain batched GEMMs)."""
        w, O, H = self.w, self.out, self.rheads
        n, T, _ = x.shape
        pe = w["attn_pool.pos_embed"]
        kv = linear(x.reshape(n * T, -1), w["attn_pool.kv_proj.weight"])
        kv = ops.layernorm(kv, w["attn_pool.ln_kv.weight"], w["attn_pool.ln_kv.bias"], 1e-6).view(n, T, O)
        qn = ops.layernorm(w["attn_pool.query"], w["attn_pool.ln_q.weight"], w["attn_pool.ln_q.bias"], 1e-6)
        wi, bi = w["attn_pool.attn.in_proj_weight"], w["attn_pool.attn.in_proj_bias"]
        Q = linear((qn.float() + pe).to(self.dtype), wi[:O], bi[:O])                       # [nq, O]
        K = linear((kv.float() + resize_pos(pe, T)[None]).to(self.dtype).reshape(n * T, O), wi[O:2 * O], bi[O:2 * O])
        V = linear(kv.reshape(n * T, O), wi[2 * O:], bi[2 * O:])
        hd = O // H
        Qh = Q.view(1, self.nq, H, hd).transpose(1, 2).float()                                # [1, H, nq, hd]
        Kh = K.view(n, T, H, hd).transpose(1, 2).float()
        Vh = V.view(n, T, H, hd).transpose(1, 2).float()
        att = torch.softmax((Qh @ Kh.transpose(-1, -2)) * hd ** -0.5, -1)                       # [n, H, nq, T]
        o = (att @ Vh).transpose(1, 2).reshape(n * self.nq, O).to(self.dtype)
        o = linear(o, w["attn_pool.attn.out_proj.weight"], w["attn_pool.attn.out_proj.bias"])
        o = ops.layernorm(o, w["ln_post.weight"], w["ln_post.bias"], 1e-6)
        return (o.float() @ w["proj"].float()).to(self.dtype)


class QwenVLForCausalLM(DecoderForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        vc = (cfg.extra or {}).get("visual") or {}
        self.visual = QwenVLVisual(vc, self.device, dtype)
        self.img_start = int(vc.get("image_start_id", 151857))
        self.img_end = self.img_start + 1
        self.img_pad = self.img_start + 2

    def init_random(self, seed: int = 0, std: float = 0.02) -> "QwenVLForCausalLM":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 5051)
        self.visual.init_random(gen, std)
        return self

    def load_hf_weights(self, weights) -> "QwenVLForCausalLM":
        def text_only():
            for name, w in weights:
                if name.startswith("transformer.visual."):
                    self.visual.load(name[len("transformer.visual."):], w)
                else:
                    yield name, w

        return super().load_hf_weights(text_only())

    def weight_bytes(self) -> int:
        return super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.img_start, self.img_end]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        """Every ``<img> ... </img>`` pair (whatever sits between: the remote tokenizer's image path
        bytes, or nothing) becomes ``<img>`` + 256 placeholder rows + ``</img>``."""
        ids, spans, pvs, k, i = [], [], [], 0, 0
        while i < len(prompt_ids):
            t = prompt_ids[i]
            if t != self.img_start:
                ids.append(t)
                i += 1
                continue
            j = i + 1
            while j < len(prompt_ids) and prompt_ids[j] != self.img_end:
                j += 1
            if k >= len(images):
                raise ValueError("more <img> markers than images")
            im = images[k]
            pvs.append(im if isinstance(im, torch.Tensor) else preprocess_qwen_vl(im, self.visual.image))
            ids.append(self.img_start)
            spans.append((len(ids), self.visual.tokens))
            ids += [self.img_pad] * self.visual.tokens
            ids.append(self.img_end)
            k += 1
            i = j + 1
        if k != len(images):
            raise ValueError(f"prompt has {k} <img> markers for {len(images)} images")
        side = self.visual.side
        return ids, MMInput(torch.cat(pvs, 0), [(1, side, side)] * len(pvs), spans)

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        return self.visual.forward(pixel_values)

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h

"""Kimi-VL (``KimiVLForConditionalGeneration``; reference catalog
``config/runtimes/srt/moonshotai/kimi-vl-a3b-instruct-rt.yaml``) and the transformers
``Kimi_K25ForConditionalGeneration`` layout of the same MoonViT + DeepSeek-V3 design.

* preprocessing (NaViT style, native resolution): scale down (never up) so the image holds at
  most ``max_patches`` 14-px patches (and ``max_side`` patches per side when set), bicubic,
  zero-pad right / bottom to multiples of 28 px, mean / std 0.5, raster-order patches;
* MoonViT tower: patch GEMM (+bias) -> learned 64 x 64 position grid bicubically resampled to
  each image's patch grid -> LayerNorm blocks: fused QKV GEMM (+bias) -> 2D rotary (column and
  row angles alternate over the frequency pairs; the original checkpoints' interleaved-pair form
  is re-laid to rotate-half form at load) -> varlen MFMA attention per image -> O GEMM;
  LayerNorm -> GELU-tanh MLP -> final LayerNorm;
* projector: LayerNorm per patch -> 2 x 2 patch merge (concatenation) -> GEMM -> GELU -> GEMM;
* language model: DeepSeek-V3 (Moonlight MoE with MLA) of ``deepseek.py``; image rows spliced into
  the embedded prompt (one ``<|media_pad|>`` per merged patch, content-hash ids).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.deepseek import DeepseekForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, expand_image_tokens, load_image
from ome_amd.parallel import state as pstate

KIMI_VL_ARCHS = {"KimiVLForConditionalGeneration", "Kimi_K25ForConditionalGeneration"}


def kimi_resize(h: int, w: int, patch: int = 14, merge: int = 2, max_patches: int = 4096,
                max_side: int | None = None) -> tuple[tuple[int, int], tuple[int, int]]:
    """-> ((resized h, w), (padded h, w)): down-scale only, pad to multiples of patch * merge."""
    n = max(1.0, h // patch) * max(1.0, w // patch)
    s = min(1.0, math.sqrt(max_patches / n))
    if max_side:
        s = min(s, max_side * patch / h, max_side * patch / w)
    nh, nw = max(1, int(h * s)), max(1, int(w * s))
    if max_side:
        nh, nw = min(nh, max_side * patch), min(nw, max_side * patch)
    f = patch * merge
    return (nh, nw), (nh + (f - nh % f) % f, nw + (f - nw % f) % f)


def preprocess_kimi_vl(image, patch: int = 14, merge: int = 2, max_patches: int = 4096, max_side: int | None = None,
                       mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
    """-> (pixel_values [gh * gw, 3 * patch * patch] float32 raster order, (1, gh, gw))."""
    from PIL import Image

    img = load_image(image)
    (nh, nw), (ph, pw) = kimi_resize(img.height, img.width, patch, merge, max_patches, max_side)
    a = np.zeros((ph, pw, 3), dtype=np.float32)
    a[:nh, :nw] = np.asarray(img.resize((nw, nh), Image.BICUBIC), dtype=np.float32)
    a = (a / 255.0 - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    gh, gw = ph // patch, pw // patch
    x = a.transpose(2, 0, 1).reshape(3, gh, patch, gw, patch).transpose(1, 3, 0, 2, 4)
    return np.ascontiguousarray(x.reshape(gh * gw, 3 * patch * patch)), (1, gh, gw)


class MoonViTTower:
    """Weights by internal name: ``patch.w/b``, ``pos`` [gh, gw, E], per block ``{b}.ln1/ln2.w/b``,
    ``{b}.qkv.w/b`` (rotate-half q / k rows), ``{b}.o.w/b``, ``{b}.fc1/fc2.w/b``, ``final.w/b``."""

    def __init__(self, vc: dict, device, dtype):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1152))
        self.depth = int(vc.get("num_hidden_layers", 27))
        self.heads = int(vc.get("num_attention_heads", 16))
        self.hd = self.E // self.heads
        self.inter = int(vc.get("intermediate_size", 4304))
        self.patch = int(vc.get("patch_size", 14))
        mk = vc.get("merge_kernel_size", (2, 2))
        self.merge = int(mk[0] if isinstance(mk, (list, tuple)) else mk)
        self.pos_h = int(vc.get("init_pos_emb_height", vc.get("pos_emb_height", 64)))
        self.pos_w = int(vc.get("init_pos_emb_width", vc.get("pos_emb_width", 64)))
        theta = float((vc.get("rope_parameters") or {}).get("rope_theta", 10000.0))
        act = vc.get("hidden_act", "gelu_pytorch_tanh")
        if act not in ("gelu_pytorch_tanh", "gelu_tanh", "gelu_new"):
            raise NotImplementedError(f"MoonViT hidden_act {act!r}")
        if self.hd % 4:
            raise ValueError("MoonViT head dim must divide by 4")
        self.inv = 1.0 / (theta ** (torch.arange(0, self.hd, 4, dtype=torch.float32)[: self.hd // 4] / self.hd))
        self.w: dict[str, torch.Tensor] = {}
        self._pend: dict[str, dict[str, torch.Tensor]] = {}

    # ------------------------------------------------------------------ weights
    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I = self.E, self.inter
        shapes = {"patch.w": (E, 3 * self.patch ** 2), "patch.b": (E,), "pos": (self.pos_h, self.pos_w, E),
                  "final.w": (E,), "final.b": (E,)}
        for b in range(self.depth):
            shapes.update({f"{b}.ln1.w": (E,), f"{b}.ln1.b": (E,), f"{b}.ln2.w": (E,), f"{b}.ln2.b": (E,),
                           f"{b}.qkv.w": (3 * E, E), f"{b}.qkv.b": (3 * E,), f"{b}.o.w": (E, E), f"{b}.o.b": (E,),
                           f"{b}.fc1.w": (I, E), f"{b}.fc1.b": (I,), f"{b}.fc2.w": (E, I), f"{b}.fc2.b": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(".w") and len(s) == 1:
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    def _deinterleave_qk(self, t: torch.Tensor) -> torch.Tensor:
        """Original MoonViT rotates adjacent pairs (2j, 2j + 1); re-lay q / k rows per head so
        pair j becomes (j, j + hd / 2) (rotate-half form).  v rows stay."""
        E, D = self.E, self.hd
        perm = torch.cat([torch.arange(0, D, 2), torch.arange(1, D, 2)])
        idx = torch.cat([h * D + perm for h in range(2 * self.heads)] + [torch.arange(2 * E, 3 * E)])
        return t[idx.to(t.device)]

    def _put(self, key: str, t: torch.Tensor) -> None:
        self.w[key] = t.to(device=self.device, dtype=self.dtype).contiguous()

    def load(self, name: str, t: torch.Tensor) -> None:
        """``name`` relative to the tower: original Kimi-VL (``patch_embed.pos_emb.weight``,
        ``encoder.blocks.{b}.wqkv`` / ``wo`` / ``norm0`` / ``norm1`` / ``mlp.fc0`` / ``mlp.fc1``,
        ``encoder.final_layernorm``) or transformers Kimi-K2.5 (``patch_embed.pos_emb.
        position_embeddings``, ``layers.{b}.attn.{q,k,v}_proj`` / ``attn.proj`` / ``norm1`` /
        ``norm2`` / ``mlp.fc1`` / ``mlp.fc2``, ``final_layernorm``)."""
        kind = "w" if name.endswith("weight") or name.endswith("position_embeddings") else "b"
        if name.startswith("patch_embed.proj."):
            self._put(f"patch.{kind}", t.reshape(t.shape[0], -1) if kind == "w" else t)
            return
        if name in ("patch_embed.pos_emb.weight", "patch_embed.pos_emb.position_embeddings"):
            self._put("pos", t)
            return
        if name.startswith(("encoder.final_layernorm.", "final_layernorm.")):
            self._put(f"final.{kind}", t)
            return
        p = name.split(".")
        if p[0] == "encoder" and p[1] == "blocks":          # original
            b, mod = int(p[2]), ".".join(p[3:-1])
            if mod == "wqkv":
                self._put(f"{b}.qkv.{kind}", self._deinterleave_qk(t))
                return
            key = {"wo": "o", "norm0": "ln1", "norm1": "ln2", "mlp.fc0": "fc1", "mlp.fc1": "fc2"}.get(mod)
        elif p[0] == "layers":                               # transformers
            b, mod = int(p[1]), ".".join(p[2:-1])
            if mod in ("attn.q_proj", "attn.k_proj", "attn.v_proj"):
                got = self._pend.setdefault(f"{b}.qkv.{kind}", {})
                got[mod] = t
                if len(got) == 3:
                    self._put(f"{b}.qkv.{kind}", torch.cat([got["attn.q_proj"], got["attn.k_proj"],
                                                            got["attn.v_proj"]]))
                    del self._pend[f"{b}.qkv.{kind}"]
                return
            key = {"attn.proj": "o", "norm1": "ln1", "norm2": "ln2", "mlp.fc1": "fc1", "mlp.fc2": "fc2"}.get(mod)
        else:
            key = None
        if key is None:
            raise KeyError(f"unexpected MoonViT weight {name!r}")
        self._put(f"{b}.{key}.{kind}", t)

    # ------------------------------------------------------------------ forward
    def _pos_embed(self, grids) -> torch.Tensor:
        table = self.w["pos"]
        out = []
        for t, h, w in grids:
            if (h, w) == (self.pos_h, self.pos_w):
                e = table.reshape(-1, self.E)
            else:
                e = F.interpolate(table.float().permute(2, 0, 1)[None], size=(h, w), mode="bicubic",
                                  align_corners=False)[0].permute(1, 2, 0).reshape(-1, self.E)
            out.append(e.repeat(t, 1))
        return torch.cat(out).to(self.dtype)

    def _angles(self, grids) -> torch.Tensor:
        """[N, hd / 2]: pair 2i rotates by column * f_i, pair 2i + 1 by row * f_i (raster order)."""
        out = []
        for t, h, w in grids:
            r = torch.arange(h, dtype=torch.float32).repeat_interleave(w)
            c = torch.arange(w, dtype=torch.float32).repeat(h)
            a = torch.stack([torch.outer(c, self.inv), torch.outer(r, self.inv)], -1).reshape(h * w, -1)
            out.append(a.repeat(t, 1))
        return torch.cat(out)

    def forward(self, pixel_values: torch.Tensor, grids: list[tuple[int, int, int]]) -> torch.Tensor:
        """-> [N, E] final-normed patch features, raster order per image."""
        dev, dt, E, Hh, D, w = self.device, self.dtype, self.E, self.heads, self.hd, self.w
        pv = pixel_values.reshape(pixel_values.shape[0], -1)     # [N, 3, ps, ps] (transformers) or flat
        x = linear(pv.to(device=dev, dtype=dt), w["patch.w"], w["patch.b"])
        x = x + self._pos_embed(grids)
        ang = self._angles(grids).to(dev)
        emb = torch.cat([ang, ang], -1)
        cos, sin = emb.cos()[:, None, :], emb.sin()[:, None, :]
        lens = [h * ww for t, h, ww in grids for _ in range(t)]
        N = x.shape[0]

        def rope(t):
            tf = t.float()
            return (tf * cos + torch.cat([-tf[..., D // 2:], tf[..., :D // 2]], -1) * sin).to(dt)

        for b in range(self.depth):
            h = ops.layernorm(x, w[f"{b}.ln1.w"], w[f"{b}.ln1.b"], 1e-5)
            qkv = linear(h, w[f"{b}.qkv.w"], w[f"{b}.qkv.b"]).view(N, 3, Hh, D)
            a = ops.varlen_attention(rope(qkv[:, 0]), rope(qkv[:, 1]), qkv[:, 2], lens, D ** -0.5).reshape(N, E)
            x = x + linear(a, w[f"{b}.o.w"], w[f"{b}.o.b"])
            h = ops.layernorm(x, w[f"{b}.ln2.w"], w[f"{b}.ln2.b"], 1e-5)
            x = x + linear(ops.act(linear(h, w[f"{b}.fc1.w"], w[f"{b}.fc1.b"]).contiguous(), 1),
                           w[f"{b}.fc2.w"], w[f"{b}.fc2.b"])
        return ops.layernorm(x, w["final.w"], w["final.b"], 1e-5)

    def merge_patches(self, x: torch.Tensor, grids) -> torch.Tensor:
        """[N, C] raster-order rows -> [N / m^2, m^2 * C] (each m x m block concatenated row-major)."""
        m, out, off = self.merge, [], 0
        for t, h, w in grids:
            n = t * h * w
            blk = x[off:off + n].view(t, h // m, m, w // m, m, -1).permute(0, 1, 3, 2, 4, 5)
            out.append(blk.reshape(t * (h // m) * (w // m), -1))
            off += n
        return torch.cat(out).contiguous()


class KimiVLForConditionalGeneration(DeepseekForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.visual = MoonViTTower(dict(ex.get("vision_config") or {}), self.device, dtype)
        self.merge = self.visual.merge
        self.image_token_id = int(ex.get("media_placeholder_token_id", ex.get("image_token_id", 163605)))
        self.media_start = int(ex.get("vision_start_token_id", 163602))
        self.media_end = int(ex.get("vision_end_token_id", 163604))
        self.max_patches = int(ex.get("in_token_limit", ex.get("max_patches", 4096)))
        self.proj_eps = float(ex.get("projection_layer_norm_eps", 1e-5))
        self.proj: dict[str, torch.Tensor] = {}

    def init_random(self, seed: int = 0, std: float = 0.02) -> "KimiVLForConditionalGeneration":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 7717)
        self.visual.init_random(gen, std)
        E4, H = self.visual.E * self.merge ** 2, self.cfg.hidden_size
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        z = lambda n: torch.zeros(n, dtype=self.dtype, device=self.device)  # noqa
        self.proj = {"ln.w": torch.ones(self.visual.E, dtype=self.dtype, device=self.device), "ln.b": z(self.visual.E),
                     "fc1.w": mk(E4, E4), "fc1.b": z(E4), "fc2.w": mk(H, E4), "fc2.b": z(H)}
        return self

    _PROJ = {"pre_norm": "ln", "linear_1": "fc1", "linear_2": "fc2", "in_proj": "fc1", "out_proj": "fc2"}

    def load_hf_weights(self, weights) -> "KimiVLForConditionalGeneration":
        def lm_only():
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") and not name.startswith("model.layers.") else name
                if n.startswith("vision_tower."):
                    self.visual.load(n[len("vision_tower."):], w)
                elif n.startswith(("multi_modal_projector.", "mm_projector.")):
                    p = n.split(".")
                    key = {"0": "fc1", "2": "fc2"}[p[2]] if p[1] == "proj" else self._PROJ[p[1]]  # proj.0 / proj.2
                    self.proj[f"{key}.{'w' if p[-1] == 'weight' else 'b'}"] = \
                        w.to(device=self.device, dtype=self.dtype).contiguous()
                elif n.startswith("language_model."):
                    rest = n[len("language_model."):]
                    yield (rest if rest.startswith(("model.", "lm_head.")) else "model." + rest), w
                else:
                    yield name, w

        super().load_hf_weights(lm_only())
        if self.visual._pend:
            raise ValueError(f"incomplete MoonViT projections: {sorted(self.visual._pend)}")
        if len(self.proj) != 6:
            raise ValueError(f"multi-modal projector incomplete: {sorted(self.proj)}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for t in self.proj.values())

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.media_start, self.image_token_id, self.media_end]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        pvs, grids = [], []
        for im in images:
            if isinstance(im, tuple):
                pv, g = im
            else:
                pv, g = preprocess_kimi_vl(im, self.visual.patch, self.merge, self.max_patches)
            pvs.append(torch.as_tensor(pv, dtype=torch.float32))
            grids.append(tuple(int(v) for v in g))
        ids, spans = expand_image_tokens(list(prompt_ids), self.image_token_id, grids, self.merge, pvs,
                                         self.cfg.vocab_size)
        return ids, MMInput(torch.cat(pvs, 0), grids, spans)

    def encode_images(self, pixel_values: torch.Tensor, grids) -> torch.Tensor:
        p = self.proj
        x = self.visual.forward(pixel_values, grids)
        x = ops.layernorm(x, p["ln.w"], p["ln.b"], self.proj_eps)
        x = self.visual.merge_patches(x, grids)
        x = ops.act(linear(x, p["fc1.w"], p["fc1.b"]).contiguous(), 3)
        return linear(x, p["fc2.w"], p["fc2.b"])

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h

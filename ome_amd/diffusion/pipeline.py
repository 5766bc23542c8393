"""Qwen-Image text-to-image and image-editing pipelines (``QwenImagePipeline``,
``QwenImageEditPipeline``, ``QwenImageEditPlusPipeline``; reference catalog
``config/runtimes/srt/Qwen/Qwen-Image*-rt.yaml``), MI355X-side:

* prompt encoding: the Qwen2.5-VL-7B text encoder (``models/qwen2_vl.py``, our own prefill
  over a paged KV cache; images through its vision tower and M-RoPE for the edit variants) ->
  final normed hidden states, the chat-template prefix dropped (34 / 64 tokens);
* denoising: the MMDiT (``qwen_image_dit.py``) on packed 2x2 latent patches, prompt and negative
  prompt evaluated in ONE forward as two packed sequences, norm-preserving true CFG
  (``comb * |cond| / |comb|``), flow-matching Euler steps (``scheduler.py``);
* edit variants: the input image(s) VAE-encoded and appended to the image sequence (their own
  RoPE frame index), the prediction cut back to the generated latents;
* decode: the VAE (``vae.py``) -> uint8 RGB.
``from_pretrained`` reads a diffusers directory (``model_index.json``, ``transformer/``,
``vae/``, ``text_encoder/``, ``tokenizer/``); ``random(preset)`` builds random-init weights of the
named architecture (the benchmark rule: no checkpoints here).
"""
from __future__ import annotations

import json
import math
import time
from pathlib import Path

import numpy as np
import torch

from ome_amd import ops
from ome_amd.diffusion.qwen_image_dit import QwenImageDiT
from ome_amd.diffusion.scheduler import FlowMatchConfig, FlowMatchEuler
from ome_amd.diffusion.vae import QwenImageVAE
from ome_amd.models.common import AttnMeta, PagedKVCache

PIPELINES = {"QwenImagePipeline": "t2i", "QwenImageEditPipeline": "edit", "QwenImageEditPlusPipeline": "edit_plus"}

T2I_TEMPLATE = ("<|im_start|>system\nDescribe the image by detailing the color, shape, size, texture, quantity, "
                "text, spatial relationships of the objects and background:<|im_end|>\n<|im_start|>user\n{}"
                "<|im_end|>\n<|im_start|>assistant\n")
EDIT_TEMPLATE = ("<|im_start|>system\nDescribe the key features of the input image (color, shape, size, texture, "
                 "objects, background), then explain how the user's text instruction should alter or modify the "
                 "image. Generate a new image that meets the user's requirements while maintaining consistency "
                 "with the original input where appropriate.<|im_end|>\n<|im_start|>user\n{}<|im_end|>\n"
                 "<|im_start|>assistant\n")
VISION_SLOT = "<|vision_start|><|image_pad|><|vision_end|>"
DROP = {"t2i": 34, "edit": 64, "edit_plus": 64}

# random-init architectures (weights synthetic; shapes of the named checkpoints)
PRESETS = {
    "qwen-image": dict(transformer=dict(num_layers=60, num_attention_heads=24, attention_head_dim=128,
                                        joint_attention_dim=3584, in_channels=64, out_channels=16, patch_size=2,
                                        axes_dims_rope=[16, 56, 56]),
                       vae=dict(base_dim=96, z_dim=16, dim_mult=[1, 2, 4, 4], num_res_blocks=2),
                       text_encoder="qwen2.5-vl-7b"),
    "tiny-qwen-image": dict(transformer=dict(num_layers=2, num_attention_heads=2, attention_head_dim=64,
                                             joint_attention_dim=256, in_channels=64, out_channels=16, patch_size=2,
                                             axes_dims_rope=[16, 24, 24]),
                            vae=dict(base_dim=16, z_dim=16, dim_mult=[1, 2, 2, 2], num_res_blocks=1),
                            text_encoder="tiny-qwen2.5-vl"),
}


def calculate_dimensions(area: int, ratio: float, unit: int = 32) -> tuple[int, int]:
    """(width, height) with about ``area`` pixels at aspect ``ratio`` (w / h), multiples of ``unit``."""
    w = math.sqrt(area * ratio)
    h = w / ratio
    return max(unit, round(w / unit) * unit), max(unit, round(h / unit) * unit)


def pack(lat: torch.Tensor) -> torch.Tensor:
    """[B, C, h, w] -> [B, (h/2)(w/2), 4C] (2x2 patches, channel-major inside a patch)."""
    B, C, h, w = lat.shape
    return lat.view(B, C, h // 2, 2, w // 2, 2).permute(0, 2, 4, 1, 3, 5).reshape(B, (h // 2) * (w // 2), C * 4)


def unpack(x: torch.Tensor, h: int, w: int) -> torch.Tensor:
    B, N, C4 = x.shape
    C = C4 // 4
    return x.view(B, h // 2, w // 2, C, 2, 2).permute(0, 3, 1, 4, 2, 5).reshape(B, C, h, w)


def _tiny_text_encoder_cfg() -> dict:
    return dict(architectures=["Qwen2_5_VLForConditionalGeneration"], model_type="qwen2_5_vl", hidden_size=256,
                num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, intermediate_size=512,
                vocab_size=152064, rms_norm_eps=1e-6, rope_theta=1000000.0, max_position_embeddings=4096,
                rope_scaling={"type": "mrope", "mrope_section": [8, 12, 12]}, image_token_id=151655,
                video_token_id=151656, vision_start_token_id=151652, vision_end_token_id=151653,
                vision_config=dict(depth=2, hidden_size=64, num_heads=2, intermediate_size=96, patch_size=14,
                                   spatial_merge_size=2, temporal_patch_size=2, in_channels=3, window_size=112,
                                   fullatt_block_indexes=[1], out_hidden_size=256, hidden_act="silu"))


class QwenImagePipeline:
    def __init__(self, dit: QwenImageDiT, vae: QwenImageVAE, text_encoder, tokenizer, kind: str = "t2i",
                 sched: FlowMatchConfig | None = None):
        self.dit, self.vae, self.te, self.tok, self.kind = dit, vae, text_encoder, tokenizer, kind
        self.sched = sched or FlowMatchConfig()
        self.device, self.dtype = dit.device, dit.dtype
        self.stats = {"images": 0, "steps": 0, "seconds": 0.0}

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_pretrained(cls, path: str, device="cuda", dtype=torch.bfloat16) -> "QwenImagePipeline":
        from ome_amd.models import build_model
        from ome_amd.models.config import ModelConfig
        from ome_amd.models.loader import iter_safetensors

        root = Path(path)
        idx = json.loads((root / "model_index.json").read_text())
        kind = PIPELINES.get(idx.get("_class_name", "QwenImagePipeline"), "t2i")
        dit = QwenImageDiT(json.loads((root / "transformer" / "config.json").read_text()), device, dtype)
        dit.load(iter_safetensors(str(root / "transformer"), device="cpu"))
        vae = QwenImageVAE(json.loads((root / "vae" / "config.json").read_text()), device, dtype)
        vae.load(iter_safetensors(str(root / "vae"), device="cpu"),
                 ("encoder", "decoder") if kind != "t2i" else ("decoder",))
        te_dir = root / "text_encoder"
        te = build_model(ModelConfig.from_path(te_dir), device, dtype, model_path=str(te_dir))
        sc = root / "scheduler" / "scheduler_config.json"
        sched = FlowMatchConfig.from_dict(json.loads(sc.read_text())) if sc.exists() else None
        return cls(dit, vae, te, _load_tokenizer(root / "tokenizer", te.cfg.vocab_size), kind, sched)

    @classmethod
    def random(cls, preset: str = "tiny-qwen-image", kind: str = "t2i", device="cuda", dtype=torch.bfloat16,
               seed: int = 0) -> "QwenImagePipeline":
        from ome_amd.models import build_model
        from ome_amd.models.config import PRESETS as LM_PRESETS, ModelConfig

        p = PRESETS[preset]
        dit = QwenImageDiT(p["transformer"], device, dtype).init_random(seed)
        vae = QwenImageVAE(p["vae"], device, dtype).init_random(seed + 1)
        te_cfg = LM_PRESETS.get(p["text_encoder"])
        if te_cfg is None:
            if not p["text_encoder"].startswith("tiny-"):
                raise KeyError(f"text encoder preset {p['text_encoder']!r} missing")
            te_cfg = _tiny_text_encoder_cfg()
        te = build_model(ModelConfig.from_hf(te_cfg), device, dtype, load_format="dummy", seed=seed + 2)
        from ome_amd.runtime.tokenizer import ByteTokenizer

        return cls(dit, vae, te, ByteTokenizer(te.cfg.vocab_size), kind)

    # ------------------------------------------------------------------ text encoder
    def _hidden(self, ids: list[int], images: list | None = None) -> torch.Tensor:
        """Final normed hidden states [T, H] of one prompt (images: PIL / arrays for the VL tower)."""
        m, dev = self.te, self.device
        pos3 = feats = rows = None
        if images:
            from ome_amd.multimodal import expand_image_tokens, mrope_positions
            from ome_amd.multimodal.inputs import preprocess_image

            pvs, grids = [], []
            for im in images:
                pv, g = preprocess_image(im, patch=m.visual.patch, merge=m.merge, temporal=m.visual.temporal)
                pvs.append(torch.as_tensor(pv, dtype=torch.float32))
                grids.append(tuple(int(v) for v in g))
            ids, spans = expand_image_tokens(list(ids), m.image_token_id, grids, m.merge, pvs, m.cfg.vocab_size)
            pos3, _ = mrope_positions(len(ids), spans, grids, m.merge)
            feats = m.encode_images(torch.cat(pvs, 0), grids)
            rows = torch.cat([torch.arange(s, s + n) for s, n in spans]).to(dev)
        T = len(ids)
        P = 16
        npg = -(-T // P)
        kv = PagedKVCache(m.cfg.num_layers, npg + 1, m.tp.hkv, m.D, P, self.dtype, dev)
        t = lambda a: torch.tensor(a, dtype=torch.int32, device=dev)  # noqa: E731
        pages = list(range(1, npg + 1))
        meta = AttnMeta("prefill", t(list(range(T))), t([pages[i // P] * P + i % P for i in range(T)]), t([pages]),
                        cu_q=t([0, T]), kv_lens=t([T]), items=t(ops.prefill_work_items([T], [T])).view(-1, 2))
        ids_t = t(ids)
        emb = None
        if images:
            emb = m.embed_with_images(ids_t, rows, feats)
            meta.extra["rope"] = (torch.arange(T, dtype=torch.int32, device=dev),
                                  m.mrope_table(torch.from_numpy(pos3)))
        return m.forward(ids_t, meta, kv, emb)

    def encode_prompt(self, prompt: str, images: list | None = None) -> torch.Tensor:
        if self.kind == "t2i":
            text = T2I_TEMPLATE.format(prompt)
        elif self.kind == "edit":
            text = EDIT_TEMPLATE.format(VISION_SLOT * len(images or []) + prompt)
        else:
            slots = "".join(f"Picture {i + 1}: {VISION_SLOT}" for i in range(len(images or [])))
            text = EDIT_TEMPLATE.format(slots + prompt)
        # the vision slots as the text encoder's own special ids (any tokenizer, incl. the byte one)
        m, parts = self.te, text.split(VISION_SLOT)
        ids = list(self.tok.encode(parts[0]))
        for seg in parts[1:]:
            ids += [m.vision_start_id, m.image_token_id, m.vision_end_id] + list(self.tok.encode(seg))
        h = self._hidden(ids, images)
        return h[DROP[self.kind]:] if h.shape[0] > DROP[self.kind] else h[-1:]

    # ------------------------------------------------------------------ generation
    @torch.no_grad()
    def __call__(self, prompt: str, negative_prompt: str | None = None, width: int = 1024, height: int = 1024,
                 steps: int = 50, true_cfg_scale: float = 4.0, seed: int = 0, images: list | None = None,
                 latents: torch.Tensor | None = None) -> np.ndarray:
        """-> uint8 [height, width, 3]."""
        t0 = time.perf_counter()
        mult = 16   # VAE 8x * 2x2 patches
        width, height = max(mult, width // mult * mult), max(mult, height // mult * mult)
        h, w = height // 8, width // 8
        cond_imgs = images or []
        if self.kind != "t2i" and not cond_imgs:
            raise ValueError("the edit pipelines need an input image")
        vl_imgs, img_lat, shapes = None, [], [(1, h // 2, w // 2)]
        if cond_imgs:
            from ome_amd.multimodal.inputs import load_image

            pil = [load_image(im) for im in cond_imgs]
            vl_area = 384 * 384 if self.kind == "edit_plus" else 1024 * 1024
            vl_imgs = [im.resize(calculate_dimensions(vl_area, im.width / im.height)) for im in pil]
            for im in pil:
                vw, vh = calculate_dimensions(1024 * 1024, im.width / im.height)
                a = np.asarray(im.convert("RGB").resize((vw, vh)), dtype=np.float32) / 127.5 - 1.0
                z = self.vae.encode(torch.from_numpy(a.transpose(2, 0, 1))[None].to(self.device))
                img_lat.append(pack(z.to(self.dtype)))
                shapes.append((1, vh // 16, vw // 16))
        txt = [self.encode_prompt(prompt, vl_imgs)]
        cfg = true_cfg_scale > 1.0 and negative_prompt is not None
        if cfg:
            txt.append(self.encode_prompt(negative_prompt, vl_imgs))
        g = torch.Generator(device="cpu").manual_seed(int(seed))
        if latents is None:
            latents = torch.randn(1, self.dit.cout, h, w, generator=g)
        x = pack(latents.to(self.device, torch.float32))
        N = x.shape[1]
        sch = FlowMatchEuler(self.sched)
        ts = sch.set_timesteps(steps, N)
        cond = torch.cat(img_lat, 1) if img_lat else None
        for i, t in enumerate(ts):
            inp = x.to(self.dtype) if cond is None else torch.cat([x.to(self.dtype), cond], 1)
            B = len(txt)
            out = self.dit.forward(inp.expand(B, -1, -1).contiguous(), txt,
                                   torch.full((B,), t / 1000.0, device=self.device), shapes)[:, :N].float()
            v = out[0:1]
            if cfg:
                comb = out[1:2] + true_cfg_scale * (out[0:1] - out[1:2])
                v = comb * (out[0:1].norm(dim=-1, keepdim=True) / comb.norm(dim=-1, keepdim=True).clamp_min(1e-12))
            x = sch.step(v, i, x)
        img = self.vae.decode(unpack(x, h, w))[0]
        self.stats["images"] += 1
        self.stats["steps"] += steps
        self.stats["seconds"] += time.perf_counter() - t0
        return ((img.permute(1, 2, 0).cpu().numpy() + 1.0) * 127.5).round().clip(0, 255).astype(np.uint8)


def _load_tokenizer(path: Path, vocab: int):
    from ome_amd.runtime.tokenizer import ByteTokenizer, HFTokenizer

    if (path / "tokenizer.json").exists():
        return HFTokenizer(path)
    if (path / "vocab.json").exists():
        try:
            from transformers import AutoTokenizer

            t = AutoTokenizer.from_pretrained(str(path), local_files_only=True)

            class _Wrap:
                def encode(self, text: str, add_bos: bool = False):
                    return t.encode(text, add_special_tokens=False)

            return _Wrap()
        except Exception:  # noqa: BLE001 - fall back to bytes
            pass
    return ByteTokenizer(vocab)

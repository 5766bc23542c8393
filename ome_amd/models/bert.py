"""BERT / RoBERTa / XLM-RoBERTa encoders: text embeddings and cross-encoder rerankers.

The reference serves these through SGLang ``--is-embedding`` runtimes:
``config/runtimes/srt/BAAI/bge-large-en-v1-5-rt.yaml`` (``BertModel``),
``config/runtimes/srt/BAAI/bge-m3-rt.yaml`` (``XLMRobertaModel``) and
``config/runtimes/srt/BAAI/bge-reranker-v2-m3-rt.yaml`` (``XLMRobertaForSequenceClassification``),
with ``pkg/hfutil/modelconfig/bert.go`` parsing the configs.

Encoder layer (post-LayerNorm), per step over the packed prompts of a batch:
  fused QKV GEMM (+bias, hipBLASLt) -> varlen bidirectional MFMA attention read in place from the
  QKV output (``csrc/kernels/varlen_attn.hip``) -> O GEMM -> fused residual-add + LayerNorm
  (``ome_layernorm``) -> up GEMM -> exact GELU (``ome_act``) -> down GEMM -> fused add + LayerNorm.
No KV cache (``kv_layers`` is empty) and no decode graphs: an encoder request is one forward.

Pooling: ``*Model`` embedders take the first token ([CLS] / <s>) and L2-normalise it (the
``ome_pool`` kernel, mode 2); ``XLMRobertaForSequenceClassification`` applies its
dense-tanh-out_proj head to the first token, ``BertForSequenceClassification`` its
pooler + classifier; the raw logits are returned (rerank relevance = logit 0).
Weights are replicated across tensor-parallel ranks (encoders of this size fit one GPU many
times over; no collective is needed).
"""
from __future__ import annotations

import math
import re

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.quant import linear

ENCODER_ARCHS = {"BertModel", "BertForSequenceClassification", "RobertaModel", "RobertaForSequenceClassification",
                 "XLMRobertaModel", "XLMRobertaForSequenceClassification"}

_ACT = {"gelu": 3, "gelu_new": 1, "gelu_pytorch_tanh": 1, "relu": 5, "silu": 0}


class _TP:
    """Replicated shapes (the runner reads ``hq`` / ``hkv``)."""

    def __init__(self, cfg: ModelConfig):
        self.tp, self.rank = 1, 0
        self.hq = self.hkv = cfg.num_heads
        self.vocab, self.vocab_start, self.vocab_end = cfg.vocab_size, 0, cfg.vocab_size


class EncoderModel:
    encoder_only = True
    tune_gemms = False

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        hf = cfg.extra or {}
        self.cfg, self.device, self.dtype = cfg, torch.device(device), dtype
        self.tp = _TP(cfg)
        self.H, self.nh = cfg.hidden_size, cfg.num_heads
        self.D = self.H // self.nh
        if self.D % 8 or self.D > 128:
            raise NotImplementedError(f"encoder head dim {self.D} (multiple of 8, <= 128)")
        self.scale = 1.0 / math.sqrt(self.D)
        self.eps = float(hf.get("layer_norm_eps", 1e-12))
        self.act = _ACT.get(str(hf.get("hidden_act", "gelu")), 3)
        arch = cfg.architecture
        self.roberta = "Roberta" in arch or cfg.model_type in ("roberta", "xlm-roberta")
        # RoBERTa positions count from padding_idx + 1 (create_position_ids_from_input_ids)
        self.pos_offset = int(hf.get("pad_token_id", 1)) + 1 if self.roberta else 0
        self.head = "roberta_cls" if arch.endswith("ForSequenceClassification") and self.roberta else \
            "bert_cls" if arch.endswith("ForSequenceClassification") else "embed"
        self.num_labels = int(hf.get("num_labels") or len(hf.get("id2label") or {}) or 1) if self.head != "embed" else 0
        L = cfg.num_layers
        self.layers = list(range(L))
        self.kv_layers: list[int] = []   # no KV cache
        self.w_qkv, self.b_qkv, self.w_o, self.b_o = [None] * L, [None] * L, [None] * L, [None] * L
        self.ln1_w, self.ln1_b, self.ln2_w, self.ln2_b = [None] * L, [None] * L, [None] * L, [None] * L
        self.w_up, self.b_up, self.w_dn, self.b_dn = [None] * L, [None] * L, [None] * L, [None] * L
        self.word = self.pos = self.ttype = self.emb_ln_w = self.emb_ln_b = None
        self.pool_w = self.pool_b = None     # BERT pooler (tanh dense on the first token)
        self.cls_w = self.cls_b = None       # RoBERTa head dense / BERT classifier
        self.out_w = self.out_b = None       # RoBERTa head out_proj

    # ------------------------------------------------------------------ weights
    def _t(self, x: torch.Tensor) -> torch.Tensor:
        return x.to(device=self.device, dtype=self.dtype).contiguous()

    def init_random(self, seed: int = 0, std: float = 0.02) -> "EncoderModel":
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        hf = self.cfg.extra or {}
        H, I, V = self.H, self.cfg.intermediate_size, self.cfg.vocab_size

        def rnd(*s):
            return self._t(torch.randn(*s, generator=g) * std)

        ones, zeros = (lambda n: self._t(torch.ones(n))), (lambda n: self._t(torch.zeros(n)))
        self.word = rnd(V, H)
        self.pos = rnd(int(hf.get("max_position_embeddings", 512)), H)
        self.ttype = rnd(max(1, int(hf.get("type_vocab_size", 2))), H)
        self.emb_ln_w, self.emb_ln_b = ones(H), zeros(H)
        for i in self.layers:
            self.w_qkv[i], self.b_qkv[i] = rnd(3 * H, H), zeros(3 * H)
            self.w_o[i], self.b_o[i] = rnd(H, H), zeros(H)
            self.w_up[i], self.b_up[i] = rnd(I, H), zeros(I)
            self.w_dn[i], self.b_dn[i] = rnd(H, I), zeros(H)
            self.ln1_w[i], self.ln1_b[i], self.ln2_w[i], self.ln2_b[i] = ones(H), zeros(H), ones(H), zeros(H)
        if self.head == "roberta_cls":
            self.cls_w, self.cls_b = rnd(H, H), zeros(H)
            self.out_w, self.out_b = rnd(self.num_labels, H), zeros(self.num_labels)
        else:
            self.pool_w, self.pool_b = rnd(H, H), zeros(H)
            if self.head == "bert_cls":
                self.cls_w, self.cls_b = rnd(self.num_labels, H), zeros(self.num_labels)
        return self

    _LAYER = re.compile(r"encoder\.layer\.(\d+)\.(.+)")

    def load_hf_weights(self, weights) -> "EncoderModel":
        per: dict[int, dict[str, torch.Tensor]] = {}
        for name, t in weights:
            n = re.sub(r"^(bert|roberta|model)\.", "", name)
            m = self._LAYER.match(n)
            if m:
                per.setdefault(int(m.group(1)), {})[m.group(2)] = t
                continue
            put = {"embeddings.word_embeddings.weight": "word", "embeddings.position_embeddings.weight": "pos",
                   "embeddings.token_type_embeddings.weight": "ttype", "embeddings.LayerNorm.weight": "emb_ln_w",
                   "embeddings.LayerNorm.bias": "emb_ln_b", "pooler.dense.weight": "pool_w",
                   "pooler.dense.bias": "pool_b", "classifier.out_proj.weight": "out_w",
                   "classifier.out_proj.bias": "out_b"}.get(n)
            if n in ("classifier.dense.weight", "classifier.weight"):
                put = "cls_w"
            elif n in ("classifier.dense.bias", "classifier.bias"):
                put = "cls_b"
            if put is not None:
                setattr(self, put, self._t(t))
        for i in self.layers:
            p = per.get(i)
            if p is None:
                raise ValueError(f"encoder layer {i} missing from the checkpoint")
            a = "attention.self."
            self.w_qkv[i] = self._t(torch.cat([p[a + "query.weight"], p[a + "key.weight"], p[a + "value.weight"]]))
            self.b_qkv[i] = self._t(torch.cat([p[a + "query.bias"], p[a + "key.bias"], p[a + "value.bias"]]))
            self.w_o[i], self.b_o[i] = self._t(p["attention.output.dense.weight"]), self._t(p["attention.output.dense.bias"])
            self.ln1_w[i] = self._t(p["attention.output.LayerNorm.weight"])
            self.ln1_b[i] = self._t(p["attention.output.LayerNorm.bias"])
            self.w_up[i], self.b_up[i] = self._t(p["intermediate.dense.weight"]), self._t(p["intermediate.dense.bias"])
            self.w_dn[i], self.b_dn[i] = self._t(p["output.dense.weight"]), self._t(p["output.dense.bias"])
            self.ln2_w[i], self.ln2_b[i] = self._t(p["output.LayerNorm.weight"]), self._t(p["output.LayerNorm.bias"])
        if self.ttype is None:
            self.ttype = self._t(torch.zeros(1, self.H))
        return self

    def weight_bytes(self) -> int:
        n = 0
        for v in vars(self).values():
            if isinstance(v, torch.Tensor):
                n += v.numel() * v.element_size()
            elif isinstance(v, list):
                n += sum(t.numel() * t.element_size() for t in v if isinstance(t, torch.Tensor))
        return n

    # ------------------------------------------------------------------ forward
    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache | None = None) -> torch.Tensor:
        lengths = meta.extra.get("lengths")
        if lengths is None:
            cu = meta.cu_q.tolist()
            lengths = [b - a for a, b in zip(cu[:-1], cu[1:])]
        pos = meta.positions.long() + self.pos_offset
        x = F.embedding(ids.long(), self.word) + F.embedding(pos, self.pos) + self.ttype[0]
        x = ops.layernorm(x.contiguous(), self.emb_ln_w, self.emb_ln_b, self.eps)
        T, H, nh, D = x.shape[0], self.H, self.nh, self.D
        for i in self.layers:
            qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
            q, k, v = (qkv[:, j * H:(j + 1) * H].view(T, nh, D) for j in range(3))
            a = ops.varlen_attention(q, k, v, lengths, self.scale)
            o = linear(a.view(T, H), self.w_o[i], self.b_o[i])
            ops.fused_add_layernorm(o, x, self.ln1_w[i], self.ln1_b[i], self.eps)  # o <- LN(x + o)
            h = ops.act(linear(o, self.w_up[i], self.b_up[i]), self.act)
            y = linear(h, self.w_dn[i], self.b_dn[i])
            ops.fused_add_layernorm(y, o, self.ln2_w[i], self.ln2_b[i], self.eps)
            x = y
        return x

    def pool(self, hidden: torch.Tensor, cu: torch.Tensor) -> torch.Tensor:
        if self.head == "embed":
            return ops.pool(hidden, cu, 2, True)
        first = hidden.index_select(0, cu[:-1].long())
        if self.head == "roberta_cls":
            h = torch.tanh(linear(first, self.cls_w, self.cls_b))
            return linear(h, self.out_w, self.out_b).float()
        pooled = torch.tanh(linear(first, self.pool_w, self.pool_b))
        return linear(pooled, self.cls_w, self.cls_b).float()

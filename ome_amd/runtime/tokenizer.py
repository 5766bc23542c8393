"""Tokenizers: HF ``tokenizer.json`` via the ``tokenizers`` library when the model directory has
one; otherwise a deterministic byte-level tokenizer (random-init benchmark models ship no
vocabulary — the token ids, not the text, are what the engine computes on)."""
from __future__ import annotations

import json
from pathlib import Path


class ByteTokenizer:
    """id = byte + 3 (0 = <pad>, 1 = <bos>, 2 = <eos>); ids >= 259 decode to a printable stand-in."""

    def __init__(self, vocab_size: int = 128256):
        self.vocab_size = vocab_size
        self.bos_token_id, self.eos_token_id, self.pad_token_id = 1, 2, 0

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = [b + 3 for b in text.encode("utf-8")]
        return ([self.bos_token_id] if add_bos else []) + ids

    def encode_special(self, text: str, pair: str | None = None) -> list[int]:
        """Encoder input: <bos> text <eos> [pair <eos>] (the [CLS] / [SEP] stand-ins)."""
        ids = [self.bos_token_id] + self.encode(text) + [self.eos_token_id]
        if pair is not None:
            ids += self.encode(pair) + [self.eos_token_id]
        return ids

    def decode(self, ids, skip_special: bool = True) -> str:
        out = bytearray()
        for i in ids:
            i = int(i)
            if 3 <= i < 259:
                out.append(i - 3)
            elif i >= 259:
                out.extend(chr(0x4E00 + (i % 20000)).encode())
            elif not skip_special:
                out.extend(f"<{i}>".encode())
        return out.decode("utf-8", errors="replace")

    def special_strings(self) -> list[str]:
        return [f"<{i}>" for i in range(3)]

    def apply_chat_template(self, messages: list[dict], add_generation_prompt: bool = True, tools=None) -> str:
        parts = []
        if tools:
            parts.append("<|tools|>\n" + json.dumps(tools) + "\n")
        for m in messages:
            content = m.get("content", "")
            if isinstance(content, list):
                content = "".join(c.get("text", "") for c in content if isinstance(c, dict))
            parts.append(f"<|{m.get('role', 'user')}|>\n{content}\n")
        if add_generation_prompt:
            parts.append("<|assistant|>\n")
        return "".join(parts)


class HFTokenizer:
    def __init__(self, path: Path):
        from tokenizers import Tokenizer

        self.tok = Tokenizer.from_file(str(path / "tokenizer.json"))
        self.vocab_size = self.tok.get_vocab_size()
        cfg = {}
        if (path / "tokenizer_config.json").exists():
            cfg = json.loads((path / "tokenizer_config.json").read_text())
        self.chat_template = cfg.get("chat_template")

        def tid(name):
            v = cfg.get(name)
            if isinstance(v, dict):
                v = v.get("content")
            return self.tok.token_to_id(v) if v else None

        self.bos_token_id = tid("bos_token")
        self.eos_token_id = tid("eos_token")
        self.pad_token_id = tid("pad_token")

    def encode(self, text: str, add_bos: bool = False) -> list[int]:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        if add_bos and self.bos_token_id is not None:
            ids = [self.bos_token_id] + ids
        return ids

    def encode_special(self, text: str, pair: str | None = None) -> list[int]:
        """Encoder input with the tokenizer's own post-processor: [CLS] a [SEP] (b [SEP]) for BERT,
        <s> a </s></s> b </s> for (XLM-)RoBERTa."""
        return self.tok.encode(text, pair, add_special_tokens=True).ids

    def decode(self, ids, skip_special: bool = True) -> str:
        return self.tok.decode([int(i) for i in ids], skip_special_tokens=skip_special)

    def special_strings(self) -> list[str]:
        try:
            return [t.content for t in self.tok.get_added_tokens_decoder().values() if t.special]
        except AttributeError:  # older tokenizers releases
            return []

    def apply_chat_template(self, messages: list[dict], add_generation_prompt: bool = True, tools=None) -> str:
        if self.chat_template:
            try:
                import jinja2

                env = jinja2.Environment()
                env.filters.setdefault("tojson", lambda v, indent=None: json.dumps(v, indent=indent))
                t = env.from_string(self.chat_template)
                return t.render(messages=messages, add_generation_prompt=add_generation_prompt, bos_token="",
                                tools=tools)
            except Exception:  # noqa: BLE001 — template dialects vary; fall back to plain format
                pass
        return ByteTokenizer.apply_chat_template(self, messages, add_generation_prompt, tools)  # type: ignore[arg-type]


def get_tokenizer(model_path: str | None, vocab_size: int = 128256):
    if model_path and (Path(model_path) / "tokenizer.json").exists():
        return HFTokenizer(Path(model_path))
    return ByteTokenizer(vocab_size)

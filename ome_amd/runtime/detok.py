"""Incremental detokenisation for streamed responses.

Decoding the whole output on every streamed token is O(n^2) in the output length (the verdict on
``runtime/server.py``).  :class:`IncrementalDetokenizer` keeps two offsets into the token list,
the same scheme SGLang / vLLM use: ``prefix`` (start of a short context window, needed because
byte-level BPE and SentencePiece merge spaces / multi-byte characters across tokens) and
``read`` (tokens already emitted).  Each push decodes only ``ids[prefix:]`` -- a few tokens --
and emits the text past ``decode(ids[prefix:read])``; a trailing U+FFFD (an incomplete UTF-8
sequence) is held back until the next token completes it.

With ``skip_special=False`` special tokens come through as text (tool / reasoning parsers need
the harmony ``<|channel|>`` / ``<|message|>`` / ``<|call|>`` and Mistral ``[TOOL_CALLS]``
markers); :func:`strip_special` removes them from what is finally shown to the client.
"""
from __future__ import annotations

_WINDOW = 6   # tokens of left context kept for the merge rules


class IncrementalDetokenizer:
    def __init__(self, tok, skip_special: bool = True):
        self.tok = tok
        self.skip = skip_special
        self.ids: list[int] = []
        self.prefix = 0
        self.read = 0
        self.text = ""

    _cache: tuple | None = None   # (prefix, end, text): the last decode of ids[prefix:end]

    def _decode(self, a: int, b: int) -> str:
        c = self._cache
        if c is not None and c[0] == a and c[1] == b:
            return c[2]
        return self.tok.decode(self.ids[a:b], skip_special=self.skip)

    def push(self, new_ids) -> str:
        """Append tokens; return the newly completed text (may be "").

        One tokenizer call per push in the steady state: the context window only slides in
        jumps (when it has grown to twice ``_WINDOW``), so ``decode(ids[prefix:read])`` is
        usually the previous push's ``after`` and comes from the cache."""
        self.ids.extend(int(t) for t in new_ids)
        if self.read >= len(self.ids):
            return ""
        before = self._decode(self.prefix, self.read)
        after = self.tok.decode(self.ids[self.prefix:], skip_special=self.skip)
        self._cache = (self.prefix, len(self.ids), after)
        if len(after) <= len(before) or after.endswith("\ufffd"):
            return ""   # nothing new yet, or an incomplete multi-byte character
        delta = after[len(before):]
        self.read = len(self.ids)
        if self.read - self.prefix >= 2 * _WINDOW:
            self.prefix = self.read - _WINDOW
        self.text += delta
        return delta

    def flush(self) -> str:
        """End of stream: emit whatever is still held back (replacement characters included)."""
        if self.read >= len(self.ids):
            return ""
        before = self.tok.decode(self.ids[self.prefix:self.read], skip_special=self.skip)
        after = self.tok.decode(self.ids[self.prefix:], skip_special=self.skip)
        delta = after[len(before):]
        self.read = len(self.ids)
        self.text += delta
        return delta


def special_strings(tok) -> list[str]:
    """The text forms of the tokenizer's special tokens (longest first)."""
    fn = getattr(tok, "special_strings", None)
    return sorted(fn() if fn else [], key=len, reverse=True)


def strip_special(text: str | None, specials: list[str]) -> str | None:
    if not text:
        return text
    for s in specials:
        if s and s in text:
            text = text.replace(s, "")
    return text


class StopMatcher:
    """Stop strings checked against the tail of the text only (each new delta plus the longest
    stop string's length of look-behind), not the whole output per token."""

    def __init__(self, stops: list[str] | None):
        self.stops = [s for s in (stops or []) if s]
        self.back = max((len(s) for s in self.stops), default=0)

    def find(self, text: str, new_len: int) -> int | None:
        """Index of the first stop string in ``text`` that ends inside the last ``new_len``
        characters, or None."""
        if not self.stops:
            return None
        lo = max(0, len(text) - new_len - self.back)
        tail = text[lo:]
        idx = [tail.find(s) for s in self.stops if s in tail]
        return lo + min(idx) if idx else None

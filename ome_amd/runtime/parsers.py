"""Reasoning and tool-call parsers for the OpenAI-compatible chat API.

The reference's runtimes turn these on per model family with SGLang flags, e.g.
``--tool-call-parser llama3_json`` (Llama 3.x), ``pythonic`` (Llama 4), ``qwen3_coder``,
``nano_v3`` (Nemotron Nano), ``gpt-oss``; ``--reasoning-parser deepseek-r1`` / ``qwen3`` /
``gpt-oss`` (``config/runtimes/srt/**``).  Same flags here (``runtime/server.py``):

* a reasoning parser splits ``reasoning_content`` from ``content`` -- non-streaming
  (:meth:`ReasoningParser.split`) and incrementally for SSE deltas (:meth:`ReasoningParser.feed`,
  holding back any suffix that could still become a marker);
* a tool parser extracts OpenAI ``tool_calls`` (``{"id", "type": "function", "function":
  {"name", "arguments": <JSON string>}}``) from the final text; when streaming, text is forwarded
  until a call marker appears and the calls are emitted as one delta at the end.
"""
from __future__ import annotations

import ast
import json
import re
import uuid

# ------------------------------------------------------------------ reasoning
_THINK = ("<think>", "</think>")


class ReasoningParser:
    """``deepseek-r1``: the generation prompt already opened ``<think>``, so output starts inside
    the reasoning block (an explicit ``<think>`` is tolerated).  ``qwen3`` / ``nano_v3`` / generic:
    reasoning only inside an explicit ``<think>...</think>``.  ``gpt-oss``: harmony channels --
    ``analysis`` is reasoning, ``final`` is content."""

    def __init__(self, kind: str):
        self.kind = kind.replace("_", "-")
        self.harmony = self.kind in ("gpt-oss", "harmony")
        self.in_reason = self.kind in ("deepseek-r1",)
        self.buf = ""
        self.started = False

    # -- non-streaming
    def split(self, text: str) -> tuple[str | None, str]:
        if self.harmony:
            return _harmony_split(text)
        start, end = _THINK
        t = text
        if self.kind == "deepseek-r1":
            t = t[t.index(start) + len(start):] if t.lstrip().startswith(start) else t
            if end not in t:
                return t.strip() or None, ""
            r, c = t.split(end, 1)
            return r.strip() or None, c.lstrip("\n")
        s = t.find(start)
        if s < 0 or t[:s].strip():
            return None, text
        rest = t[s + len(start):]
        if end not in rest:
            return rest.strip() or None, ""
        r, c = rest.split(end, 1)
        return r.strip() or None, c.lstrip("\n")

    # -- streaming: feed the new text, get (reasoning_delta, content_delta)
    def feed(self, delta: str) -> tuple[str, str]:
        if self.harmony:
            self.buf += delta
            r, c = _harmony_split(self.buf, partial=True)
            r, c = r or "", c or ""
            out = (r[len(getattr(self, "_sent_r", "")):], c[len(getattr(self, "_sent_c", "")):])
            self._sent_r, self._sent_c = r, c
            return out
        self.buf += delta
        start, end = _THINK
        reason, content = [], []
        while self.buf:
            if not self.started and not self.in_reason:
                stripped = self.buf.lstrip()
                if stripped.startswith(start):
                    self.buf = stripped[len(start):]
                    self.in_reason = self.started = True
                    continue
                if start.startswith(stripped) and stripped:
                    break               # could still be the opening tag
                self.started = True
                continue
            if self.in_reason:
                if not self.started:   # deepseek-r1: an explicit <think> may still open the output
                    st = self.buf.lstrip()
                    if st.startswith(start):
                        self.buf = st[len(start):]
                        self.started = True
                        continue
                    if st and start.startswith(st):
                        break
                self.started = True
                i = self.buf.find(end)
                if i >= 0:
                    reason.append(self.buf[:i])
                    self.buf = self.buf[i + len(end):].lstrip("\n")
                    self.in_reason = False
                    continue
                keep = _partial_suffix(self.buf, end)
                reason.append(self.buf[:len(self.buf) - keep])
                self.buf = self.buf[len(self.buf) - keep:]
                break
            content.append(self.buf)
            self.buf = ""
        return "".join(reason), "".join(content)

    def flush(self) -> tuple[str, str]:
        b, self.buf = self.buf, ""
        if self.harmony:
            return "", ""
        return (b, "") if self.in_reason else ("", b)


def _partial_suffix(text: str, marker: str) -> int:
    """Length of the longest suffix of ``text`` that is a proper prefix of ``marker``."""
    for k in range(min(len(marker) - 1, len(text)), 0, -1):
        if marker.startswith(text[-k:]):
            return k
    return 0


_HARMONY_MSG = re.compile(r"<\|channel\|>(\w+)(?:(?!<\|message\|>).)*<\|message\|>(.*?)(?=<\|end\|>|<\|return\|>|"
                          r"<\|call\|>|<\|start\|>|$)", re.S)


def _harmony_split(text: str, partial: bool = False) -> tuple[str | None, str]:
    if "<|channel|>" not in text:
        return None, ("" if partial and text.startswith("<|") else text)
    reason, content = [], []
    for ch, body in _HARMONY_MSG.findall(text):
        (reason if ch == "analysis" else content if ch == "final" else []).append(body)
    return ("".join(reason) or None), "".join(content)


# ------------------------------------------------------------------ tool calls
def _call(name: str, args) -> dict:
    if not isinstance(args, str):
        args = json.dumps(args, ensure_ascii=False)
    return {"id": f"call_{uuid.uuid4().hex[:24]}", "type": "function", "function": {"name": name, "arguments": args}}


def _json_objects(text: str) -> list:
    """Every top-level JSON value in ``text`` (objects / arrays), in order."""
    dec, out, i = json.JSONDecoder(), [], 0
    while i < len(text):
        j = min([k for k in (text.find("{", i), text.find("[", i)) if k >= 0], default=-1)
        if j < 0:
            break
        try:
            v, end = dec.raw_decode(text, j)
        except json.JSONDecodeError:
            i = j + 1
            continue
        out.append(v)
        i = end
    return out


def _from_dicts(objs) -> list[dict]:
    calls = []
    for o in objs:
        for d in (o if isinstance(o, list) else [o]):
            if isinstance(d, dict) and isinstance(d.get("name"), str):
                args = d.get("arguments", d.get("parameters", {}))
                calls.append(_call(d["name"], args))
    return calls


class ToolParser:
    MARKERS = {"llama3_json": ("<|python_tag|>", "{"), "pythonic": ("[",), "qwen3_coder": ("<tool_call>",),
               "hermes": ("<tool_call>",), "qwen25": ("<tool_call>",), "nano_v3": ("<TOOLCALL>",),
               "gpt-oss": ("<|channel|>commentary", " to=functions."), "mistral": ("[TOOL_CALLS]",)}

    def __init__(self, kind: str):
        if kind not in self.MARKERS:
            raise ValueError(f"unknown tool-call parser {kind!r} (have {sorted(self.MARKERS)})")
        self.kind = kind

    def start_index(self, text: str) -> int:
        """Where a tool call begins in the (partial) output, -1 if none yet (streaming cut point)."""
        if self.kind == "llama3_json":
            t = text.lstrip()
            if t.startswith("<|python_tag|>") or t.startswith("{"):
                return len(text) - len(t)
            return text.find("<|python_tag|>")
        if self.kind == "pythonic":
            t = text.lstrip()
            return len(text) - len(t) if t.startswith("[") else -1
        idx = [text.find(m) for m in self.MARKERS[self.kind] if m in text]
        return min(idx) if idx else -1

    def safe_len(self, text: str) -> int:
        """How much of ``text`` (no call found yet) can be streamed: hold back a suffix that may
        still grow into a call marker."""
        return len(text) - max((_partial_suffix(text, m) for m in self.MARKERS[self.kind]), default=0)

    def parse(self, text: str) -> tuple[str, list[dict]]:
        """-> (content without the calls, tool_calls)."""
        k = self.kind
        try:
            if k == "llama3_json":
                i = self.start_index(text)
                if i < 0:
                    return text, []
                body = text[i:].replace("<|python_tag|>", "")
                calls = _from_dicts(_json_objects(body))
                return (text[:i].strip(), calls) if calls else (text, [])
            if k == "pythonic":
                i = self.start_index(text)
                if i < 0:
                    return text, []
                src = text[i:].strip()
                src = src[:src.rfind("]") + 1]
                tree = ast.parse(src, mode="eval").body
                if not isinstance(tree, ast.List):
                    return text, []
                calls = []
                for c in tree.elts:
                    if not isinstance(c, ast.Call):
                        return text, []
                    name = ast.unparse(c.func)
                    calls.append(_call(name, {kw.arg: ast.literal_eval(kw.value) for kw in c.keywords}))
                return text[:i].strip(), calls
            if k in ("hermes", "qwen25"):
                blocks = re.findall(r"<tool_call>(.*?)(?:</tool_call>|$)", text, re.S)
                calls = _from_dicts([o for b in blocks for o in _json_objects(b)])
                return (text[:text.find("<tool_call>")].strip(), calls) if calls else (text, [])
            if k == "qwen3_coder":
                calls = []
                for fn, body in re.findall(r"<function=([^>\s]+)>(.*?)(?:</function>|$)", text, re.S):
                    args = {}
                    for pn, pv in re.findall(r"<parameter=([^>\s]+)>(.*?)(?:</parameter>|(?=<parameter=)|$)", body,
                                             re.S):
                        v = pv.strip("\n")
                        try:
                            args[pn] = json.loads(v)
                        except (json.JSONDecodeError, ValueError):
                            args[pn] = v
                    calls.append(_call(fn, args))
                i = text.find("<tool_call>")
                if i < 0:
                    i = text.find("<function=")
                return (text[:i].strip(), calls) if calls else (text, [])
            if k == "nano_v3":
                blocks = re.findall(r"<TOOLCALL>(.*?)(?:</TOOLCALL>|$)", text, re.S)
                calls = _from_dicts([o for b in blocks for o in _json_objects(b)])
                return (text[:text.find("<TOOLCALL>")].strip(), calls) if calls else (text, [])
            if k == "mistral":
                i = text.find("[TOOL_CALLS]")
                if i < 0:
                    return text, []
                calls = _from_dicts(_json_objects(text[i + len("[TOOL_CALLS]"):]))
                return (text[:i].strip(), calls) if calls else (text, [])
            if k == "gpt-oss":
                calls = []
                for name, body in re.findall(r"to=functions\.([\w.\-]+)(?:(?!<\|message\|>).)*<\|message\|>(.*?)"
                                             r"(?=<\|call\|>|<\|end\|>|<\|start\|>|$)", text, re.S):
                    objs = _json_objects(body)
                    calls.append(_call(name, objs[0] if objs else body.strip()))
                if not calls:
                    return text, []
                _, content = _harmony_split(text)
                return content, calls
        except (SyntaxError, ValueError):
            return text, []
        return text, []

"""Kubernetes resource.Quantity parsing ("288Gi", "500m", "1.5e3", "8T")."""
from __future__ import annotations

import re
from decimal import Decimal

_BIN = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DEC = {"n": Decimal("1e-9"), "u": Decimal("1e-6"), "m": Decimal("1e-3"), "": Decimal(1), "k": Decimal(10**3),
        "M": Decimal(10**6), "G": Decimal(10**9), "T": Decimal(10**12), "P": Decimal(10**15), "E": Decimal(10**18)}
_RE = re.compile(r"^([+-]?[0-9.]+(?:[eE][+-]?[0-9]+)?)(Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E)?$")


def parse_quantity(q) -> Decimal:
    if q is None:
        raise ValueError("empty quantity")
    if isinstance(q, (int, float)):
        return Decimal(str(q))
    s = str(q).strip()
    m = _RE.match(s)
    if not m:
        raise ValueError(f"invalid quantity {q!r}")
    num, suf = Decimal(m.group(1)), m.group(2) or ""
    if suf in _BIN:
        return num * _BIN[suf]
    return num * _DEC[suf]


def to_float(q, default: float = 0.0) -> float:
    try:
        return float(parse_quantity(q))
    except (ValueError, TypeError):
        return default


def to_gib(q) -> float:
    return to_float(q) / 2**30


def format_bytes(n: float) -> str:
    for u, f in (("Ti", 2**40), ("Gi", 2**30), ("Mi", 2**20), ("Ki", 2**10)):
        if n >= f:
            return f"{n / f:.0f}{u}"
    return str(int(n))

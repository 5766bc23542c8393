"""Model / framework version parsing with precision and major-prefix semantics.

Behaviour parity with ``pkg/modelver/util.go``: ``[v]MAJOR[.MINOR[.PATCH[.devN][-pre][+build]]]``;
``precision`` = number of dotted parts given; only lowercase ``v`` is an accepted major prefix;
numeric parts reject leading zeroes.  Ordering compares major/minor/patch numerically, then
the pre / build / dev identifier lists lexicographically (shorter list first on ties).
"""
from __future__ import annotations

from dataclasses import dataclass, field


class VersionError(ValueError):
    pass


@dataclass(frozen=True)
class Version:
    major: int
    minor: int = 0
    patch: int = 0
    major_prefix: str = ""
    pre: tuple[str, ...] = field(default_factory=tuple)
    build: tuple[str, ...] = field(default_factory=tuple)
    dev: tuple[str, ...] = field(default_factory=tuple)
    precision: int = 3

    @property
    def unofficial(self) -> bool:
        return bool(self.pre or self.build or self.dev)


def _num(s: str, what: str) -> int:
    if not s or not s.isdigit() or not s.isascii():
        raise VersionError(f"invalid character(s) in {what} number {s!r}")
    if len(s) > 1 and s[0] == "0":
        raise VersionError(f"{what} must not have leading zeroes: {s!r}")
    return int(s)


def _ids(s: str, what: str) -> tuple[str, ...]:
    parts = tuple(s.split("."))
    if any(p == "" for p in parts):
        raise VersionError(f"{what} meta data is empty")
    return parts


def parse(s: str) -> Version:
    if not s:
        raise VersionError("version string empty")
    parts = s.split(".", 2)
    precision = len(parts)
    major_s, prefix = parts[0], ""
    if major_s.startswith("v"):
        prefix, major_s = "v", major_s[1:]
    major = _num(major_s, "major")
    minor = _num(parts[1], "minor") if precision > 1 else 0
    rest = parts[2] if precision > 2 else "0"
    build = pre = dev = ()
    if "+" in rest:
        rest, b = rest.split("+", 1)
        build = _ids(b, "build")
    if "-" in rest:
        rest, p = rest.split("-", 1)
        pre = _ids(p, "prerelease")
    if "." in rest:
        rest, d = rest.split(".", 1)
        dev = _ids(d, "dev")
    patch = _num(rest, "patch")
    return Version(major, minor, patch, prefix, pre, build, dev, precision)


def _cmp_ids(a: tuple[str, ...], b: tuple[str, ...]) -> int:
    for x, y in zip(a, b):
        if x != y:
            return -1 if x < y else 1
    return (len(a) > len(b)) - (len(a) < len(b))


def compare(v: Version, o: Version) -> int:
    for x, y in ((v.major, o.major), (v.minor, o.minor), (v.patch, o.patch)):
        if x != y:
            return -1 if x < y else 1
    for a, b in ((v.pre, o.pre), (v.build, o.build), (v.dev, o.dev)):
        c = _cmp_ids(a, b)
        if c:
            return c
    return 0


def satisfies(supported: str, model: str, operator: str | None) -> bool:
    """Does a model's version satisfy a runtime's ``(version, operator)`` requirement?

    ``supported OP model`` with OP in Equal (default) / GreaterThan / GreaterThanOrEqual, i.e.
    GreaterThan means the runtime's version is newer than the model's.  Unofficial versions
    (pre/build/dev) only ever match Equal; precision and major-prefix must agree otherwise.
    """
    try:
        m, s = parse(model), parse(supported)
    except VersionError:
        return False
    op = operator or "Equal"
    if m.unofficial or s.unofficial or op == "Equal":
        return compare(s, m) == 0
    if m.precision != s.precision or m.major_prefix != s.major_prefix:
        return False
    c = compare(s, m)
    if op == "GreaterThan":
        return c == 1
    if op == "GreaterThanOrEqual":
        return c >= 0
    return c == 0

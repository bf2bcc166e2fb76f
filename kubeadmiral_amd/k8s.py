"""Third-party semantics the host packer needs (product code).

The reference resolves these inside k8s.io/apimachinery v0.26.6 / k8s.io/api
v0.26.6 on every (SchedulingUnit, cluster) pair; the packer resolves them once
per batch / snapshot so the device only compares interned ids:

* ``resource.Quantity`` parsing, ``Value()`` / ``MilliValue()`` (rounded away
  from zero) — used by ``framework.Resource.Add/Sub``
  (pkg/controllers/scheduler/framework/util.go:98-168) and rsp
  (plugins/rsp/rsp.go:183-325).
* ``validation.IsQualifiedName`` / ``IsValidLabelValue`` — label requirement
  validation in ``labels.NewRequirement`` (called from
  pkg/controllers/util/clusterselector/util.go:54).
* ``strconv.ParseInt(s, 10, 64)`` — Gt/Lt requirements.
* ``corev1.Toleration.ToleratesTaint`` — called from
  framework/util.go:406-413.
* ``IsScalarResourceName`` — framework/util.go:359-403.
"""

from __future__ import annotations

import math
import re
from fractions import Fraction

INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1
INT32_MIN, INT32_MAX = -(1 << 31), (1 << 31) - 1

_BIN = {"Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30, "Ti": 1 << 40, "Pi": 1 << 50, "Ei": 1 << 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 10 ** 3), "": Fraction(1),
        "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
        "P": Fraction(10 ** 15), "E": Fraction(10 ** 18)}
_NUM = re.compile(r"([+-]?(?:\d+(?:\.\d*)?|\.\d+))(.*)")
_qcache = {}


def quantity(s) -> Fraction:
    """Exact value of a Kubernetes quantity string (nano precision, rounded up)."""
    if isinstance(s, (int, Fraction)):
        return Fraction(s)
    v = _qcache.get(s)
    if v is not None:
        return v
    m = _NUM.fullmatch(s.strip())
    if not m:
        raise ValueError(f"invalid quantity {s!r}")
    num, suf = Fraction(m.group(1)), m.group(2)
    if suf in _BIN:
        v = num * _BIN[suf]
    elif suf in _DEC:
        v = num * _DEC[suf]
    elif suf[:1] in ("e", "E") and re.fullmatch(r"[+-]?\d+", suf[1:]):
        v = num * Fraction(10) ** int(suf[1:])
    else:
        raise ValueError(f"invalid quantity suffix {s!r}")
    n = v * 10 ** 9
    if n.denominator != 1:
        v = Fraction(_ceil_away(n), 10 ** 9)
    if len(_qcache) < 1 << 16:
        _qcache[s] = v
    return v


def _ceil_away(x: Fraction) -> int:
    return math.ceil(x) if x >= 0 else -math.ceil(-x)


def value(q) -> int:
    return _ceil_away(quantity(q))


def milli_value(q) -> int:
    return _ceil_away(quantity(q) * 1000)


def wrap64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


_DNS1123 = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*")
_QNAME = re.compile(r"([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]")
_LVALUE = re.compile(r"(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?")


def is_qualified_name(v: str) -> bool:
    parts = v.split("/")
    if len(parts) == 2:
        prefix, name = parts
        if not prefix or len(prefix) > 253 or not _DNS1123.fullmatch(prefix):
            return False
    elif len(parts) == 1:
        name = parts[0]
    else:
        return False
    return 0 < len(name) <= 63 and _QNAME.fullmatch(name) is not None


def is_valid_label_value(v: str) -> bool:
    return len(v) <= 63 and _LVALUE.fullmatch(v) is not None


def parse_int64(s: str):
    """strconv.ParseInt(s, 10, 64) → (value, ok)."""
    if not s:
        return 0, False
    body = s[1:] if s[0] in "+-" else s
    if not body or not body.isascii() or not body.isdigit():
        return 0, False
    v = int(s)
    if v < INT64_MIN or v > INT64_MAX:
        return 0, False
    return v, True


def tolerates_taint(tol, taint) -> bool:
    if tol.effect and tol.effect != taint.effect:
        return False
    if tol.key and tol.key != taint.key:
        return False
    if tol.operator in ("", "Equal"):
        return tol.value == taint.value
    return tol.operator == "Exists"


def is_scalar_resource_name(name: str) -> bool:
    native = "/" not in name or "kubernetes.io/" in name
    extended = (not native and not name.startswith("requests.") and is_qualified_name("requests." + name))
    return (extended or name.startswith("hugepages-") or "kubernetes.io/" in name
            or name.startswith("attachable-volumes-"))


def fnv1_32(data: bytes, h: int = 2166136261) -> int:
    for b in data:
        h = ((h * 16777619) & 0xFFFFFFFF) ^ b
    return h

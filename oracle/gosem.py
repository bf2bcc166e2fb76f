"""Go / k8s third-party semantics used by the oracle (TEST INFRASTRUCTURE ONLY).

This module is part of ``oracle/`` — a CPU restatement of the KubeAdmiral
scheduling hot path used only by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` as the *checker*. Product code never
imports it.

The reference's Go toolchain and its un-vendored dependencies are absent
(SURVEY.md §0, §8c), so these restate the pinned versions' published
algorithms:

* Go 1.19 integer arithmetic: int64 wrap-around, truncating ``/``;
  ``math.Round`` (half away from zero); float64→int64 conversion on amd64
  (truncate; NaN / out-of-range → MinInt64, the CVTTSD2SQ "integer indefinite").
* Go 1.19 ``sort.Slice`` / ``sort.Sort`` = ``pdqsort_func`` (src/sort/zsortfunc.go).
* Go ``hash/fnv`` New32 (FNV-1, not FNV-1a).
* k8s.io/apimachinery v0.26.6 ``resource.Quantity`` parsing, ``Value()`` /
  ``MilliValue()`` (rounded away from zero), ``util/validation``
  (``IsQualifiedName``, ``IsDNS1123Subdomain``, ``IsValidLabelValue``),
  ``labels.Requirement`` construction + ``Matches``, ``fields`` one-term
  selectors.
* k8s.io/api v0.26.6 ``Toleration.ToleratesTaint``.
"""

from __future__ import annotations

import math
import re
from fractions import Fraction

INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1


# ----------------------------------------------------------------- integers
def wrap64(x: int) -> int:
    """Go int64 two's-complement wrap-around."""
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


def go_div(a: int, b: int) -> int:
    """Go int64 ``a / b``: truncation toward zero (MinInt64 / -1 wraps)."""
    if b == 0:
        raise ZeroDivisionError("integer divide by zero")
    q = abs(a) // abs(b)
    if (a < 0) != (b < 0):
        q = -q
    return wrap64(q)


# ------------------------------------------------------------------- floats
def go_round(x: float) -> float:
    """Go ``math.Round``: nearest integer, halves away from zero."""
    if math.isnan(x) or math.isinf(x):
        return x
    t = float(math.trunc(x))
    if abs(x - t) >= 0.5:
        t += math.copysign(1.0, x)
    return t


def go_f64_to_i64(x: float) -> int:
    """Go ``int64(f)`` on amd64 (CVTTSD2SQ): truncate; NaN/overflow → MinInt64."""
    if math.isnan(x) or math.isinf(x):
        return INT64_MIN
    t = math.trunc(x)
    if t < INT64_MIN or t > INT64_MAX:
        return INT64_MIN
    return int(t)


# --------------------------------------------------------------------- FNV
def fnv1_32(data: bytes, h: int = 2166136261) -> int:
    """hash/fnv New32 (FNV-1): multiply then xor."""
    for b in data:
        h = (h * 16777619) & 0xFFFFFFFF
        h ^= b
    return h


# ------------------------------------------------------- Go 1.19 pdqsort
class XorShiftVariant:
    GO119 = (13, 17, 5)   # src/sort/sort.go in go1.19 (builder image golang:1.19)
    GO121 = (13, 7, 17)   # later 64-bit triple (selectable)


class _XorShift:
    def __init__(self, seed: int, triple):
        self.r = seed & 0xFFFFFFFFFFFFFFFF
        self.t = triple

    def next(self) -> int:
        a, b, c = self.t
        m = 0xFFFFFFFFFFFFFFFF
        self.r ^= (self.r << a) & m
        self.r ^= self.r >> b
        self.r ^= (self.r << c) & m
        return self.r


def _bits_len(n: int) -> int:
    return int(n).bit_length()


class GoSort:
    """Exact restatement of Go 1.19 ``pdqsort_func`` (src/sort/zsortfunc.go).

    ``less(i, j)`` and ``swap(i, j)`` operate on the caller's data, exactly
    like ``sort.Slice``'s ``lessSwap``.
    """

    UNKNOWN, INCREASING, DECREASING = 0, 1, 2

    def __init__(self, less, swap, triple=XorShiftVariant.GO119):
        self.less = less
        self.swap = swap
        self.triple = triple

    # sort.Slice(x, less) — sort.go: limit := bits.Len(uint(length))
    def sort(self, n: int):
        self.pdqsort(0, n, _bits_len(n))

    def insertion_sort(self, a, b):
        for i in range(a + 1, b):
            j = i
            while j > a and self.less(j, j - 1):
                self.swap(j, j - 1)
                j -= 1

    def sift_down(self, lo, hi, first):
        root = lo
        while True:
            child = 2 * root + 1
            if child >= hi:
                return
            if child + 1 < hi and self.less(first + child, first + child + 1):
                child += 1
            if not self.less(first + root, first + child):
                return
            self.swap(first + root, first + child)
            root = child

    def heap_sort(self, a, b):
        first = a
        lo = 0
        hi = b - a
        i = (hi - 1) // 2
        while i >= 0:
            self.sift_down(i, hi, first)
            i -= 1
        i = hi - 1
        while i >= 0:
            self.swap(first, first + i)
            self.sift_down(lo, i, first)
            i -= 1

    def pdqsort(self, a, b, limit):
        max_insertion = 12
        was_balanced = True
        was_partitioned = True
        while True:
            length = b - a
            if length <= max_insertion:
                self.insertion_sort(a, b)
                return
            if limit == 0:
                self.heap_sort(a, b)
                return
            if not was_balanced:
                self.break_patterns(a, b)
                limit -= 1
            pivot, hint = self.choose_pivot(a, b)
            if hint == self.DECREASING:
                self.reverse_range(a, b)
                pivot = (b - 1) - (pivot - a)
                hint = self.INCREASING
            if was_balanced and was_partitioned and hint == self.INCREASING:
                if self.partial_insertion_sort(a, b):
                    return
            if a > 0 and not self.less(a - 1, pivot):
                mid = self.partition_equal(a, b, pivot)
                a = mid
                continue
            mid, already = self.partition(a, b, pivot)
            was_partitioned = already
            left_len, right_len = mid - a, b - mid
            balance_threshold = length // 8
            if left_len < right_len:
                was_balanced = left_len >= balance_threshold
                self.pdqsort(a, mid, limit)
                a = mid + 1
            else:
                was_balanced = right_len >= balance_threshold
                self.pdqsort(mid + 1, b, limit)
                b = mid

    def partition(self, a, b, pivot):
        self.swap(a, pivot)
        i, j = a + 1, b - 1
        while i <= j and self.less(i, a):
            i += 1
        while i <= j and not self.less(j, a):
            j -= 1
        if i > j:
            self.swap(j, a)
            return j, True
        self.swap(i, j)
        i += 1
        j -= 1
        while True:
            while i <= j and self.less(i, a):
                i += 1
            while i <= j and not self.less(j, a):
                j -= 1
            if i > j:
                break
            self.swap(i, j)
            i += 1
            j -= 1
        self.swap(j, a)
        return j, False

    def partition_equal(self, a, b, pivot):
        self.swap(a, pivot)
        i, j = a + 1, b - 1
        while True:
            while i <= j and not self.less(a, i):
                i += 1
            while i <= j and self.less(a, j):
                j -= 1
            if i > j:
                break
            self.swap(i, j)
            i += 1
            j -= 1
        return i

    def partial_insertion_sort(self, a, b):
        max_steps = 5
        shortest_shifting = 50
        i = a + 1
        for _ in range(max_steps):
            while i < b and not self.less(i, i - 1):
                i += 1
            if i == b:
                return True
            if b - a < shortest_shifting:
                return False
            self.swap(i, i - 1)
            if i - a >= 2:
                j = i - 1
                while j >= 1:  # sic: Go's lower bound is 1, not a+1
                    if not self.less(j, j - 1):
                        break
                    self.swap(j, j - 1)
                    j -= 1
            if b - i >= 2:
                j = i + 1
                while j < b:
                    if not self.less(j, j - 1):
                        break
                    self.swap(j, j - 1)
                    j += 1
        return False

    def break_patterns(self, a, b):
        length = b - a
        if length >= 8:
            rnd = _XorShift(length, self.triple)
            modulus = 1 << _bits_len(length)
            idx = a + (length // 4) * 2 - 1
            for i in range(3):
                other = rnd.next() & (modulus - 1)
                if other >= length:
                    other -= length
                self.swap(idx - 1 + i, a + other)

    def choose_pivot(self, a, b):
        shortest_ninther = 50
        max_swaps = 4 * 3
        l = b - a
        swaps = [0]
        i = a + l // 4 * 1
        j = a + l // 4 * 2
        k = a + l // 4 * 3
        if l >= 8:
            if l >= shortest_ninther:
                i = self.median_adjacent(i, swaps)
                j = self.median_adjacent(j, swaps)
                k = self.median_adjacent(k, swaps)
            j = self.median(i, j, k, swaps)
        if swaps[0] == 0:
            return j, self.INCREASING
        if swaps[0] == max_swaps:
            return j, self.DECREASING
        return j, self.UNKNOWN

    def order2(self, a, b, swaps):
        if self.less(b, a):
            swaps[0] += 1
            return b, a
        return a, b

    def median(self, a, b, c, swaps):
        a, b = self.order2(a, b, swaps)
        b, c = self.order2(b, c, swaps)
        a, b = self.order2(a, b, swaps)
        return b

    def median_adjacent(self, a, swaps):
        return self.median(a - 1, a, a + 1, swaps)

    def reverse_range(self, a, b):
        i, j = a, b - 1
        while i < j:
            self.swap(i, j)
            i += 1
            j -= 1


def go_sort_slice(items: list, less_items, triple=XorShiftVariant.GO119) -> None:
    """``sort.Slice(items, func(i, j) bool { return less_items(items[i], items[j]) })`` in place."""

    def less(i, j):
        return less_items(items[i], items[j])

    def swap(i, j):
        items[i], items[j] = items[j], items[i]

    GoSort(less, swap, triple).sort(len(items))


def go_sort_sort(items: list, less_items, triple=XorShiftVariant.GO119) -> None:
    """``sort.Sort``: same pdqsort, but returns early for n <= 1 (sort.go)."""
    if len(items) <= 1:
        return
    go_sort_slice(items, less_items, triple)


# ------------------------------------------------------------- Quantity
_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": Fraction(1),
        "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
        "P": Fraction(10 ** 15), "E": Fraction(10 ** 18)}
_QTY_RE = re.compile(r"([+-]?(?:[0-9]+(?:\.[0-9]*)?|\.[0-9]+))(.*)")


def parse_quantity(s: str) -> Fraction:
    """resource.ParseQuantity → exact value (rounded up to nano precision)."""
    if isinstance(s, (int, Fraction)):
        return Fraction(s)
    s = s.strip() if isinstance(s, str) else s
    m = _QTY_RE.fullmatch(s)
    if not m:
        raise ValueError(f"quantities must match the regular expression: {s!r}")
    num = Fraction(m.group(1))
    suf = m.group(2)
    if suf in _BIN:
        v = num * _BIN[suf]
    elif suf in _DEC:
        v = num * _DEC[suf]
    elif suf[:1] in ("e", "E") and re.fullmatch(r"[+-]?[0-9]+", suf[1:]):
        v = num * Fraction(10) ** int(suf[1:])
    else:
        raise ValueError(f"unable to parse quantity's suffix: {s!r}")
    # values more precise than nano are rounded up (away from zero)
    nano = v * 10 ** 9
    if nano.denominator != 1:
        v = Fraction(_ceil_away(nano), 10 ** 9)
    return v


def _ceil_away(x: Fraction) -> int:
    if x >= 0:
        return math.ceil(x)
    return -math.ceil(-x)


def qty_value(q) -> int:
    """Quantity.Value(): ceil(q) away from zero."""
    return _ceil_away(parse_quantity(q))


def qty_milli_value(q) -> int:
    """Quantity.MilliValue(): ceil(q*1000) away from zero."""
    return _ceil_away(parse_quantity(q) * 1000)


# ------------------------------------------------------------ validation
_DNS1123_SUB = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*")
_QNAME = re.compile(r"([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]")
_LABEL_VALUE = re.compile(r"(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?")


def is_dns1123_subdomain(v: str) -> bool:
    return len(v) <= 253 and _DNS1123_SUB.fullmatch(v) is not None


def is_qualified_name(v: str) -> bool:
    """util/validation.IsQualifiedName → True when no errors."""
    parts = v.split("/")
    if len(parts) == 1:
        name = parts[0]
    elif len(parts) == 2:
        prefix, name = parts
        if len(prefix) == 0 or not is_dns1123_subdomain(prefix):
            return False
    else:
        return False
    if len(name) == 0 or len(name) > 63:
        return False
    return _QNAME.fullmatch(name) is not None


def is_valid_label_value(v: str) -> bool:
    return len(v) <= 63 and _LABEL_VALUE.fullmatch(v) is not None


def go_parse_int64(s: str):
    """strconv.ParseInt(s, 10, 64) → (value, ok)."""
    if not s:
        return 0, False
    body = s
    if body[0] in "+-":
        body = body[1:]
    if not body or not all("0" <= ch <= "9" for ch in body):
        return 0, False
    v = int(s)
    if v < INT64_MIN or v > INT64_MAX:
        return 0, False
    return v, True


# ------------------------------------------------------------- labels
class Requirement:
    """labels.Requirement (apimachinery v0.26.6 pkg/labels/selector.go)."""

    # selection operators
    IN, NOT_IN, EXISTS, DNE, GT, LT, EQUALS = "in", "notin", "exists", "!", "gt", "lt", "="

    def __init__(self, key, op, values):
        self.key, self.op, self.values = key, op, list(values or [])

    @staticmethod
    def new(key, op, vals):
        """labels.NewRequirement: returns (req, err_bool)."""
        vals = list(vals or [])
        err = not is_qualified_name(key)
        if op in (Requirement.IN, Requirement.NOT_IN):
            if len(vals) == 0:
                err = True
        elif op in (Requirement.EXISTS, Requirement.DNE):
            if len(vals) != 0:
                err = True
        elif op in (Requirement.GT, Requirement.LT):
            if len(vals) != 1:
                err = True
            for v in vals:
                if not go_parse_int64(v)[1]:
                    err = True
        else:
            err = True
        for v in vals:
            if not is_valid_label_value(v):
                err = True
        return Requirement(key, op, vals), err

    def matches(self, labels: dict) -> bool:
        has = labels is not None and self.key in labels
        if self.op in (Requirement.IN, Requirement.EQUALS):
            return has and labels[self.key] in self.values
        if self.op == Requirement.NOT_IN:
            return (not has) or labels[self.key] not in self.values
        if self.op == Requirement.EXISTS:
            return has
        if self.op == Requirement.DNE:
            return not has
        if self.op in (Requirement.GT, Requirement.LT):
            if not has:
                return False
            lv, ok = go_parse_int64(labels[self.key])
            if not ok or len(self.values) != 1:
                return False
            rv, ok = go_parse_int64(self.values[0])
            if not ok:
                return False
            return (self.op == Requirement.GT and lv > rv) or (self.op == Requirement.LT and lv < rv)
        return False


class LabelSelector:
    def __init__(self, reqs, nothing=False):
        self.reqs, self.nothing = reqs, nothing

    def matches(self, labels) -> bool:
        if self.nothing:
            return False
        return all(r.matches(labels) for r in self.reqs)


def selector_from_set(s: dict) -> LabelSelector:
    """labels.SelectorFromSet: Equals requirements, no validation; nil/empty = Everything."""
    return LabelSelector([Requirement(k, Requirement.EQUALS, [v]) for k, v in (s or {}).items()])


# --------------------------------------------------------------- taints
def tolerates_taint(tol, taint) -> bool:
    """corev1.Toleration.ToleratesTaint (k8s.io/api v0.26.6)."""
    if tol.effect != "" and tol.effect != taint.effect:
        return False
    if tol.key != "" and tol.key != taint.key:
        return False
    if tol.operator in ("", "Equal"):
        return tol.value == taint.value
    if tol.operator == "Exists":
        return True
    return False

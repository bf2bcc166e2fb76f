"""Go ``encoding/json`` semantics the scheduler's object handling depends on.

The reference turns annotation strings and unstructured objects into typed Go
structs with ``json.Unmarshal`` (``schedulingunit.go:261-668``,
``util/overrides.go:205-212``) and hashes ``json.Marshal`` output
(``schedulingtriggers.go:136``). Results only match the reference if the
decoding rules match Go 1.19's, so this module restates the ones that change
outcomes:

* struct fields match JSON keys exactly first, else case-insensitively
  (``bytes.EqualFold`` incl. the K/ſ folds); unknown keys are ignored; a key
  seen twice is decoded twice (the later one wins; objects/maps merge into the
  value already decoded, slices are replaced);
* ``null`` leaves non-pointer values untouched and sets pointers / slices /
  maps to nil;
* integers only from integer literals inside the target's range, floats from
  any number (``interface{}`` numbers are float64), no NaN/Infinity;
* a type mismatch anywhere is an error for the whole call (the reference
  discards every partial result on error).

Encoding restates ``encodeState.string`` with HTML escaping (``<``, ``>``,
``&`` → ``\\u003c`` …, U+2028/2029 escaped; unpaired surrogates, which a Go
string cannot hold, are written as the U+FFFD Go's decoder puts there) — what
``json.Marshal`` produces for the trigger struct.
"""

from __future__ import annotations

import json
import json.encoder
import re
from typing import Any, Callable, Dict, List, Optional, Tuple

INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1
INT32_MIN, INT32_MAX = -(1 << 31), (1 << 31) - 1


class GoJSONError(ValueError):
    """json.Unmarshal returned a non-nil error (syntax or UnmarshalTypeError)."""


class JObj(list):
    """A JSON object as the ordered list of its (key, value) members (duplicates kept)."""


def _reject_constant(name):
    raise GoJSONError(f"invalid character in literal {name}")


def _fix_str(s: str) -> str:
    # Go replaces unpaired surrogate escapes with U+FFFD
    if any(0xD800 <= ord(c) <= 0xDFFF for c in s):
        return "".join("\ufffd" if 0xD800 <= ord(c) <= 0xDFFF else c for c in s)
    return s


def loads(text: str):
    """Parse JSON text into Python values with objects as :class:`JObj`."""
    try:
        v = json.loads(text, object_pairs_hook=JObj, parse_constant=_reject_constant)
    except (ValueError, RecursionError) as e:
        raise GoJSONError(str(e)) from None
    return _fix_strings(v)


def _fix_strings(v):
    if isinstance(v, str):
        return _fix_str(v)
    if isinstance(v, JObj):
        return JObj((_fix_str(k), _fix_strings(x)) for k, x in v)
    if isinstance(v, list):
        return [_fix_strings(x) for x in v]
    return v


def from_unstructured(v):
    """An unstructured value (dicts from a decoded object) as Go would re-read it.

    ``UnstructuredToInterface`` marshals the object (map keys sorted bytewise)
    and unmarshals the bytes, so members are visited in sorted key order.
    """
    if isinstance(v, dict):
        return JObj((k, from_unstructured(v[k])) for k in sorted(v, key=lambda k: k.encode("utf-8", "surrogatepass")))
    if isinstance(v, (list, tuple)):
        return [from_unstructured(x) for x in v]
    return v


# --------------------------------------------------------------- decoding
def _fold(s: str) -> str:
    # bytes.EqualFold: ASCII case folding plus the two non-ASCII runes that fold to ASCII letters
    # (str.lower maps KELVIN SIGN to "k"; LATIN SMALL LONG S is lowercase already)
    return s.replace("\u017f", "s").lower()


class T:
    """Go target types for :func:`decode`."""

    def __init__(self, kind: str, sub=None, fields=None, make=None):
        self.kind = kind        # string bool int64 int32 float64 any slice map ptr struct
        self.sub = sub
        self.fields = fields    # struct: list of (json name, attribute, T)
        self.make = make        # struct: factory of the zero value


STRING, BOOL, INT64, INT32, ANY = T("string"), T("bool"), T("int64"), T("int32"), T("any")


def slice_of(t):
    return T("slice", t)


def map_of(t):
    return T("map", t)


def ptr_to(t):
    return T("ptr", t)


def struct(make: Callable[[], Any], fields: List[Tuple[str, str, T]]):
    return T("struct", fields=fields, make=make)


def _zero(t: T):
    if t.kind == "string":
        return ""
    if t.kind == "bool":
        return False
    if t.kind in ("int64", "int32"):
        return 0
    if t.kind == "struct":
        return t.make()
    return None  # any, slice, map, ptr: nil


def _type_err(t, v):
    raise GoJSONError(f"json: cannot unmarshal {type(v).__name__} into Go value of type {t.kind}")


def decode(t: T, v, cur=None):
    """Decode parsed JSON ``v`` into a Go value of type ``t`` that currently holds ``cur``."""
    if cur is None and t.kind in ("string", "bool", "int64", "int32", "struct"):
        cur = _zero(t)
    if v is None:  # JSON null
        return None if t.kind in ("any", "slice", "map", "ptr") else cur
    k = t.kind
    if k == "any":
        if isinstance(v, bool) or isinstance(v, str):
            return v
        if isinstance(v, int):
            try:
                return float(v)
            except OverflowError:
                raise GoJSONError("json: number out of range") from None
        if isinstance(v, float):
            if v != v or v in (float("inf"), float("-inf")):
                raise GoJSONError("json: number out of range")
            return v
        if isinstance(v, JObj):
            out = {}
            for key, x in v:
                out[key] = decode(ANY, x)
            return out
        return [decode(ANY, x) for x in v]
    if k == "string":
        if not isinstance(v, str):
            _type_err(t, v)
        return v
    if k == "bool":
        if not isinstance(v, bool):
            _type_err(t, v)
        return v
    if k in ("int64", "int32"):
        if isinstance(v, bool) or not isinstance(v, int):
            _type_err(t, v)
        lo, hi = (INT64_MIN, INT64_MAX) if k == "int64" else (INT32_MIN, INT32_MAX)
        if not lo <= v <= hi:
            _type_err(t, v)
        return v
    if k == "slice":
        if not isinstance(v, list) or isinstance(v, JObj):
            _type_err(t, v)
        return [decode(t.sub, x) for x in v]
    if k == "map":
        if not isinstance(v, JObj):
            _type_err(t, v)
        out = dict(cur) if cur is not None else {}
        for key, x in v:
            out[key] = decode(t.sub, x)  # every element is decoded into a fresh zero value
        return out
    if k == "ptr":
        return decode(t.sub, v, cur)
    if k == "struct":
        if not isinstance(v, JObj):
            _type_err(t, v)
        exact = {name: (attr, ft) for name, attr, ft in t.fields}
        folded = {}
        for name, attr, ft in t.fields:
            folded.setdefault(name.lower(), (attr, ft))
        for key, x in v:
            f = exact.get(key) or folded.get(_fold(key))
            if f is None:
                continue
            attr, ft = f
            setattr(cur, attr, decode(ft, x, getattr(cur, attr)))
        return cur
    raise AssertionError(k)


def unmarshal(text: str, t: T, cur=None):
    """``json.Unmarshal([]byte(text), &x)`` with x holding ``cur``; raises GoJSONError on error."""
    return decode(t, loads(text), cur)


# --------------------------------------------------------------- encoding
_HEX = "0123456789abcdef"


def _escape_table():
    t = {c: "\\u00" + _HEX[c >> 4] + _HEX[c & 0xF] for c in range(0x20)}  # control characters
    t.update({ord("\n"): "\\n", ord("\r"): "\\r", ord("\t"): "\\t", ord('"'): '\\"', ord("\\"): "\\\\"})
    t.update({ord(ch): "\\u00" + _HEX[ord(ch) >> 4] + _HEX[ord(ch) & 0xF] for ch in "<>&"})
    t.update({0x2028: "\\u2028", 0x2029: "\\u2029"})
    t.update({c: "\ufffd" for c in range(0xD800, 0xE000)})  # a Go string holds U+FFFD there
    return t


_ESCAPES = _escape_table()


# where Python's C string encoder (json.encoder.encode_basestring) and Go's differ: HTML characters, U+2028/9,
# surrogates, and \b / \f (Go 1.19 writes \u0008 / \u000c)
_GO_DIFF = re.compile("[<>&\u2028\u2029\ud800-\udfff\x08\x0c]")
_c_encode = json.encoder.encode_basestring


def _enc_str(s: str, out: List[str]) -> None:
    """encodeState.string with HTML escaping (_enc_str_ref: the per-character restatement it equals,
    tests/test_objects.py): Python's C encoder where the two agree, one str.translate elsewhere."""
    out.append(_c_encode(s) if _GO_DIFF.search(s) is None else '"' + s.translate(_ESCAPES) + '"')


def _enc_str_ref(s: str, out: List[str]) -> None:
    out.append('"')
    for ch in s:
        c = ord(ch)
        if c < 0x80:
            if ch == '"':
                out.append('\\"')
            elif ch == "\\":
                out.append("\\\\")
            elif c >= 0x20 and ch not in "<>&":
                out.append(ch)
            elif ch == "\n":
                out.append("\\n")
            elif ch == "\r":
                out.append("\\r")
            elif ch == "\t":
                out.append("\\t")
            else:
                out.append("\\u00" + _HEX[c >> 4] + _HEX[c & 0xF])
        elif 0xD800 <= c <= 0xDFFF:
            out.append("\ufffd")  # a Go string holds U+FFFD where JSON text had an unpaired surrogate
        elif c in (0x2028, 0x2029):
            out.append("\\u202" + _HEX[c & 0xF])
        else:
            out.append(ch)
    out.append('"')


def encode_string(s: str) -> str:
    out: List[str] = []
    _enc_str(s, out)
    return "".join(out)


class Raw:
    """Pre-encoded JSON text inserted verbatim by :func:`marshal`."""

    def __init__(self, text: str):
        self.text = text


def _enc(v, out: List[str]) -> None:
    if v is None:
        out.append("null")
    elif isinstance(v, Raw):
        out.append(v.text)
    elif isinstance(v, bool):
        out.append("true" if v else "false")
    elif isinstance(v, int):
        out.append(str(v))
    elif isinstance(v, str):
        _enc_str(v, out)
    elif isinstance(v, (list, tuple)) and not isinstance(v, JObj):
        out.append("[")
        for i, x in enumerate(v):
            if i:
                out.append(",")
            _enc(x, out)
        out.append("]")
    elif isinstance(v, (JObj, dict)):
        # a struct: members in declaration order, as given
        items = v if isinstance(v, JObj) else list(v.items())
        out.append("{")
        for i, (k, x) in enumerate(items):
            if i:
                out.append(",")
            _enc_str(k, out)
            out.append(":")
            _enc(x, out)
        out.append("}")
    else:
        raise TypeError(f"cannot encode {type(v).__name__}")


def marshal(v) -> bytes:
    """json.Marshal of a value built from str/int/bool/None/list and ordered dicts (= structs)."""
    out: List[str] = []
    _enc(v, out)
    return "".join(out).encode("utf-8")


def atoi(s: str) -> Optional[int]:
    """strconv.Atoi on a 64-bit platform; None where Go returns an error."""
    body = s[1:] if s[:1] in ("+", "-") else s
    if not body or not body.isascii() or not body.isdigit():
        return None
    v = int(s)
    return v if INT64_MIN <= v <= INT64_MAX else None

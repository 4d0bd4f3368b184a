"""Python restatement of the Go drop-in's object transfer (TEST INFRASTRUCTURE).

integration/go/gpudiff/gpudiff.go:jsonOf turns an informer object (the
``map[string]interface{}`` tree of an ``*unstructured.Unstructured``) into the
JSON text the engine decodes.  Go is not installed in this image, so the tests
run the same rules here over the oracle's decoded trees (``int`` = Go int64,
``float`` = Go float64, ``str``, ``bool``, ``None``, ``dict``, ``list``) and
submit the result through the C-ABI: the engine must then reach the oracle's
decision on the ORIGINAL JSON, i.e. the transfer loses nothing the predicates
(specsyncer.go:17-41, statussyncer.go:15-27) compare.

``go_marshal_json`` restates what the binding did before (``u.MarshalJSON``,
Go's encoding/json), kept to show the defect the marker contract removes:
float64(3) becomes ``3`` and reads back as int64.
"""
from __future__ import annotations

import decimal
import math
from typing import Any, Optional

from oracle import gpudiff_oracle as O
from oracle.upsert_oracle import go_marshal

MAX_NESTING = 10000  # encoding/json scanner maxNestingDepth
_HEX = "0123456789abcdef"


class NotTransferable(Exception):
    """appendValue's ok = false: the caller reports the pair dirty (specsyncer.go:20-22)."""


def go_format_g(f: float) -> str:
    """strconv.FormatFloat(f, 'g', -1, 64): the shortest round-trip digits, in %e form when the
    decimal exponent is < -4 or >= 6 (eprec = 6 for shortest), else %f; exponent at least two
    digits with a sign."""
    neg = math.copysign(1.0, f) < 0
    if f == 0:
        return "-0" if neg else "0"
    _sign, digs, exp = decimal.Decimal(repr(abs(f))).normalize().as_tuple()
    d = "".join(map(str, digs))
    nd, dp = len(d), len(d) + exp  # digits d, decimal point after dp digits
    x = dp - 1
    if x < -4 or x >= 6:
        s = d[0] + ("." + d[1:] if nd > 1 else "")
        s += "e" + ("-" if x < 0 else "+") + ("%02d" % abs(x))
    elif dp <= 0:
        s = "0." + "0" * (-dp) + d
    elif dp >= nd:
        s = d + "0" * (dp - nd)
    else:
        s = d[:dp] + "." + d[dp:]
    return ("-" if neg else "") + s


def _string(s: str, out: list):
    try:
        s.encode("utf-8")  # a lone surrogate = a Go string that is not valid UTF-8
    except UnicodeEncodeError:
        raise NotTransferable("string not valid UTF-8")
    out.append('"')
    for ch in s:
        c = ord(ch)
        if c >= 0x20 and ch not in '"\\':
            out.append(ch)
        elif ch in '"\\':
            out.append("\\" + ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        else:
            out.append("\\u00" + _HEX[c >> 4] + _HEX[c & 15])
    out.append('"')


def _value(v: Any, depth: int, out: list):
    if v is None:
        out.append("null")
    elif v is True:
        out.append("true")
    elif v is False:
        out.append("false")
    elif isinstance(v, int):
        if not O.INT64_MIN <= v <= O.INT64_MAX:
            raise NotTransferable("not an int64")
        out.append(str(v))
    elif isinstance(v, float):
        if math.isnan(v) or math.isinf(v):
            raise NotTransferable("NaN/Inf")
        s = go_format_g(v)
        if not any(c in s for c in ".eE"):
            s += ".0"
        out.append(s)
    elif isinstance(v, str):
        _string(v, out)
    elif isinstance(v, dict):
        if depth + 1 > MAX_NESTING:
            raise NotTransferable("too deep")
        out.append("{")
        for i, (k, e) in enumerate(v.items()):
            if i:
                out.append(",")
            _string(k, out)
            out.append(":")
            _value(e, depth + 1, out)
        out.append("}")
    elif isinstance(v, list):
        if depth + 1 > MAX_NESTING:
            raise NotTransferable("too deep")
        out.append("[")
        for i, e in enumerate(v):
            if i:
                out.append(",")
            _value(e, depth + 1, out)
        out.append("]")
    else:
        raise NotTransferable(type(v).__name__)


def shim_json(obj: Any, deep: bool = False) -> Optional[bytes]:
    """jsonOf(u) for u.Object == obj: the type-marked text, or None (not transferable).
    deep: the tree may nest past Python's default stack (runs on a big stack)."""
    if obj is None:
        obj = {}
    out: list = []
    try:
        if deep:
            O._on_big_stack(_value, obj, 0, out)
        else:
            _value(obj, 0, out)
    except NotTransferable:
        return None
    return "".join(out).encode("utf-8")


def go_marshal_json(obj: Any) -> bytes:
    """The old transfer: u.MarshalJSON() = encoding/json Marshal of the map (type-lossy for
    integral float64 values)."""
    return go_marshal(obj)


def informer_object(json_bytes: bytes):
    """What the informer hands UpdateFunc for this JSON: the decoded tree, or None when the
    informer could not deliver an *unstructured.Unstructured (Go decode error, or the list probe,
    oracle.informer_decode) -- the shim's type assertion then fails and the pair is dirty."""
    try:
        if O._nesting_bound(json_bytes) > 1000:
            return O._on_big_stack(O.informer_decode, json_bytes)
        return O.informer_decode(json_bytes)
    except O.DecodeError:
        return None


def shim_pair(a_json: bytes, b_json: bytes):
    """The pair the Go Batcher hands gpudiff_submit for an Update event (old, new), or None when
    the batcher reports it dirty itself (not Unstructured / not transferable: ``bad[i]``)."""
    a, b = informer_object(a_json), informer_object(b_json)
    if a is None or b is None:
        return None
    deep = O._nesting_bound(a_json) + O._nesting_bound(b_json) > 1000
    ja, jb = shim_json(a, deep), shim_json(b, deep)
    if ja is None or jb is None:
        return None
    return ja, jb

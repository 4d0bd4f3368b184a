"""CPU oracle for the syncer's write path -- TEST
INFRASTRUCTURE ONLY.  Like gpudiff_oracle, only ``tests/``, ``smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product never does.

What it restates (reference paths relative to /root/reference):

* ``upsertIntoDownstream`` -- pkg/syncer/specsyncer.go:86-132: DeepCopy, then
  ``SetUID("")`` / ``SetResourceVersion("")`` (:97-98), the ``kcp.dev/owned-by``
  label read through ``GetLabels()`` (:100), every owner reference whose
  ``Name`` equals it dropped (:101-107), ``SetOwnerReferences`` (:108), and the
  object handed to ``client.Create`` (:110).
* ``updateStatusInUpstream`` -- pkg/syncer/statussyncer.go:41-63: DeepCopy,
  ``SetUID("")`` / ``SetResourceVersion("")`` (:47-48).
* The request body the dynamic client sends for that object:
  ``runtime.Encode(unstructured.UnstructuredJSONScheme, obj)`` ->
  ``json.NewEncoder(w).Encode(obj.Object)``: Go 1.16 (go.mod:3)
  ``encoding/json`` Marshal of ``map[string]interface{}`` (keys sorted by
  bytes, HTML-safe string escaping, floats in the shortest round-trip form with
  the 'e' switch at 1e-6 / 1e21) plus the encoder's trailing newline.

The Unstructured accessors (third-party, apimachinery fork pinned at go.mod:33,
``pkg/apis/meta/v1/unstructured/{unstructured.go,helpers.go}``) are restated
from their published algorithms:

* ``SetUID("")``/``SetResourceVersion("")`` = ``RemoveNestedField(obj,
  "metadata", f)``: deletes the key only when ``metadata`` is a map.
* ``GetLabels`` = ``NestedStringMap``: nil unless ``metadata.labels`` is a map
  of strings, so the owned-by name is "" otherwise.
* ``GetOwnerReferences``: nil unless ``metadata.ownerReferences`` is a list of
  maps; each map -> OwnerReference{Kind, Name, APIVersion, UID: the string
  value or "", Controller / BlockOwnerDeletion: set only for a bool}.
* ``SetOwnerReferences(nil)`` = ``RemoveNestedField``; otherwise each kept
  reference is converted back with ``DefaultUnstructuredConverter
  .ToUnstructured``: ``apiVersion``, ``kind``, ``name``, ``uid`` always (no
  omitempty), ``controller`` / ``blockOwnerDeletion`` only when set.  The Go
  variable is nil unless at least one reference was appended (:102), so an
  empty result removes the field.

PARITY STATUS: the reference has no tests for this path and Go is absent, so
this restatement is pinned by the hand-written known-answer cases in
``tests/test_upsert.py`` (each stating the Go output it expects) and
cross-checked against the independent C++ host path; against a run of the
reference itself parity is UNPINNED.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .gpudiff_oracle import DecodeError, _nesting_bound, _on_big_stack, go_json_decode, nested_string_map

MODE_SPEC = 0    # upsertIntoDownstream (specsyncer.go:86-110): the Create body
MODE_STATUS = 1  # updateStatusInUpstream (statussyncer.go:41-48)

OWNED_BY = "kcp.dev/owned-by"  # specsyncer.go:100


# ---------------------------------------------------------------- transform

def _extract_owner_reference(v: Dict[str, Any]) -> Dict[str, Any]:
    """unstructured.extractOwnerReference + ToUnstructured(&ref)."""
    def s(k):
        x = v.get(k)
        return x if isinstance(x, str) else ""
    out: Dict[str, Any] = {"apiVersion": s("apiVersion"), "kind": s("kind"), "name": s("name"), "uid": s("uid")}
    for k in ("controller", "blockOwnerDeletion"):
        x = v.get(k)
        if isinstance(x, bool):
            out[k] = x
    return out


def _get_owner_references(obj: Dict[str, Any]) -> Optional[List[Dict[str, Any]]]:
    md = obj.get("metadata")
    if not isinstance(md, dict) or "ownerReferences" not in md:
        return None
    lst = md["ownerReferences"]
    if not isinstance(lst, list):
        return None
    if any(not isinstance(e, dict) for e in lst):
        return None
    return [_extract_owner_reference(e) for e in lst]


def transform(obj: Dict[str, Any], mode: int = MODE_SPEC) -> Dict[str, Any]:
    """The object the syncer writes (a deep copy; `obj` is not modified)."""
    import copy
    obj = copy.deepcopy(obj)
    md = obj.get("metadata")
    if isinstance(md, dict):            # SetUID("") / SetResourceVersion("")
        md.pop("uid", None)
        md.pop("resourceVersion", None)
    if mode == MODE_STATUS:
        return obj
    labels = nested_string_map(obj, "metadata", "labels")
    owned = (labels or {}).get(OWNED_BY, "")
    refs = _get_owner_references(obj) or []
    kept = [r for r in refs if r["name"] != owned]
    md = obj.get("metadata")
    if isinstance(md, dict):
        if kept:
            md["ownerReferences"] = kept
        else:
            md.pop("ownerReferences", None)
    return obj


# ---------------------------------------------------------------- Go marshal

_HEX = "0123456789abcdef"


def _go_string(s: str, out: bytearray):
    """encodeState.string(s, escapeHTML=true) of Go 1.16."""
    out.append(0x22)
    for ch in s:
        c = ord(ch)
        if c < 0x80:
            if c == 0x22 or c == 0x5C:
                out += b"\\" + bytes([c])
            elif c == 0x0A:
                out += b"\\n"
            elif c == 0x0D:
                out += b"\\r"
            elif c == 0x09:
                out += b"\\t"
            elif c < 0x20 or c in (0x3C, 0x3E, 0x26):
                out += b"\\u00" + bytes([ord(_HEX[c >> 4]), ord(_HEX[c & 15])])
            else:
                out.append(c)
        elif c == 0x2028 or c == 0x2029:
            out += ("\\u202" + _HEX[c & 15]).encode()
        else:
            out += ch.encode("utf-8")
    out.append(0x22)


def go_float(f: float) -> bytes:
    """floatEncoder(64).encode: strconv.AppendFloat(f, 'f' or 'e', -1, 64)."""
    if math.isinf(f) or math.isnan(f):
        raise ValueError("unsupported float")
    a = abs(f)
    if a != 0 and (a < 1e-6 or a >= 1e21):
        s = np.format_float_scientific(f, unique=True, trim="-", exp_digits=2)
        # numpy writes "1e+21" / "1.5e-07"; Go cleans e-07 -> e-7
        if len(s) >= 4 and s[-4] == "e" and s[-3] == "-" and s[-2] == "0":
            s = s[:-2] + s[-1]
    else:
        s = np.format_float_positional(f, unique=True, trim="-")
        if s == "-0" or (f == 0 and math.copysign(1.0, f) < 0):
            s = "-0"
    return s.encode("ascii")


def _marshal(x: Any, out: bytearray):
    if x is None:
        out += b"null"
    elif x is True:
        out += b"true"
    elif x is False:
        out += b"false"
    elif isinstance(x, int):
        out += str(x).encode()
    elif isinstance(x, float):
        out += go_float(x)
    elif isinstance(x, str):
        _go_string(x, out)
    elif isinstance(x, list):
        out.append(0x5B)
        for i, v in enumerate(x):
            if i:
                out.append(0x2C)
            _marshal(v, out)
        out.append(0x5D)
    elif isinstance(x, dict):
        out.append(0x7B)
        for i, k in enumerate(sorted(x.keys(), key=lambda k: k.encode("utf-8"))):
            if i:
                out.append(0x2C)
            _go_string(k, out)
            out.append(0x3A)
            _marshal(x[k], out)
        out.append(0x7D)
    else:
        raise TypeError(type(x))


def go_marshal(obj: Any) -> bytes:
    out = bytearray()
    _marshal(obj, out)
    return bytes(out)


def upsert_body(json_bytes: bytes, mode: int = MODE_SPEC) -> Optional[bytes]:
    """The request body for the write the syncer issues for this object:
    json.NewEncoder(w).Encode(transform(decode(json))) -- Marshal plus '\\n'.
    None if the informer could never have delivered the object (Go decode
    error)."""
    if _nesting_bound(json_bytes) > 1000:  # recursion as deep as Go's 10000-level limit
        return _on_big_stack(_upsert_body, json_bytes, mode)
    return _upsert_body(json_bytes, mode)


def _upsert_body(json_bytes: bytes, mode: int) -> Optional[bytes]:
    try:
        obj = go_json_decode(json_bytes)
    except DecodeError:
        return None
    return go_marshal(transform(obj, mode)) + b"\n"


PLAN_SPEC, PLAN_STATUS, PLAN_UPSTREAM_DOWNSTREAM = 0x1, 0x2, 0x4  # gpudiff_write_plan_get_ex modes


def write_plan(pairs, mode: int = 0) -> List[Tuple[int, int, bool, Optional[bytes]]]:
    """The writes the syncer issues for a batch of pairs, as
    gpudiff_write_plan_get_ex lists them: every spec-dirty pair
    (upsertIntoDownstream, pkg/syncer/specsyncer.go:86-132, MODE_SPEC), then
    every status-dirty pair (updateStatusInUpstream, statussyncer.go:41-63,
    MODE_STATUS); PLAN_SPEC / PLAN_STATUS restrict the kinds (neither = both).

    Which document a write renders: for informer pairs (old, new) -- the
    default -- UpdateFunc enqueues newObj (specsyncer.go:47-50,
    statussyncer.go:32-35) and the worker writes it, so both kinds render new;
    with PLAN_UPSTREAM_DOWNSTREAM the pairs are (A upstream, B downstream) and
    the spec write renders A, the status write B.  A write the oracle marks
    no-op (gpudiff_oracle.diff_pair spec_noop / status_noop) has no body.
    Returns [(pair index, mode, noop, body or None if undecodable)]."""
    from .gpudiff_oracle import diff_pair
    kinds = mode & (PLAN_SPEC | PLAN_STATUS) or (PLAN_SPEC | PLAN_STATUS)
    spec_side = 0 if mode & PLAN_UPSTREAM_DOWNSTREAM else 1
    rs = [diff_pair(a, b) for a, b in pairs]
    out = []
    for bit, kind, dirty, noop, side in ((PLAN_SPEC, MODE_SPEC, "spec_dirty", "spec_noop", spec_side),
                                         (PLAN_STATUS, MODE_STATUS, "status_dirty", "status_noop", 1)):
        if not kinds & bit:
            continue
        for i, r in enumerate(rs):
            if r[dirty]:
                skip = bool(r[noop])
                out.append((i, kind, skip, b"" if skip else upsert_body(pairs[i][side], kind)))
    return out

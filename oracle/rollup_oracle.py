"""CPU oracle for the Deployment splitter's status roll-up (SURVEY.md §8(f)
row 4) -- TEST INFRASTRUCTURE ONLY.  Like gpudiff_oracle, only ``tests/``,
``smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it; the product
never does.

What it restates (reference paths relative to /root/reference):

* ``reconcile`` of a leaf Deployment -- pkg/reconciler/deployment/deployment.go:
  41-91: the leaf's ``kcp.dev/owned-by`` label names its root (:42); every
  cached Deployment matching the selector ``kcp.dev/owned-by=<root>`` (:44-51,
  ``c.lister.List(sel)``: all namespaces, all logical clusters) is summed into
  the root's ``status.{replicas, updatedReplicas, readyReplicas,
  availableReplicas, unavailableReplicas}`` (:74-85, ``int32`` additions, so Go
  wrap-around), and the root's ``status.conditions`` become ``others[0]``'s
  (:89-91).  The lister's order is unspecified (a cache index walk); the batch
  form fixes ``others[0]`` to the member with the lowest document index.

* The objects are typed ``appsv1.Deployment`` values decoded from JSON by Go
  1.16 ``encoding/json`` (third-party, k8s.io/api, go.mod:34).  Restated for the
  fields the splitter reads:

  - struct fields match keys exactly or, failing that, case-insensitively
    (``bytes.EqualFold`` for ASCII names: ``"Status"`` fills ``status``);
  - a repeated key decodes again INTO the same field: structs merge (fields
    the second object omits keep their values), maps merge (``labels`` gains
    the second object's entries, a repeated label key last-wins);
  - ``null`` leaves a struct or an int32 field untouched and sets a map to nil;
  - an ``int32`` field takes a number literal that ``strconv.ParseInt(s, 10,
    64)`` accepts and that fits int32; anything else (``3.0``, ``1e2``, a
    string, a bool, an object, overflow) is an ``UnmarshalTypeError`` -- the
    object is never delivered to the informer, so the batch reports it as a
    decode error (group -2) and leaves it out;
  - ``labels`` is ``map[string]string``: a null value stores ``""`` (the
    element's zero value); a non-string value, or a non-object
    ``labels``/``metadata``/``status``, is a decode error as well;
  - only JSON syntax is checked elsewhere (Go's scanner); other typed fields of
    the Deployment are not read by the roll-up and not type-checked here.

PARITY STATUS: the reference has no tests for the splitter and Go is absent, so
this restatement is pinned by the hand-written known-answer cases in
``tests/rollup_cases.py`` (each stating the Go outcome) and cross-checked
against the independent C++ host path; against a run of the reference itself
parity is UNPINNED.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

from .gpudiff_oracle import DecodeError, _Parser

OWNED_BY = "kcp.dev/owned-by"     # deployment.go:18
FIELDS = ("replicas", "updatedReplicas", "readyReplicas", "availableReplicas", "unavailableReplicas")
INT32_MIN, INT32_MAX = -(1 << 31), (1 << 31) - 1

GROUP_NONE = -1     # no owned-by label: not a leaf of any root
GROUP_DECODE = -2   # Go cannot decode the object into an appsv1.Deployment


class _Num(str):
    """A number literal, kept as text (typed decode parses it per field)."""


class _Pairs(list):
    """A JSON object as its (key, value) members in document order."""


class _PairParser(_Parser):
    def number(self):
        b, i, n = self.b, self.i, self.n
        s = i
        if b[i] == ord('-'):
            i += 1
        if i >= n:
            raise DecodeError("bad number")
        if b[i] == ord('0'):
            i += 1
        elif 0x31 <= b[i] <= 0x39:
            while i < n and 0x30 <= b[i] <= 0x39:
                i += 1
        else:
            raise DecodeError("bad number")
        if i < n and b[i] == ord('.'):
            i += 1
            if i >= n or not (0x30 <= b[i] <= 0x39):
                raise DecodeError("bad fraction")
            while i < n and 0x30 <= b[i] <= 0x39:
                i += 1
        if i < n and b[i] in b"eE":
            i += 1
            if i < n and b[i] in b"+-":
                i += 1
            if i >= n or not (0x30 <= b[i] <= 0x39):
                raise DecodeError("bad exponent")
            while i < n and 0x30 <= b[i] <= 0x39:
                i += 1
        self.i = i
        return _Num(b[s:i].decode('ascii'))

    def obj(self, depth: int):
        if depth > 10000:
            raise DecodeError("exceeded max depth")
        self.i += 1
        m = _Pairs()
        self.ws()
        if self.i < self.n and self.b[self.i] == ord('}'):
            self.i += 1
            return m
        while True:
            self.ws()
            if self.i >= self.n or self.b[self.i] != 0x22:
                raise DecodeError("expected key")
            k = self.string()
            self.ws()
            if self.i >= self.n or self.b[self.i] != ord(':'):
                raise DecodeError("expected colon")
            self.i += 1
            m.append((k, self.value(depth)))
            self.ws()
            if self.i >= self.n:
                raise DecodeError("unterminated object")
            c = self.b[self.i]
            self.i += 1
            if c == ord(','):
                continue
            if c == ord('}'):
                return m
            raise DecodeError("expected , or }")


def _parse(data: bytes) -> _Pairs:
    p = _PairParser(data)
    p.ws()
    if p.i >= p.n or p.b[p.i] != ord('{'):
        raise DecodeError("top level is not an object")
    v = p.value(0)
    p.ws()
    if p.i != p.n:
        raise DecodeError("trailing data")
    return v


def _field_matches(name: str, key: str) -> bool:
    """encoding/json field lookup (Go 1.16 fold.go): ASCII case-insensitive;
    for names holding 's'/'k' (equalFoldRight) a non-ASCII key rune matches only
    U+017F LATIN SMALL LETTER LONG S for 's' and U+212A KELVIN SIGN for 'k'."""
    if len(key) != len(name):
        return False
    for c, t in zip(name, key):
        if t.isascii():
            if c.lower() != t.lower():
                return False
        elif not ((c in "sS" and t == "\u017f") or (c in "kK" and t == "\u212a")):
            return False
    return True


def _struct_members(obj: _Pairs, names: Tuple[str, ...]):
    """Members of a JSON object that land in one of the struct fields `names`,
    in document order (Go decodes each occurrence into the field again).  An
    exact name match wins over a fold match among the fields (Go 1.16 object():
    first exact, else first fold)."""
    for k, v in obj:
        hit = None
        for nm in names:
            if k == nm:
                hit = nm
                break
        if hit is None:
            for nm in names:
                if _field_matches(nm, k):
                    hit = nm
                    break
        if hit is not None:
            yield hit, v


def _int32(v: Any, cur: int) -> int:
    if v is None:
        return cur             # null into an int: no-op
    if not isinstance(v, _Num):
        raise DecodeError("cannot unmarshal %s into int32" % type(v).__name__)
    try:
        x = int(v, 10)         # strconv.ParseInt(s, 10, 64): digits only
    except ValueError:
        raise DecodeError("cannot unmarshal number %s into int32" % v)
    if not (INT32_MIN <= x <= INT32_MAX):
        raise DecodeError("number %s overflows int32" % v)
    return x


def extract(data: bytes) -> Dict[str, Any]:
    """The roll-up fields of one cached Deployment: {'status': [5 x int32],
    'owned_by': str or None}.  Raises DecodeError where Go's typed decode fails."""
    if isinstance(data, str):
        data = data.encode('utf-8')
    root = _parse(data)
    status = [0] * 5
    labels: Optional[Dict[str, str]] = None
    for name, v in _struct_members(root, ("metadata", "status")):
        if v is None:
            continue                                  # null into a struct: no-op
        if not isinstance(v, _Pairs):
            raise DecodeError("%s is not an object" % name)
        if name == "metadata":
            for _, lv in _struct_members(v, ("labels",)):
                if lv is None:
                    labels = None                     # null into a map: nil
                    continue
                if not isinstance(lv, _Pairs):
                    raise DecodeError("labels is not an object")
                if labels is None:
                    labels = {}
                for lk, lval in lv:
                    if lval is None:
                        lval = ""                      # null into a map element: its zero value
                    if isinstance(lval, _Num) or not isinstance(lval, str):
                        raise DecodeError("label value is not a string")
                    labels[lk] = lval                  # map: last wins, entries merge
        else:
            for f, fv in _struct_members(v, FIELDS):
                i = FIELDS.index(f)
                status[i] = _int32(fv, status[i])
    owned = labels.get(OWNED_BY) if labels is not None else None
    return {"status": status, "owned_by": owned}


def _wrap32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


def rollup(docs: List[bytes]) -> Dict[str, Any]:
    """Batch form: groups = distinct owned-by values in order of first
    appearance; per group the member count, the int32 sums (Go wrap-around) and
    others[0] = the lowest member index.  doc_group[i] = group index, -1 (no
    owned-by label) or -2 (decode error)."""
    doc_group: List[int] = []
    groups: List[Dict[str, Any]] = []
    index: Dict[str, int] = {}
    for i, d in enumerate(docs):
        try:
            e = extract(d)
        except DecodeError:
            doc_group.append(GROUP_DECODE)
            continue
        ob = e["owned_by"]
        if ob is None:
            doc_group.append(GROUP_NONE)
            continue
        g = index.get(ob)
        if g is None:
            g = index[ob] = len(groups)
            groups.append({"owned_by": ob, "first_doc": i, "n_members": 0, "sums": [0] * 5})
        G = groups[g]
        G["n_members"] += 1
        G["sums"] = [_wrap32(a + b) for a, b in zip(G["sums"], e["status"])]
        doc_group.append(g)
    return {"doc_group": doc_group, "groups": groups}

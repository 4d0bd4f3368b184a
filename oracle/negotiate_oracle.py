"""CPU oracle for the API-negotiation update classifier (SURVEY.md §8(f) row 4,
second half) -- TEST INFRASTRUCTURE ONLY.  Like gpudiff_oracle, only
``tests/``, ``smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it;
the product never does.

What it restates (reference paths relative to /root/reference):

* ``Controller.enqueue`` for an "Update" of an ``APIResourceImport`` or a
  ``NegotiatedAPIResource`` -- pkg/reconciler/apiresource/controller.go:238-295,
  with ``toQueueElementType`` (:184-236) supplying the typed metadata and the
  typed ``.Status`` value:

  - no old object                                  -> Created   (:258-261)
  - equal ``resourceVersion`` strings               -> ignored   (:263-265)
  - different ``generation``                        -> SpecChanged (:267-270)
  - ``!Semantic.DeepEqual(oldStatus, newStatus)``   -> StatusOnlyChanged (:272-275)
  - ``!DeepEqual(annotations) || DeepEqual(labels)`` -> AnnotationOrLabelsOnlyChanged
    (:277-281; the missing ``!`` before the labels term at :278 is reproduced:
    equal labels classify as a metadata change, differing labels with equal
    annotations are ignored)
  - otherwise                                       -> ignored   (:282-283)

* Both kinds have the status ``{conditions: [{type, status,
  lastTransitionTime, reason, message}]}``
  (pkg/apis/apiresource/v1alpha1/apiresourceimport_types.go:123-143,
  negociatedapiresource_types.go:85-104).  The objects are decoded by Go 1.16
  ``encoding/json`` (third party); restated for the fields read:

  - struct field lookup exact, else case-insensitive (rollup_oracle's rules);
    a repeated key decodes again INTO the field (maps merge, structs merge);
  - ``null`` leaves a string / int64 / struct untouched, sets a map or slice
    to nil, and sets ``lastTransitionTime`` to the zero Time (metav1.Time's
    UnmarshalJSON runs for null);
  - a JSON array decodes into the existing slice: element i is decoded INTO the
    element already there (merging), the length becomes the array's, capacity
    grows as Go's ``cap + cap/2`` (min 4), so a later longer array can expose
    elements of an earlier decode that sit within the capacity;
  - ``generation`` is an int64 (``strconv.ParseInt``), ``resourceVersion`` and
    the condition strings are strings; anything else is a decode error;
  - ``lastTransitionTime``: ``time.Parse(time.RFC3339, s)`` (Go 1.16:
    4-digit year, 2-digit month/day/minute/second, 1-or-2-digit hour,
    fractional seconds of any length after the seconds, ``Z`` or
    ``±hh:mm`` with ``atoi`` on each part and no offset range check, day
    checked against the month).

* ``equality.Semantic.DeepEqual`` (apimachinery fork): nil and empty maps and
  slices are equal; metav1.Time compares ``a.UTC() == b.UTC()``, i.e. the
  instant to the nanosecond.

DECODE (-1) means: a side is not valid JSON, is not an object, or one of the
fields read above fails Go's typed decode (the reference's informer would
never deliver such an object).  Type errors in fields the classifier does not
read (spec, metadata.name, creationTimestamp, ...) are not checked: Go's typed
Unmarshal would reject those objects too, so no reference outcome exists for
them, and the classification here follows the fields read (KAT
"outside-domain-spec-type-error").  A root ``null`` (a zero object to Go's
Unmarshal; never a watch event body) is reported as DECODE.

* ``CustomResourceDefinition`` events (the third kind, :186-199; ``kind=
  KIND_CRD``): the typed status is apiextensions/v1
  ``CustomResourceDefinitionStatus`` (k8s.io/apiextensions-apiserver, pinned by
  go.mod:32 to kcp-dev/kubernetes c954268bf177; not vendored in the reference,
  restated from its published types): ``conditions`` (the same five fields),
  ``acceptedNames`` -- a struct ``{plural, singular, shortNames []string, kind,
  listKind, categories []string}`` (null leaves it as it is, a repeated key
  merges into it) -- and ``storedVersions []string``.  ``[]string`` decodes
  like ``conditions``: element i INTO the string already there (a null
  element leaves it, so "" in a fresh backing array), Go's growth rule, a
  later longer array exposing stale capacity.  Semantic.DeepEqual compares the
  three fields with nil == empty slices.

PARITY STATUS: no reference tests exist for the controller and Go is absent,
so this restatement is pinned by the hand-written known-answer cases in
``tests/negotiate_cases.py`` (each stating the Go outcome) and cross-checked
against the independent C++ host path; against a run of the reference itself
parity is UNPINNED.
"""
from __future__ import annotations

from typing import Any, List, Optional, Tuple

from .gpudiff_oracle import DecodeError
from .rollup_oracle import _Num, _Pairs, _parse, _struct_members

IGNORE, SPEC_CHANGED, STATUS_ONLY, META_ONLY, CREATED, DECODE = 0, 1, 2, 3, 4, -1
ACTION_NAMES = {IGNORE: "ignored", SPEC_CHANGED: "SpecChanged", STATUS_ONLY: "StatusOnlyChanged",
                META_ONLY: "AnnotationOrLabelsOnlyChanged", CREATED: "Created", DECODE: "decode-error"}

COND_FIELDS = ("type", "status", "lastTransitionTime", "reason", "message")
# apiextensions/v1 CustomResourceDefinitionStatus / CustomResourceDefinitionNames field order (the fold lookup's order)
CRD_STATUS_FIELDS = ("conditions", "acceptedNames", "storedVersions")
CRD_NAMES_FIELDS = ("plural", "singular", "shortNames", "kind", "listKind", "categories")
KIND_KCP, KIND_CRD = 0, 1
META_FIELDS = ("resourceVersion", "generation", "labels", "annotations")
INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1
ZERO_TIME = (-62135596800, 0)  # time.Time{}: 0001-01-01T00:00:00Z as (unix seconds, ns)


# ------------------------------------------------------------------ time.Parse(time.RFC3339, s), Go 1.16
def _days_from_civil(y: int, m: int, d: int) -> int:
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    doy = (153 * (m + (-3 if m > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def _days_in(m: int, y: int) -> int:
    if m == 2:
        return 29 if (y % 4 == 0 and (y % 100 != 0 or y % 400 == 0)) else 28
    return 30 if m in (4, 6, 9, 11) else 31


def _isdig(s: str, i: int) -> bool:
    return i < len(s) and "0" <= s[i] <= "9"


def _getnum(s: str, fixed: bool) -> Tuple[int, str]:
    if not _isdig(s, 0):
        raise DecodeError("time: bad number")
    if not _isdig(s, 1):
        if fixed:
            raise DecodeError("time: bad number")
        return ord(s[0]) - 48, s[1:]
    return (ord(s[0]) - 48) * 10 + ord(s[1]) - 48, s[2:]


def _atoi(s: str) -> int:
    """time.atoi: optional sign, then leadingInt over the rest, which must be
    all digits and must not overflow int64."""
    neg = False
    if s and s[0] in "+-":
        neg = s[0] == "-"
        s = s[1:]
    i, x = 0, 0
    while i < len(s) and "0" <= s[i] <= "9":
        if x > (1 << 63) // 10:
            raise DecodeError("time: bad number")
        x = x * 10 + ord(s[i]) - 48
        if x >= 1 << 63:
            raise DecodeError("time: bad number")
        i += 1
    if i != len(s) or i == 0 and s != "":
        raise DecodeError("time: bad number")
    if i == 0:  # leadingInt("") = 0, no error
        return 0
    return -x if neg else x


def parse_rfc3339(s: str) -> Tuple[int, int]:
    """(unix seconds, nanoseconds) of the instant, or DecodeError."""
    v = s
    if len(v) < 4 or not _isdig(v, 0):
        raise DecodeError("time: bad year")
    year = _atoi(v[:4])
    v = v[4:]
    if not v.startswith("-"):
        raise DecodeError("time: expected -")
    month, v = _getnum(v[1:], True)
    if month <= 0 or month > 12:
        raise DecodeError("time: month out of range")
    if not v.startswith("-"):
        raise DecodeError("time: expected -")
    day, v = _getnum(v[1:], True)
    if not v.startswith("T"):
        raise DecodeError("time: expected T")
    hour, v = _getnum(v[1:], False)
    if hour >= 24:
        raise DecodeError("time: hour out of range")
    if not v.startswith(":"):
        raise DecodeError("time: expected :")
    minute, v = _getnum(v[1:], True)
    if minute >= 60:
        raise DecodeError("time: minute out of range")
    if not v.startswith(":"):
        raise DecodeError("time: expected :")
    sec, v = _getnum(v[1:], True)
    if sec >= 60:
        raise DecodeError("time: second out of range")
    nsec = 0
    if len(v) >= 2 and v[0] == "." and _isdig(v, 1):
        n = 2
        while n < len(v) and _isdig(v, n):
            n += 1
        ns = _atoi(v[1:n])
        if ns < 0 or ns >= 10 ** 9:
            raise DecodeError("time: fractional second out of range")
        for _ in range(10 - n):
            ns *= 10
        nsec = ns
        v = v[n:]
    if v.startswith("Z"):
        off = 0
        v = v[1:]
    else:
        if len(v) < 6 or v[3] != ":":
            raise DecodeError("time: bad zone")
        sign, hh, mm, v = v[0], v[1:3], v[4:6], v[6:]
        off = (_atoi(hh) * 60 + _atoi(mm)) * 60
        if sign == "-":
            off = -off
        elif sign != "+":
            raise DecodeError("time: bad zone sign")
    if v:
        raise DecodeError("time: extra text")
    if day < 1 or day > _days_in(month, year):
        raise DecodeError("time: day out of range")
    secs = _days_from_civil(year, month, day) * 86400 + hour * 3600 + minute * 60 + sec - off
    return (secs, nsec)


# ------------------------------------------------------------------ typed decode of the fields read
class _Cond:
    __slots__ = ("type", "status", "time", "reason", "message")

    def __init__(self):
        self.type = self.status = self.reason = self.message = ""
        self.time = ZERO_TIME

    def key(self):
        return (self.type, self.status, self.time, self.reason, self.message)


def _string(v: Any, cur: str) -> str:
    if v is None:
        return cur
    if isinstance(v, _Num) or not isinstance(v, str):
        raise DecodeError("cannot unmarshal into string")
    return v


def _int64(v: Any, cur: int) -> int:
    if v is None:
        return cur
    if not isinstance(v, _Num):
        raise DecodeError("cannot unmarshal into int64")
    try:
        x = int(v, 10)
    except ValueError:
        raise DecodeError("cannot unmarshal number %s into int64" % v)
    if not (INT64_MIN <= x <= INT64_MAX):
        raise DecodeError("number %s overflows int64" % v)
    return x


def _string_map(v: Any, cur: Optional[dict]) -> Optional[dict]:
    if v is None:
        return None
    if not isinstance(v, _Pairs):
        raise DecodeError("map is not an object")
    m = {} if cur is None else cur
    for k, x in v:
        if x is None:
            x = ""
        if isinstance(x, _Num) or not isinstance(x, str):
            raise DecodeError("map value is not a string")
        m[k] = x
    return m


def _cond_into(c: _Cond, v: Any) -> None:
    if v is None:
        return
    if not isinstance(v, _Pairs):
        raise DecodeError("condition is not an object")
    for f, x in _struct_members(v, COND_FIELDS):
        if f == "lastTransitionTime":
            if x is None:
                c.time = ZERO_TIME
            elif isinstance(x, _Num) or not isinstance(x, str):
                raise DecodeError("lastTransitionTime is not a string")
            else:
                c.time = parse_rfc3339(x)
        else:
            setattr(c, f, _string(x, getattr(c, f)))


class _Slice:
    """A Go slice header over a backing array (len, cap) -- enough of it to
    reproduce decoding a repeated array key into the same field.  `zero` makes
    an element's zero value, `into(cur, v)` decodes v into an element and
    returns it (Go decodes element i INTO the value already there)."""

    def __init__(self, zero=_Cond, into=None, what="conditions"):
        self.nil = True
        self.backing: List[Any] = []  # len(backing) == cap
        self.len = 0
        self.zero = zero
        self.into = into or _cond_elem
        self.what = what

    def decode(self, v: Any) -> None:
        if v is None:
            self.nil, self.backing, self.len = True, [], 0
            return
        if isinstance(v, _Pairs) or not isinstance(v, list):
            raise DecodeError("%s is not an array" % self.what)
        i = 0
        for e in v:
            if i >= len(self.backing):  # reflect growth: cap + cap/2, at least 4; the first len elements copied
                newcap = max(4, len(self.backing) + len(self.backing) // 2)
                nb = [self.zero() for _ in range(newcap)]
                for k in range(self.len):
                    nb[k] = self.backing[k]
                self.backing = nb
            if i >= self.len:
                self.len = i + 1
            self.backing[i] = self.into(self.backing[i], e)
            i += 1
        if i < self.len:
            self.len = i
        if i == 0:
            self.backing, self.len = [], 0
        self.nil = False

    def value(self) -> Tuple:
        return tuple(_key(self.backing[k]) for k in range(self.len))


def _key(e: Any) -> Any:
    return e.key() if isinstance(e, _Cond) else e


def _cond_elem(c: _Cond, v: Any) -> _Cond:
    _cond_into(c, v)
    return c


def _string_elem(cur: str, v: Any) -> str:
    return _string(v, cur)  # null leaves the element as it is (the zero "" in a fresh backing array)


def _strings() -> _Slice:
    return _Slice(zero=str, into=_string_elem, what="[]string")


class _Names:
    """apiextensions/v1 CustomResourceDefinitionNames: plural, singular,
    shortNames, kind, listKind, categories -- a struct, so a repeated
    acceptedNames key merges into it and null leaves it as it is."""

    def __init__(self):
        self.s = {"plural": "", "singular": "", "kind": "", "listKind": ""}
        self.shortNames = _strings()
        self.categories = _strings()

    def into(self, v: Any) -> None:
        if v is None:
            return
        if not isinstance(v, _Pairs):
            raise DecodeError("acceptedNames is not an object")
        for f, x in _struct_members(v, CRD_NAMES_FIELDS):
            if f in self.s:
                self.s[f] = _string(x, self.s[f])
            else:
                getattr(self, f).decode(x)

    def value(self) -> Tuple:
        return (self.s["plural"], self.s["singular"], self.s["kind"], self.s["listKind"],
                self.shortNames.value(), self.categories.value())


def extract(data: bytes, kind: int = KIND_KCP) -> dict:
    """The fields the classifier reads from one object, or DecodeError.
    kind KIND_CRD reads a CustomResourceDefinition's status (conditions,
    acceptedNames, storedVersions)."""
    if isinstance(data, str):
        data = data.encode("utf-8")
    root = _parse(data)
    rv, gen = "", 0
    labels: Optional[dict] = None
    ann: Optional[dict] = None
    conds = _Slice()
    names = _Names()
    stored = _strings()
    for name, v in _struct_members(root, ("metadata", "status")):
        if v is None:
            continue
        if not isinstance(v, _Pairs):
            raise DecodeError("%s is not an object" % name)
        if name == "metadata":
            for f, x in _struct_members(v, META_FIELDS):
                if f == "resourceVersion":
                    rv = _string(x, rv)
                elif f == "generation":
                    gen = _int64(x, gen)
                elif f == "labels":
                    labels = _string_map(x, labels)
                else:
                    ann = _string_map(x, ann)
        elif kind == KIND_CRD:
            for f, x in _struct_members(v, CRD_STATUS_FIELDS):
                if f == "conditions":
                    conds.decode(x)
                elif f == "acceptedNames":
                    names.into(x)
                else:
                    stored.decode(x)
        else:
            for _, x in _struct_members(v, ("conditions",)):
                conds.decode(x)
    status: Tuple = (conds.value(),)
    if kind == KIND_CRD:
        status = (conds.value(), names.value(), stored.value())
    return {"resourceVersion": rv, "generation": gen, "labels": labels or {},
            "annotations": ann or {}, "conditions": conds.value(), "status": status}


def classify(old: Optional[bytes], new: bytes, kind: int = KIND_KCP) -> int:
    """controller.go:238-295 for one Update event of an object of `kind`."""
    try:
        n = extract(new, kind)
        if old is None:
            return CREATED
        o = extract(old, kind)
    except DecodeError:
        return DECODE
    if o["resourceVersion"] == n["resourceVersion"]:
        return IGNORE
    if o["generation"] != n["generation"]:
        return SPEC_CHANGED
    if o["status"] != n["status"]:   # Semantic.DeepEqual: nil == empty slices; times by instant
        return STATUS_ONLY
    if o["annotations"] != n["annotations"] or o["labels"] == n["labels"]:
        return META_ONLY
    return IGNORE


def classify_batch(pairs: List[Tuple[Optional[bytes], bytes]], kind: int = KIND_KCP) -> List[int]:
    return [classify(a, b, kind) for a, b in pairs]

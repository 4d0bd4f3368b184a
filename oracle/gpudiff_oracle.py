"""CPU oracle for the kcp syncer change-detection hot path (TEST INFRASTRUCTURE ONLY).

This module is a checker. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it. The product path
(``kcp_amd``) never imports, links or calls anything under ``oracle/``.

What it restates (reference paths relative to /root/reference):

* ``deepEqualApartFromStatus``  -- pkg/syncer/specsyncer.go:17-41
* ``deepEqualStatus``           -- pkg/syncer/statussyncer.go:15-27
* ``equality.Semantic.DeepEqual`` on JSON-derived unstructured content,
  ``Unstructured.GetLabels/GetAnnotations`` (NestedStringMap) and the k8s
  JSON decode rules of ``k8s.io/apimachinery/pkg/util/json`` over Go's
  ``encoding/json``.  These live in the third-party module pinned at
  go.mod:33 (github.com/kcp-dev/kubernetes/staging/src/k8s.io/apimachinery
  v0.0.0-20211004150937-c954268bf177) and Go 1.16's encoding/json, neither of
  which is vendored in /root/reference; they are restated here from their
  published algorithms.
* the build-defined field-path diff and canonical
  leaf encoding (DESIGN.md "Canonical encoding").

PARITY STATUS: the reference has no tests for pkg/syncer and its Go toolchain
and module cache are absent, so no reference-run vectors exist.  This oracle is
pinned by (a) the known-answer table of SURVEY.md Appendix A.4 (tests/
test_oracle_kat.py), (b) xxh64 vectors from the Python ``xxhash`` 3.8.1 package
(the published XXH64 algorithm), (c) property tests of the two theorems
specDirty <=> P_spec != {} and statusDirty <=> P_status != {}.  Against the
reference *run* itself parity is UNPINNED (DESIGN.md "Parity status").
"""
from __future__ import annotations

import math
import struct
import sys
from typing import Any, Dict, List, Optional, Tuple

import xxhash

sys.setrecursionlimit(max(sys.getrecursionlimit(), 50000))

# ---------------------------------------------------------------------------
# Go encoding/json decode (UseNumber) + k8s util/json number conversion
# ---------------------------------------------------------------------------

MAX_DEPTH = 10000          # encoding/json scanner maxNestingDepth
INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1


class DecodeError(ValueError):
    pass


_WS = b" \t\r\n"
_ESC = {ord('"'): 0x22, ord('\\'): 0x5C, ord('/'): 0x2F, ord('b'): 0x08,
        ord('f'): 0x0C, ord('n'): 0x0A, ord('r'): 0x0D, ord('t'): 0x09}
_REPL = "�".encode()


def _go_decode_rune(b: bytes, i: int) -> Tuple[int, int]:
    """utf8.DecodeRune semantics: (rune, size); invalid -> (-1, 1)."""
    n = len(b)
    c0 = b[i]
    if c0 < 0x80:
        return c0, 1
    if 0xC2 <= c0 <= 0xDF:
        size, lo, hi, acc = 2, 0x80, 0xBF, c0 & 0x1F
    elif c0 == 0xE0:
        size, lo, hi, acc = 3, 0xA0, 0xBF, c0 & 0x0F
    elif 0xE1 <= c0 <= 0xEC or 0xEE <= c0 <= 0xEF:
        size, lo, hi, acc = 3, 0x80, 0xBF, c0 & 0x0F
    elif c0 == 0xED:
        size, lo, hi, acc = 3, 0x80, 0x9F, c0 & 0x0F
    elif c0 == 0xF0:
        size, lo, hi, acc = 4, 0x90, 0xBF, c0 & 0x07
    elif 0xF1 <= c0 <= 0xF3:
        size, lo, hi, acc = 4, 0x80, 0xBF, c0 & 0x07
    elif c0 == 0xF4:
        size, lo, hi, acc = 4, 0x80, 0x8F, c0 & 0x07
    else:
        return -1, 1
    if i + size > n:
        # Go: a short sequence is RuneError,1 (after checking what exists)
        return -1, 1
    c1 = b[i + 1]
    if not (lo <= c1 <= hi):
        return -1, 1
    acc = (acc << 6) | (c1 & 0x3F)
    for k in range(2, size):
        ck = b[i + k]
        if not (0x80 <= ck <= 0xBF):
            return -1, 1
        acc = (acc << 6) | (ck & 0x3F)
    return acc, size


_HEX_DIGITS = frozenset(b"0123456789abcdefABCDEF")


def _getu4(b: bytes, i: int) -> int:
    if i + 6 > len(b) or b[i] != 0x5C or b[i + 1] != ord('u'):
        return -1
    h = b[i + 2:i + 6]
    # four hex digits exactly (decode.go getu4); int(..., 16) alone would also take whitespace, a sign or '_'
    if any(c not in _HEX_DIGITS for c in h):
        return -1
    return int(h.decode('ascii'), 16)


class _Parser:
    def __init__(self, data: bytes):
        self.b = data
        self.i = 0
        self.n = len(data)

    def ws(self):
        b, i, n = self.b, self.i, self.n
        while i < n and b[i] in _WS:
            i += 1
        self.i = i

    def value(self, depth: int):
        self.ws()
        if self.i >= self.n:
            raise DecodeError("unexpected end")
        c = self.b[self.i]
        if c == ord('{'):
            return self.obj(depth + 1)
        if c == ord('['):
            return self.arr(depth + 1)
        if c == ord('"'):
            return self.string()
        if c == ord('t'):
            return self.lit(b"true", True)
        if c == ord('f'):
            return self.lit(b"false", False)
        if c == ord('n'):
            return self.lit(b"null", None)
        if c == ord('-') or 0x30 <= c <= 0x39:
            return self.number()
        raise DecodeError("invalid character %r" % chr(c))

    def lit(self, word: bytes, val):
        if self.b[self.i:self.i + len(word)] != word:
            raise DecodeError("invalid literal")
        self.i += len(word)
        return val

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
        is_int = True
        if i < n and b[i] == ord('.'):
            is_int = False
            i += 1
            if i >= n or not (0x30 <= b[i] <= 0x39):
                raise DecodeError("bad fraction")
            while i < n and 0x30 <= b[i] <= 0x39:
                i += 1
        if i < n and b[i] in b"eE":
            is_int = False
            i += 1
            if i < n and b[i] in b"+-":
                i += 1
            if i >= n or not (0x30 <= b[i] <= 0x39):
                raise DecodeError("bad exponent")
            while i < n and 0x30 <= b[i] <= 0x39:
                i += 1
        self.i = i
        text = b[s:i].decode('ascii')
        # k8s util/json convertNumber: json.Number.Int64() (strconv.ParseInt
        # base 10) first, then Float64() (strconv.ParseFloat, correctly
        # rounded; +-Inf on overflow is an error).
        if is_int:
            v = int(text)
            if INT64_MIN <= v <= INT64_MAX:
                return v
        f = float(text)
        if math.isinf(f):
            raise DecodeError("float overflow")
        return f

    def string(self) -> str:
        b, n = self.b, self.n
        i = self.i + 1
        out = bytearray()
        while True:
            if i >= n:
                raise DecodeError("unterminated string")
            c = b[i]
            if c == 0x22:
                i += 1
                break
            if c == 0x5C:
                if i + 1 >= n:
                    raise DecodeError("bad escape")
                e = b[i + 1]
                if e in _ESC:
                    out.append(_ESC[e])
                    i += 2
                    continue
                if e == ord('u'):
                    rr = _getu4(b, i)
                    if rr < 0:
                        raise DecodeError("bad \\u escape")
                    i += 6
                    if 0xD800 <= rr < 0xE000:
                        rr1 = _getu4(b, i)
                        if 0xD800 <= rr < 0xDC00 and 0xDC00 <= rr1 < 0xE000:
                            dec = (((rr - 0xD800) << 10) | (rr1 - 0xDC00)) + 0x10000
                            out += chr(dec).encode('utf-8')
                            i += 6
                            continue
                        rr = 0xFFFD
                    out += chr(rr).encode('utf-8')
                    continue
                raise DecodeError("bad escape")
            if c < 0x20:
                raise DecodeError("control character in string")
            if c < 0x80:
                out.append(c)
                i += 1
                continue
            r, size = _go_decode_rune(b, i)
            if r < 0:
                out += _REPL
                i += 1
            else:
                out += b[i:i + size]
                i += size
        self.i = i
        return out.decode('utf-8')

    def obj(self, depth: int) -> Dict[str, Any]:
        if depth > MAX_DEPTH:                 # scanner maxNestingDepth
            raise DecodeError("exceeded max depth")
        self.i += 1
        m: Dict[str, Any] = {}
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
            v = self.value(depth)
            if k in m:          # duplicate key: last one wins
                del m[k]
            m[k] = v
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

    def arr(self, depth: int) -> List[Any]:
        if depth > MAX_DEPTH:
            raise DecodeError("exceeded max depth")
        self.i += 1
        a: List[Any] = []
        self.ws()
        if self.i < self.n and self.b[self.i] == ord(']'):
            self.i += 1
            return a
        while True:
            a.append(self.value(depth))
            self.ws()
            if self.i >= self.n:
                raise DecodeError("unterminated array")
            c = self.b[self.i]
            self.i += 1
            if c == ord(','):
                continue
            if c == ord(']'):
                return a
            raise DecodeError("expected , or ]")


def go_json_decode(data: bytes) -> Dict[str, Any]:
    """Decode one unstructured object the way the informer's JSON scheme does.

    Top level must be an object; trailing non-whitespace is rejected (the build
    treats it as a decode error -> pair reported dirty)."""
    if isinstance(data, str):
        data = data.encode('utf-8')
    p = _Parser(data)
    p.ws()
    if p.i >= p.n or p.b[p.i] != ord('{'):
        raise DecodeError("top level is not an object")
    v = p.value(0)
    p.ws()
    if p.i != p.n:
        raise DecodeError("trailing data")
    return v


class NotUnstructured(DecodeError):
    """The informer's decoder yields an UnstructuredList, not an Unstructured."""


_SMALL_LONG_ESS, _KELVIN = 0x17F, 0x212A


def go_equal_fold_right(name: bytes, key: bytes) -> bool:
    """encoding/json fold.go equalFoldRight (Go 1.16), the matcher Go picks for
    a field name holding 's' or 'k': ASCII case folding, plus U+017F (long s)
    for s/S and U+212A (Kelvin sign) for k/K."""
    t = key
    for sb in name:
        if not t:
            return False
        tb = t[0]
        if tb < 0x80:
            if sb != tb:
                up = sb & 0xDF
                if not (0x41 <= up <= 0x5A) or up != (tb & 0xDF):
                    return False
            t = t[1:]
            continue
        r, size = _go_decode_rune(t, 0)
        if sb in b"sS":
            if r != _SMALL_LONG_ESS:
                return False
        elif sb in b"kK":
            if r != _KELVIN:
                return False
        else:
            return False
        t = t[size:]
    return not t


def is_list_probe_match(obj: Dict[str, Any]) -> bool:
    """apimachinery unstructuredJSONScheme.decode [3P] first unmarshals the
    bytes into ``struct{ Items json.RawMessage }`` with encoding/json: a
    top-level key equal to "Items" under Go's case folding -- with any value,
    ``null`` included (RawMessage.UnmarshalJSON keeps the 4 bytes) -- makes
    ``Items != nil`` and the object decodes as an UnstructuredList."""
    return any(go_equal_fold_right(b"Items", k.encode("utf-8", "surrogatepass")) for k in obj)


def informer_decode(data: bytes) -> Dict[str, Any]:
    """What reaches the predicates: go_json_decode, then the list probe of the
    informer's JSON scheme (reached from pkg/syncer/syncer.go:105-108).  A
    list-shaped object is not an *unstructured.Unstructured, so both type
    assertions (specsyncer.go:18-22, statussyncer.go:16-20) fail and both
    predicates return false: the pair is dirty, like a decode error.  (In a
    live informer the reflector drops such a watch event on its expectedType
    check; the batch API receives JSON pairs and keeps the predicates' rule.)"""
    obj = go_json_decode(data)
    if is_list_probe_match(obj):
        raise NotUnstructured("decodes as an UnstructuredList")
    return obj


def _nesting_bound(data: bytes) -> int:
    return data.count(b"[") + data.count(b"{")


def _on_big_stack(fn, *args):
    """Runs fn on a thread with a 1 GiB stack: the recursive restatement goes
    as deep as Go's 10000-level nesting limit."""
    import threading
    box = {}

    def run():
        try:
            box["r"] = fn(*args)
        except BaseException as e:  # re-raised on the caller's thread
            box["e"] = e
    old = threading.stack_size(1 << 30)
    try:
        t = threading.Thread(target=run)
        t.start()
    finally:
        threading.stack_size(old)
    t.join()
    if "e" in box:
        raise box["e"]
    return box["r"]


# ---------------------------------------------------------------------------
# equality.Semantic.DeepEqual restricted to JSON-derived values  [3P]
# ---------------------------------------------------------------------------

def deep_equal(x: Any, y: Any) -> bool:
    """Forked reflect DeepEqual (apimachinery third_party/forked/golang/reflect):
    nil interfaces equal only each other; dynamic types must match exactly;
    empty and nil maps/slices are equal; maps by length + per-key; slices
    element-wise; scalars by Go ==."""
    if x is None or y is None:
        return x is None and y is None
    tx = type(x)
    if tx is not type(y):
        return False
    if tx is dict:
        if len(x) == 0 or len(y) == 0:
            return len(x) == 0 and len(y) == 0
        if len(x) != len(y):
            return False
        for k, v in x.items():
            if k not in y:
                return False
            if not deep_equal(v, y[k]):
                return False
        return True
    if tx is list:
        if len(x) == 0 or len(y) == 0:
            return len(x) == 0 and len(y) == 0
        if len(x) != len(y):
            return False
        return all(deep_equal(a, b) for a, b in zip(x, y))
    return x == y


def nested_string_map(obj: Dict[str, Any], *fields: str) -> Optional[Dict[str, str]]:
    """unstructured.NestedStringMap as used by GetLabels/GetAnnotations: nil if
    any step is missing or not a map, or if any value is not a string."""
    v: Any = obj
    for f in fields:
        if type(v) is not dict or f not in v:
            return None
        v = v[f]
    if type(v) is not dict:
        return None
    out: Dict[str, str] = {}
    for k, val in v.items():
        if type(val) is not str:
            return None
        out[k] = val
    return out


def _de_string_map(a: Optional[Dict[str, str]], b: Optional[Dict[str, str]]) -> bool:
    # typed map[string]string: nil and empty compare equal under the fork
    if not a or not b:
        return not a and not b
    return a == b


def deep_equal_apart_from_status(old: Dict[str, Any], new: Dict[str, Any]) -> bool:
    """pkg/syncer/specsyncer.go:17-41."""
    if not _de_string_map(nested_string_map(old, "metadata", "annotations"),
                          nested_string_map(new, "metadata", "annotations")):
        return False                                            # :23
    if not _de_string_map(nested_string_map(old, "metadata", "labels"),
                          nested_string_map(new, "metadata", "labels")):
        return False                                            # :26
    for key in set(old) | set(new):                             # :30-32
        if key == "metadata" or key == "status":               # :33-35
            continue
        if not deep_equal(old.get(key), new.get(key)):         # :36
            return False
    return True


def deep_equal_status(old: Dict[str, Any], new: Dict[str, Any]) -> bool:
    """pkg/syncer/statussyncer.go:15-27 (asymmetric: new must have 'status')."""
    if "status" in new:                                        # :22
        return deep_equal(old.get("status"), new["status"])    # :23-24
    return False                                               # :26


# ---------------------------------------------------------------------------
# Canonical leaves and the field-path diff (build-defined)
# ---------------------------------------------------------------------------

TAG_NULL, TAG_FALSE, TAG_TRUE, TAG_INT, TAG_FLOAT, TAG_STR, TAG_EOBJ, TAG_EARR = range(8)
KIND_CHANGED, KIND_ADDED, KIND_REMOVED, KIND_STATUS_ABSENT = 0, 1, 2, 3
REGION_SPEC, REGION_STATUS = 0, 1
# the build's path-hash width (include/gpudiff_format.h GPUDIFF_PATH_HASH_BITS):
# segments keep, and results report, the chained hash cut to 32 bits
PATH_HASH_BITS = 32

Path = Tuple[Tuple[str, Any], ...]


def encode_path(path: Path) -> bytes:
    out = bytearray()
    for kind, c in path:
        if kind == 'K':
            kb = c.encode('utf-8')
            out += b'\x01' + struct.pack('<I', len(kb)) + kb
        else:
            out += b'\x02' + struct.pack('<I', c)
    return bytes(out)


def path_hash(path: Path, seed: int = 0) -> int:
    """Chained XXH64 over the path's encoded components (build-defined, as the
    whole field-path diff is): h(()) = seed and
    h(p + (c,)) = XXH64(encode_path((c,)), seed=h(p)).  A child's hash is a
    function of its parent's hash and its own component only, which is what
    lets the device tokenizer hash a document tree level by level."""
    h = seed
    for comp in path:
        h = xxhash.xxh64_intdigest(encode_path((comp,)), seed=h)
    return h


def render_path(path: Path) -> str:
    s = ""
    for kind, c in path:
        if kind == 'K':
            s += ("." if s else "") + c
        else:
            s += "[%d]" % c
    return s


def canonical_value(x: Any) -> Tuple[int, bytes]:
    t = type(x)
    if x is None:
        return TAG_NULL, b""
    if t is bool:
        return (TAG_TRUE if x else TAG_FALSE), b""
    if t is int:
        return TAG_INT, struct.pack('<q', x)
    if t is float:
        return TAG_FLOAT, struct.pack('<d', 0.0 if x == 0.0 else x)
    if t is str:
        return TAG_STR, x.encode('utf-8')
    if t is dict:
        assert not x
        return TAG_EOBJ, b""
    if t is list:
        assert not x
        return TAG_EARR, b""
    raise TypeError(t)


def _flatten(x: Any, path: Path, out: Dict[Path, Tuple[int, bytes]]):
    if type(x) is dict and x:
        for k, v in x.items():
            _flatten(v, path + (('K', k),), out)
    elif type(x) is list and x:
        for i, v in enumerate(x):
            _flatten(v, path + (('I', i),), out)
    else:
        out[path] = canonical_value(x)


def spec_leaves(obj: Dict[str, Any]) -> Dict[Path, Tuple[int, bytes]]:
    """Regions S (top-level keys except metadata/status, top-level nulls
    dropped), L (canonical labels) and N (canonical annotations)."""
    out: Dict[Path, Tuple[int, bytes]] = {}
    for k, v in obj.items():
        if k in ("metadata", "status") or v is None:
            continue
        _flatten(v, (('K', k),), out)
    for field in ("labels", "annotations"):
        m = nested_string_map(obj, "metadata", field)
        if m:
            for k, v in m.items():
                out[(('K', 'metadata'), ('K', field), ('K', k))] = (TAG_STR, v.encode('utf-8'))
    return out


def status_leaves(obj: Dict[str, Any]) -> Dict[Path, Tuple[int, bytes]]:
    out: Dict[Path, Tuple[int, bytes]] = {}
    if obj.get("status") is not None:
        _flatten(obj["status"], (('K', 'status'),), out)
    return out


def _region_diff(la, lb, seed: int, region: int, mask: int):
    res = []
    for p in set(la) | set(lb):
        a, b = la.get(p), lb.get(p)
        if a == b:
            continue
        kind = KIND_ADDED if a is None else KIND_REMOVED if b is None else KIND_CHANGED
        res.append((path_hash(p, seed) & mask, region, kind, p))
    res.sort(key=lambda e: e[0])
    return res


MAX_SEED = 255


def pair_seed(sa, sb, ta, tb, hash_bits: int = PATH_HASH_BITS) -> int:
    """Smallest seed s in [0, 255] for which the path hash is injective over
    the pair's spec-path union and, separately, over its status-path union
    plus the sentinel path ``status`` (the build re-seeds per pair on a
    collision; results carry the region bit, so (region, hash) is exact).
    Returns -1 if no seed works (the pair is then reported dirty, like a
    decode error)."""
    mask = (1 << hash_bits) - 1
    spec_paths = set(sa) | set(sb)
    stat_paths = set(ta) | set(tb) | {(('K', 'status'),)}
    for s in range(MAX_SEED + 1):
        ok = True
        for paths in (spec_paths, stat_paths):
            hs = {}
            for p in paths:
                h = path_hash(p, s) & mask
                if h in hs and hs[h] != p:
                    ok = False
                    break
                hs[h] = p
            if not ok:
                break
        if ok:
            return s
    return -1


def diff_pair(a_json: bytes, b_json: bytes, hash_bits: int = PATH_HASH_BITS) -> Dict[str, Any]:
    """Oracle result for one (A=old/upstream, B=new/downstream) pair.

    Returns spec_dirty, status_dirty, decode_error, seed and the changed-path
    list [(pathHash, region, kind, path)] in output order: spec entries by
    ascending pathHash, then status entries by ascending pathHash, then the
    status-absent-in-new sentinel."""
    if isinstance(a_json, str):
        a_json = a_json.encode("utf-8")
    if isinstance(b_json, str):
        b_json = b_json.encode("utf-8")
    if _nesting_bound(a_json) + _nesting_bound(b_json) > 1000:
        return _on_big_stack(_diff_pair, a_json, b_json, hash_bits)
    return _diff_pair(a_json, b_json, hash_bits)


def _diff_pair(a_json: bytes, b_json: bytes, hash_bits: int) -> Dict[str, Any]:
    try:
        a = informer_decode(a_json)
        b = informer_decode(b_json)
    except DecodeError:
        return dict(spec_dirty=True, status_dirty=True, decode_error=True, seed=0, paths=[], spec_noop=False,
                    status_noop=False)
    sa, sb = spec_leaves(a), spec_leaves(b)
    ta, tb = status_leaves(a), status_leaves(b)
    seed = pair_seed(sa, sb, ta, tb, hash_bits)
    if seed < 0:
        return dict(spec_dirty=True, status_dirty=True, decode_error=True, seed=0, paths=[], spec_noop=False,
                    status_noop=False)
    spec_dirty = not deep_equal_apart_from_status(a, b)
    status_dirty = not deep_equal_status(a, b)
    mask = (1 << hash_bits) - 1
    paths = _region_diff(sa, sb, seed, REGION_SPEC, mask)
    spec_noop = spec_dirty and all(wire_equal_number(sa.get(p), sb.get(p)) for _h, _r, _k, p in paths)
    status_noop = False
    if status_dirty:
        tpaths = _region_diff(ta, tb, seed, REGION_STATUS, mask)
        status_noop = all(wire_equal_number(ta.get(p), tb.get(p)) for _h, _r, _k, p in tpaths)
        paths += tpaths
        if "status" not in b:
            sp = (('K', 'status'),)
            paths.append((path_hash(sp, seed) & mask, REGION_STATUS, KIND_STATUS_ABSENT, sp))
            status_noop = status_noop and "status" not in a
    return dict(spec_dirty=spec_dirty, status_dirty=status_dirty, decode_error=False,
                seed=seed, paths=paths, spec_noop=spec_noop, status_noop=status_noop)


def wire_equal_number(la, lb) -> bool:
    """The write-path no-op rule for one changed leaf (build-defined, DESIGN.md
    §4g): an int64 v on one side and a float64 f == v on the other, |v| <=
    2^53.  Go's json.Marshal writes float64(v) and int64(v) as the same digits
    for such values, and the API server decodes those digits back to int64 v
    (k8s util/json convertNumber), so writing one side over the other changes
    nothing a predicate compares."""
    if la is None or lb is None:
        return False
    (ta, ba), (tb, bb) = la, lb
    if {ta, tb} != {TAG_INT, TAG_FLOAT}:
        return False
    v = struct.unpack('<q', ba if ta == TAG_INT else bb)[0]
    f = struct.unpack('<d', bb if ta == TAG_INT else ba)[0]
    return -(1 << 53) <= v <= (1 << 53) and float(v) == f


def theorem_holds(a_json: bytes, b_json: bytes) -> bool:
    """specDirty <=> P_spec != {} and statusDirty <=> P_status != {}."""
    if _nesting_bound(a_json) + _nesting_bound(b_json) > 1000:
        return _on_big_stack(_theorem_holds, a_json, b_json)
    return _theorem_holds(a_json, b_json)


def _theorem_holds(a_json: bytes, b_json: bytes) -> bool:
    r = _diff_pair(a_json, b_json, PATH_HASH_BITS)
    if r["decode_error"]:
        return True
    ps = [e for e in r["paths"] if e[1] == REGION_SPEC]
    pt = [e for e in r["paths"] if e[1] == REGION_STATUS]
    a = informer_decode(a_json)
    b = informer_decode(b_json)
    s_leaf = spec_leaves(a) != spec_leaves(b)
    t_leaf = (status_leaves(a) != status_leaves(b)) or ("status" not in b)
    return (r["spec_dirty"] == bool(ps) == s_leaf) and (r["status_dirty"] == bool(pt) == t_leaf)

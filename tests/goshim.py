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
from typing import Any, List, Optional, Tuple

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


# ---------------------------------------------------------------- Batcher (gpudiff.go Batcher.loop / flush)
SPEC_DIRTY, STATUS_DIRTY = 0x1, 0x2  # GPUDIFF_SPEC_DIRTY / GPUDIFF_STATUS_DIRTY: the Which of an event


class JsonBuf:
    """gpudiff.go jsonBuf: every object of one flush rendered into ONE buffer (the Go side's C
    allocation); objects are addressed by (offset, length), pointers are taken only after the last
    add (the buffer may move while it grows)."""

    def __init__(self, pinned: bool = False):
        """pinned: the engine-pinned buffer of a device-encode engine (gpudiff_host_alloc) in the zero-copy
        layout -- each object followed by zeros up to its staged span, len + 32 rounded up to 16 (span),
        and 32 more bytes after the last (tail)"""
        self.buf = bytearray()
        self.pinned = pinned

    def _span(self, start: int):
        if self.pinned:
            n = len(self.buf) - start
            self.buf += bytes(((n + 32 + 15) & ~15) - n)

    def add(self, tree) -> Optional[Tuple[int, int]]:
        if tree is None:  # not an *unstructured.Unstructured: nothing added
            return None
        j = shim_json(tree)
        if j is None:  # not transferable: the partial object is dropped
            return None
        off = len(self.buf)
        self.buf += j
        self._span(off)
        return off, len(j)

    def raw(self, b: bytes) -> Tuple[int, int]:
        off = len(self.buf)
        self.buf += b
        self._span(off)
        return off, len(b)

    def tail(self):
        if self.pinned:
            self.buf += bytes(32)

    def mark(self) -> int:
        return len(self.buf)

    def truncate(self, m: int):
        del self.buf[m:]


class Batcher:
    """Restatement of gpudiff.go's Batcher over a simulated clock: events arrive as
    (t, old_json, new_json, which, name); a flush happens when maxBatch events are pending or `window`
    has passed since the timer was last armed.  The timer is re-armed after every loop turn; the Go
    code stops and drains it first, so a tick that fired while a full batch was being flushed does NOT
    flush the next (small) batch at once.  `drain=False` models the old code (Reset without draining).
    decide(pairs) -> flags per pair (the engine: gpudiff_submit + gpudiff_wait; the oracle in CPU
    tests).  Dirty events are enqueued in arrival order; a pair the shim cannot transfer is enqueued
    without asking the engine (specsyncer.go:20-22)."""

    def __init__(self, decide, max_batch: int, window: float, flush_cost: float = 0.0, drain: bool = True,
                 engine=None):
        """engine (NewBatcherPipelined): an object with submit(pairs) -> ticket and wait(ticket) -> flags; batch
        k + 1 is submitted before batch k is waited and enqueued, and a window with no new events settles the
        batch in flight."""
        self.decide, self.max_batch, self.window = decide, max_batch, window
        self.flush_cost, self.drain, self.engine = flush_cost, drain, engine
        self.enqueued: List[str] = []
        self.flushes: List[int] = []
        self.buffers: List[bytes] = []
        self.inflight = None
        self.pinned = False  # a device-encode engine: flush buffers in the zero-copy layout (gpudiff.go jsonBuf.e)
        self.layouts: List[list] = []

    def _stage(self, evs):
        jb = JsonBuf(self.pinned)
        bad, offs = [], []
        for (_t, a, b, _which, _name) in evs:
            m = jb.mark()
            oa = jb.add(informer_object(a))
            ob = jb.add(informer_object(b)) if oa is not None else None
            if oa is None or ob is None:
                jb.truncate(m)
                oa, ob = jb.raw(b"{}"), jb.raw(b"{}")  # two copies: the zero-copy layout wants pair order
                bad.append(True)
            else:
                bad.append(False)
            offs.append((oa, ob))
        jb.tail()
        buf = bytes(jb.buf)
        self.buffers.append(buf)
        self.layouts.append(offs)
        return bad, [(buf[oa[0]:oa[0] + oa[1]], buf[ob[0]:ob[0] + ob[1]]) for oa, ob in offs]

    def _enqueue(self, evs, flags, bad):
        for (ev, f, bd) in zip(evs, flags, bad):
            if bd or (f & ev[3]):
                self.enqueued.append(ev[4])

    def flush(self, evs):
        bad, pairs = self._stage(evs)
        self.flushes.append(len(evs))
        if self.engine is None:
            self._enqueue(evs, self.decide(pairs), bad)
            return
        # pipelined (gpudiff.go submitFlight / finishFlight): submit this batch, then settle the one before
        flight = (list(evs), bad, self.engine.submit(pairs))
        self.settle()
        self.inflight = flight

    def settle(self):
        if self.inflight is not None:
            evs, bad, ticket = self.inflight
            self.inflight = None
            self._enqueue(evs, self.engine.wait(ticket), bad)

    def run(self, events):
        """events sorted by arrival time; returns the enqueued names in order.  Events that arrived while
        a flush ran wait in the channel (the Go side's buffered chan); when both a queued event and a
        fired tick are ready, Go's select picks at random -- modeled as: one event, then the tick."""
        pending = []
        now = 0.0
        deadline = self.window  # timer armed at 0
        stale_tick = False      # a fired tick left in the channel (the old Reset-without-drain code)
        i = 0
        while i < len(events) or pending or self.inflight is not None:
            nxt = events[i][0] if i < len(events) else float("inf")
            if stale_tick:
                stale_tick = False
                if nxt <= now:
                    pending.append(events[i])
                    i += 1
                fire = True
            elif nxt <= deadline:
                now = max(now, nxt)
                pending.append(events[i])
                i += 1
                if len(pending) < self.max_batch:
                    continue
                fire = False
            else:
                now = max(now, deadline)
                fire = True
            if pending:
                self.flush(pending)
                pending = []
            elif fire:
                self.settle()  # a window with no new events: the batch in flight is waited and enqueued
            now += self.flush_cost
            if not fire and now >= deadline and not self.drain:
                stale_tick = True  # the timer fired during the flush and Reset does not drain it
            deadline = now + self.window
        return self.enqueued


# ---------------------------------------------------------------- gpudiff.go Batcher.submitStored (store path)
def stage_stored(evs, seen: set, pinned: bool = True):
    """gpudiff.go submitStored for one flush of store events [(slot, old_json or None, new_json)] whose new object
    is an *unstructured.Unstructured (the others never reach the store).  On a device-encode store (pinned) the
    documents the store encodes go into ONE engine-pinned buffer in the zero-copy layout, in order: a slot's old
    object when the slot is new to the store (`seen`, the Go Store.seen mirror, updated here), then the new object
    (an untransferable one as the undecodable "{"); every other old object -- read only on a collision -- goes into a
    plain buffer of its own.  Returns (pinned bytes, plain bytes, [(slot, new (off, len), old (off, len) or None,
    old in the pinned buffer)])."""
    jb, jold = JsonBuf(pinned), JsonBuf(False)
    entries = []
    for slot, old, new in evs:
        o, in_jb = None, False
        tree_old = informer_object(old) if old is not None else None
        if slot not in seen:
            o = jb.add(tree_old)
            in_jb = o is not None
        else:
            o = jold.add(tree_old)
        seen.add(slot)
        n = jb.add(informer_object(new))
        if n is None:
            n = jb.raw(b"{")  # undecodable: reported dirty, slot emptied
        entries.append((slot, n, o, in_jb))
    jb.tail()
    return bytes(jb.buf), bytes(jold.buf), entries

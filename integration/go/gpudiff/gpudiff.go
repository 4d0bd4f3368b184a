// Package gpudiff is the cgo binding a kcp maintainer adds as pkg/gpudiff to
// route the syncer's change-detection predicates
// (pkg/syncer/specsyncer.go:17-41, pkg/syncer/statussyncer.go:15-27) to the
// MI355X engine behind include/gpudiff.h.
//
// Compile-untested here: this image has no Go toolchain (see DESIGN.md §8).
package gpudiff

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../kcp_amd -lgpudiff -Wl,-rpath,${SRCDIR}/../../../kcp_amd
#include <stdlib.h>
#include "gpudiff.h"
*/
import "C"

import (
	"bytes"
	"errors"
	"fmt"
	"math"
	"strconv"
	"sync"
	"time"
	"unicode/utf8"
	"unsafe"

	"k8s.io/apimachinery/pkg/apis/meta/v1/unstructured"
)

// Engine owns one gpudiff context (one GPU, one stream).  A context is not
// reentrant, so every call goes through mu; the Batcher is the intended
// single submitter.
type Engine struct {
	mu     sync.Mutex
	ctx    *C.gpudiff_ctx
	devEnc bool // GPUDIFF_OPT_DEVICE_ENCODE: the batcher renders flushes into engine-pinned memory
}

func errOf(rc C.int) error {
	if rc == C.GPUDIFF_OK {
		return nil
	}
	return fmt.Errorf("gpudiff: %s (%d)", C.GoString(C.gpudiff_strerror(rc)), int(rc))
}

// Open creates an engine on HIP device `device` (-1 = current).
func Open(device int) (*Engine, error) {
	return OpenWith(device, 0)
}

// OpenWith is Open with GPUDIFF_OPT_* flags, e.g. C.GPUDIFF_OPT_DEVICE_ENCODE to send the
// batcher's JSON pairs to the GPU tokenizer (kernel K0) instead of the host encoder.
func OpenWith(device int, flags uint32) (*Engine, error) {
	// the header this package was built against must match the library loaded at run time (ABI 4: value
	// heads in the leaf records, no value digests; the digest options are ignored)
	if v := int(C.gpudiff_abi_version()); v != int(C.GPUDIFF_ABI_VERSION) {
		return nil, fmt.Errorf("gpudiff: libgpudiff.so has ABI %d, this binding was built for %d", v, int(C.GPUDIFF_ABI_VERSION))
	}
	var opts C.gpudiff_opts
	opts.device = C.int32_t(device)
	opts.flags = C.uint32_t(flags)
	var ctx *C.gpudiff_ctx
	if err := errOf(C.gpudiff_open(&opts, &ctx)); err != nil {
		return nil, err
	}
	return &Engine{ctx: ctx, devEnc: flags&uint32(C.GPUDIFF_OPT_DEVICE_ENCODE) != 0}, nil
}

func (e *Engine) Close() {
	e.mu.Lock()
	defer e.mu.Unlock()
	if e.ctx != nil {
		C.gpudiff_close(e.ctx)
		e.ctx = nil
	}
}

// jsonOf renders an informer object as the JSON text the engine decodes.
//
// Marker contract.  The engine reads numbers with k8s util/json's rule (an integer literal ->
// int64, a literal with a fraction or an exponent -> float64), and the predicates compare Go
// dynamic types (equality.Semantic.DeepEqual: int64(3) != float64(3), specsyncer.go:36;
// SURVEY.md A.4 rows 7/8/25/26).  u.MarshalJSON cannot be used: encoding/json writes
// float64(3) as "3" and float64(-0) as "-0", which the engine reads back as int64 -- an
// int64-vs-float64 difference would come out "equal".  appendValue writes instead:
//
//	int64                  decimal digits, never a '.', 'e' or 'E'
//	float64                shortest round-trip digits (strconv 'g', -1) that always carry a '.'
//	                       or an exponent: 3 -> "3.0", -0 -> "-0.0", 1e21 -> "1e+21";
//	                       NaN / Inf -> not transferable
//	string, map key        a JSON string whose decoded bytes are the Go string's bytes
//	                       (only '"', '\\' and bytes < 0x20 escaped); a string that is not
//	                       valid UTF-8 -> not transferable (the decoder would fold it to U+FFFD)
//	bool, nil              true / false / null
//	map[string]interface{} an object (Go's iteration order: the engine's encoding is canonical)
//	[]interface{}          an array
//	anything else          not transferable: int, int32, float32, json.Number, structs ... never
//	                       come out of the informer's JSON decode, DeepEqual tells them apart from
//	                       int64/float64 by type, so no JSON text can stand for them
//	nesting deeper than 10000 containers: not transferable (encoding/json's limit)
//
// A not-transferable object gives ok = false, which every caller treats as "differs" -- the
// reference's rule for a failed type assertion (specsyncer.go:20-22) -- so the transfer can
// cost an unnecessary enqueue, never a false "equal".  tests/goshim.py restates this function
// and tests/test_gpu_goshim.py runs every known-answer and golden pair through that restatement
// and the C-ABI against the oracle.  It is also cheaper than MarshalJSON on the informer path: no
// reflection, no key sort and no HTML escaping.
func jsonOf(obj interface{}) ([]byte, bool) {
	u, ok := obj.(*unstructured.Unstructured)
	if !ok || u == nil {
		return nil, false
	}
	var m interface{} = u.Object
	if u.Object == nil {
		m = map[string]interface{}{}
	}
	return appendValue(make([]byte, 0, 2048), m, 0)
}

const maxNesting = 10000 // encoding/json scanner maxNestingDepth

func appendValue(buf []byte, v interface{}, depth int) ([]byte, bool) {
	switch x := v.(type) {
	case nil:
		return append(buf, "null"...), true
	case bool:
		if x {
			return append(buf, "true"...), true
		}
		return append(buf, "false"...), true
	case int64:
		return strconv.AppendInt(buf, x, 10), true
	case float64:
		if math.IsNaN(x) || math.IsInf(x, 0) {
			return buf, false
		}
		start := len(buf)
		buf = strconv.AppendFloat(buf, x, 'g', -1, 64)
		if bytes.IndexAny(buf[start:], ".eE") < 0 {
			buf = append(buf, '.', '0')
		}
		return buf, true
	case string:
		return appendString(buf, x)
	case map[string]interface{}:
		if depth+1 > maxNesting {
			return buf, false
		}
		buf = append(buf, '{')
		first := true
		for k, e := range x {
			if !first {
				buf = append(buf, ',')
			}
			first = false
			var ok bool
			if buf, ok = appendString(buf, k); !ok {
				return buf, false
			}
			buf = append(buf, ':')
			if buf, ok = appendValue(buf, e, depth+1); !ok {
				return buf, false
			}
		}
		return append(buf, '}'), true
	case []interface{}:
		if depth+1 > maxNesting {
			return buf, false
		}
		buf = append(buf, '[')
		for i, e := range x {
			if i > 0 {
				buf = append(buf, ',')
			}
			var ok bool
			if buf, ok = appendValue(buf, e, depth+1); !ok {
				return buf, false
			}
		}
		return append(buf, ']'), true
	}
	return buf, false
}

const hexDigits = "0123456789abcdef"

func appendString(buf []byte, s string) ([]byte, bool) {
	if !utf8.ValidString(s) {
		return buf, false
	}
	buf = append(buf, '"')
	start := 0
	for i := 0; i < len(s); i++ {
		c := s[i]
		if c >= 0x20 && c != '"' && c != '\\' {
			continue
		}
		buf = append(buf, s[start:i]...)
		switch c {
		case '"', '\\':
			buf = append(buf, '\\', c)
		case '\n':
			buf = append(buf, '\\', 'n')
		case '\r':
			buf = append(buf, '\\', 'r')
		case '\t':
			buf = append(buf, '\\', 't')
		default:
			buf = append(buf, '\\', 'u', '0', '0', hexDigits[c>>4], hexDigits[c&15])
		}
		start = i + 1
	}
	buf = append(buf, s[start:]...)
	return append(buf, '"'), true
}

func cbytes(b []byte) (*C.uint8_t, C.size_t) {
	if len(b) == 0 {
		return nil, 0
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0])), C.size_t(len(b))
}

// cmem copies b into C memory: pointers stored inside C-allocated arrays
// (gpudiff_json_pair, gpudiff_event) must not be Go pointers (cgo rules).
func cmem(b []byte) (*C.uint8_t, C.size_t) {
	if len(b) == 0 {
		return nil, 0
	}
	return (*C.uint8_t)(C.CBytes(b)), C.size_t(len(b))
}

// DeepEqualApartFromStatus is the drop-in for specsyncer.go:17-41.
func (e *Engine) DeepEqualApartFromStatus(oldObj, newObj interface{}) bool {
	a, ok1 := jsonOf(oldObj)
	b, ok2 := jsonOf(newObj)
	if !ok1 || !ok2 {
		return false // failed type assertion: "differs" (specsyncer.go:20-22)
	}
	e.mu.Lock()
	defer e.mu.Unlock()
	pa, la := cbytes(a)
	pb, lb := cbytes(b)
	var eq C.int
	if rc := C.gpudiff_spec_equal(e.ctx, pa, la, pb, lb, &eq); rc != C.GPUDIFF_OK {
		return false
	}
	return eq != 0
}

// DeepEqualStatus is the drop-in for statussyncer.go:15-27.
func (e *Engine) DeepEqualStatus(oldObj, newObj interface{}) bool {
	a, ok1 := jsonOf(oldObj)
	b, ok2 := jsonOf(newObj)
	if !ok1 || !ok2 {
		return false
	}
	e.mu.Lock()
	defer e.mu.Unlock()
	pa, la := cbytes(a)
	pb, lb := cbytes(b)
	var eq C.int
	if rc := C.gpudiff_status_equal(e.ctx, pa, la, pb, lb, &eq); rc != C.GPUDIFF_OK {
		return false
	}
	return eq != 0
}

// Which predicate an Update event is gated by.
type Which uint8

const (
	Spec   Which = C.GPUDIFF_SPEC_DIRTY
	Status Which = C.GPUDIFF_STATUS_DIRTY
)

type event struct {
	old, new interface{}
	which    Which
	enqueue  func(obj interface{})
	slot     int64 // >= 0: decided against the Store's resident version of this slot
}

// Batcher collects UpdateFunc events from all informers (MPSC) and decides
// them in one gpudiff_submit per window; dirty events call their enqueue
// (Controller.AddToQueue, syncer.go:222-224) in arrival order.
type Batcher struct {
	e        *Engine
	store    *Store
	ch       chan event
	maxBatch int
	window   time.Duration
	avgBytes float64 // JSON bytes per event, running average: the next flush's jsonBuf size
	// pipelined (NewBatcherPipelined): batch k + 1 is submitted before batch k is waited, so the engine
	// overlaps their host staging, upload, K0 and diff pass; an event's enqueue can then come up to two
	// windows after its arrival.  The engine keeps two pair batches in flight and a third submit drops the
	// oldest, so a pipelined batcher must be the engine's only gpudiff_submit user (no one-pair helpers on it).
	pipelined bool
	bufs      []*jsonBuf // idle flush buffers (getJSONBuf)
}

func (b *Batcher) bytesHint(n int) int { return int(b.avgBytes*float64(n)*1.25) + 4096 }

// getJSONBuf / putJSONBuf keep up to three flush buffers (pinned ones are costly to allocate; a pipelined
// batcher has two batches' buffers alive at once)
func (b *Batcher) getJSONBuf(hint int) *jsonBuf { return b.getJSONBufPinned(hint, b.e.devEnc) }

// getJSONBufPinned: an idle pooled buffer (the pool holds pinned ones only) or a new one
func (b *Batcher) getJSONBufPinned(hint int, pinned bool) *jsonBuf {
	for k, jb := range b.bufs {
		if pinned && jb.n >= hint {
			b.bufs = append(b.bufs[:k], b.bufs[k+1:]...)
			jb.buf = jb.buf[:0]
			return jb
		}
	}
	return newJSONBufPinned(b.e, hint, pinned)
}

func (b *Batcher) putJSONBuf(jb *jsonBuf) {
	if jb.e == nil || len(b.bufs) >= 3 {
		jb.free()
		return
	}
	b.bufs = append(b.bufs, jb)
}

func (b *Batcher) noteBytes(total, n int) {
	if n > 0 {
		b.avgBytes = 0.75*b.avgBytes + 0.25*float64(total)/float64(n)
	}
}

func NewBatcher(e *Engine, maxBatch int, window time.Duration) *Batcher {
	b := &Batcher{e: e, ch: make(chan event, 4*maxBatch), maxBatch: maxBatch, window: window}
	go b.loop()
	return b
}

// NewBatcherPipelined is NewBatcher with two batches in flight (see Batcher.pipelined): at 131k config3
// pairs a batch the engine then streams at the PCIe link's rate (DESIGN.md §6, 7.45M pairs/s vs 6.2-6.6M
// waiting each batch before the next).  tests/goshim.py Batcher(engine=...) restates it.
func NewBatcherPipelined(e *Engine, maxBatch int, window time.Duration) *Batcher {
	b := &Batcher{e: e, ch: make(chan event, 4*maxBatch), maxBatch: maxBatch, window: window, pipelined: true}
	go b.loop()
	return b
}

// Update replaces `if !deepEqual...(old, new) { c.AddToQueue(gvr, new) }`.
func (b *Batcher) Update(oldObj, newObj interface{}, which Which, enqueue func(obj interface{})) {
	b.ch <- event{oldObj, newObj, which, enqueue, -1}
}

// UpdateStored is Update against the batcher's Store: only the new object is
// uploaded; oldObj is read only if the slot is empty or a path-hash collision
// needs a re-seed.  All events of one Batcher go either here or to Update.
func (b *Batcher) UpdateStored(slot uint32, oldObj, newObj interface{}, which Which, enqueue func(obj interface{})) {
	b.ch <- event{oldObj, newObj, which, enqueue, int64(slot)}
}

// loop flushes when maxBatch events are pending or the window has passed since the last flush,
// whichever comes first; events are decided and enqueued in arrival order.  Before the timer is
// re-armed it is stopped and, if it had fired while a full batch was being flushed, its tick is
// drained: Reset does not empty the channel, and a stale tick would flush the next batch at once,
// shrinking batches exactly when the load is high (tests/goshim.py Batcher restates this loop).
func (b *Batcher) loop() {
	var pending []event
	var inflight *flight // pipelined: the batch submitted last, not yet waited
	timer := time.NewTimer(b.window)
	for {
		select {
		case ev := <-b.ch:
			pending = append(pending, ev)
			if len(pending) < b.maxBatch {
				continue
			}
		case <-timer.C:
		}
		if len(pending) > 0 && b.pipelined {
			f := b.submitFlight(pending) // the engine works on it while the previous batch is settled
			if inflight != nil {
				b.finishFlight(inflight)
			}
			inflight = f
			pending = make([]event, 0, b.maxBatch) // f keeps the old slice
		} else if len(pending) > 0 {
			b.flush(pending)
			pending = pending[:0]
		} else if inflight != nil { // a window with no new events: settle the batch in flight
			b.finishFlight(inflight)
			inflight = nil
		}
		if !timer.Stop() {
			select {
			case <-timer.C: // fired during the flush (or just received above: then empty)
			default:
			}
		}
		timer.Reset(b.window)
	}
}

// jsonBuf holds one flush's objects as JSON in ONE C allocation: appendValue appends straight into
// a slice whose backing array is the C memory, so each object is written once, where the engine
// reads it (no jsonOf-then-C.CBytes copy and no allocation per object).  An object that would run
// past the allocation makes append move the slice to the Go heap; add then grows the C buffer
// (C.realloc) and copies that object's bytes over -- rare once capHint tracks the flush size.
// Offsets are handed out, not pointers: the buffer may move until the last object is added.
type jsonBuf struct {
	p   unsafe.Pointer
	n   int // capacity of the allocation
	buf []byte
	e   *Engine // non-nil: p is engine-pinned memory (gpudiff_host_alloc) in the zero-copy layout:
	// every object 16-B aligned and followed by its staged span (len + 32 rounded up to 16, zeroed), so
	// gpudiff_submit uploads the flush straight from it (gpudiff.h)
}

// cslice views n bytes of C memory as a Go slice (Go 1.16, the reference's toolchain: no unsafe.Slice)
func cslice(p unsafe.Pointer, n int) []byte { return (*[1 << 40]byte)(p)[:n:n] }

func newJSONBuf(e *Engine, capHint int) *jsonBuf {
	return newJSONBufPinned(e, capHint, e != nil && e.devEnc)
}

// newJSONBufPinned: pinned (engine memory, zero-copy layout) when asked and the engine can give it
func newJSONBufPinned(e *Engine, capHint int, pinned bool) *jsonBuf {
	if capHint < 4096 {
		capHint = 4096
	}
	if e != nil && pinned {
		var p unsafe.Pointer
		e.mu.Lock()
		rc := C.gpudiff_host_alloc(e.ctx, C.size_t(capHint), &p)
		e.mu.Unlock()
		if rc == C.GPUDIFF_OK {
			return &jsonBuf{p: p, n: capHint, buf: cslice(p, capHint)[:0], e: e}
		}
	}
	p := C.malloc(C.size_t(capHint))
	return &jsonBuf{p: p, n: capHint, buf: cslice(p, capHint)[:0]}
}

func (j *jsonBuf) grow(out []byte, start int) {
	nn := 2 * cap(out)
	if j.e == nil {
		np := C.realloc(j.p, C.size_t(nn)) // keeps [0, start): the objects already in C memory
		dst := cslice(np, nn)
		copy(dst[start:len(out)], out[start:])
		j.p, j.n, j.buf = np, nn, dst[:len(out)]
		return
	}
	var np unsafe.Pointer
	j.e.mu.Lock()
	rc := C.gpudiff_host_alloc(j.e.ctx, C.size_t(nn), &np)
	j.e.mu.Unlock()
	if rc != C.GPUDIFF_OK { // pinned memory exhausted: continue in malloc'd memory (the staged upload)
		np = C.malloc(C.size_t(nn))
	}
	dst := cslice(np, nn)
	copy(dst[:start], cslice(j.p, j.n)[:start])
	copy(dst[start:len(out)], out[start:])
	j.free()
	if rc != C.GPUDIFF_OK {
		j.e = nil
	}
	j.p, j.n, j.buf = np, nn, dst[:len(out)]
}

// span closes the object at [start, len(buf)) in the zero-copy layout: zeros up to its staged span
func (j *jsonBuf) span(start int) {
	if j.e == nil {
		return
	}
	n := len(j.buf) - start
	pad := ((n+32+15)&^15) - n
	out := j.buf
	for k := 0; k < pad; k++ {
		out = append(out, 0)
	}
	j.commit(out, len(j.buf))
}

// tail: the 32 bytes the upload reads past the last object's span
func (j *jsonBuf) tail() {
	if j.e != nil {
		out := append(j.buf, make([]byte, 32)...)
		j.commit(out, len(j.buf))
	}
}

// add renders obj (jsonOf's rules) at the end of the buffer: its offset and length, ok = false
// for a non-transferable object (nothing added).
func (j *jsonBuf) add(obj interface{}) (off, n int, ok bool) {
	u, isU := obj.(*unstructured.Unstructured)
	if !isU || u == nil {
		return 0, 0, false
	}
	var m interface{} = u.Object
	if u.Object == nil {
		m = map[string]interface{}{}
	}
	start := len(j.buf)
	out, ok := appendValue(j.buf, m, 0)
	if !ok { // j.buf is unchanged: the partial object (in C memory or a Go copy) is dropped
		return 0, 0, false
	}
	j.commit(out, start)
	n := len(j.buf) - start
	j.span(start)
	return start, n, true
}

// raw appends literal bytes (the "{}" stand-in of a non-transferable object)
func (j *jsonBuf) raw(b []byte) (off, n int) {
	start := len(j.buf)
	j.commit(append(j.buf, b...), start)
	j.span(start)
	return start, len(b)
}

func (j *jsonBuf) commit(out []byte, start int) bool {
	if cap(out) > 0 && unsafe.Pointer(&out[:1][0]) != j.p {
		j.grow(out, start)
	} else {
		j.buf = out
	}
	return true
}

// at is the C pointer of the object at offset off (valid until the buffer is freed)
func (j *jsonBuf) at(off, n int) (*C.uint8_t, C.size_t) {
	if n == 0 {
		return nil, 0
	}
	return (*C.uint8_t)(unsafe.Pointer(uintptr(j.p) + uintptr(off))), C.size_t(n)
}

func (j *jsonBuf) free() {
	if j.e != nil {
		j.e.mu.Lock()
		C.gpudiff_host_free(j.e.ctx, j.p)
		j.e.mu.Unlock()
	} else {
		C.free(j.p)
	}
}

// flight is one submitted batch: its events, which pair each event became (-1: enqueued without asking
// the engine, e.g. a non-transferable object), the C memory the engine reads until gpudiff_wait, the ticket.
type flight struct {
	evs    []event
	pairOf []int
	ok     []bool // per pair: transferable (false: reported dirty whatever the engine says)
	n      int
	rc     C.int
	ticket C.gpudiff_ticket
	jb     *jsonBuf
	jold   *jsonBuf // store path: old objects the store reads only on a collision (outside the upload)
	cmem   unsafe.Pointer
}

func (b *Batcher) flush(evs []event) { b.finishFlight(b.submitFlight(evs)) }

// submitFlight stages a batch and submits it (gpudiff_submit or gpudiff_store_submit) without waiting.
func (b *Batcher) submitFlight(evs []event) *flight {
	if b.store != nil {
		return b.submitStored(evs)
	}
	n := len(evs)
	f := &flight{evs: evs, pairOf: make([]int, n), ok: make([]bool, n), n: n}
	pairs := (*[1 << 28]C.gpudiff_json_pair)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.gpudiff_json_pair{}))))[:n:n]
	f.cmem = unsafe.Pointer(&pairs[0])
	f.jb = b.getJSONBuf(b.bytesHint(n))
	jb := f.jb
	offs := make([]int, 4*n) // old off, len, new off, len: pointers only once the buffer stops moving
	for i, ev := range evs {
		f.pairOf[i] = i
		mark := len(jb.buf)
		oa, la, ok1 := jb.add(ev.old)
		var oc, lc int
		ok2 := false
		if ok1 {
			oc, lc, ok2 = jb.add(ev.new)
		}
		f.ok[i] = ok1 && ok2
		if !f.ok[i] {
			jb.buf = jb.buf[:mark]
			oa, la = jb.raw([]byte("{}"))
			oc, lc = jb.raw([]byte("{}")) // its own copy: the zero-copy layout wants pair order
		}
		offs[4*i], offs[4*i+1], offs[4*i+2], offs[4*i+3] = oa, la, oc, lc
	}
	b.noteBytes(len(jb.buf), n)
	jb.tail()
	for i := range evs {
		pa, la := jb.at(offs[4*i], offs[4*i+1])
		pc, lc := jb.at(offs[4*i+2], offs[4*i+3])
		pairs[i] = C.gpudiff_json_pair{old_json: pa, old_len: la, new_json: pc, new_len: lc,
			pair_id: C.uint32_t(i)}
	}
	b.e.mu.Lock()
	f.rc = C.gpudiff_submit(b.e.ctx, &pairs[0], C.size_t(n), &f.ticket)
	b.e.mu.Unlock()
	return f
}

// finishFlight waits for a submitted batch and calls its events' enqueue in arrival order: the dirty ones
// for their own predicate, the non-transferable ones, and every one if the engine failed (conservative,
// like the reference's failed type assertion -> enqueue, specsyncer.go:20-22).
func (b *Batcher) finishFlight(f *flight) {
	flags := make([]uint8, f.n)
	rc := f.rc
	if f.n > 0 {
		b.e.mu.Lock()
		var res C.gpudiff_result
		if rc == C.GPUDIFF_OK {
			rc = C.gpudiff_wait(b.e.ctx, f.ticket, &res)
		}
		if rc == C.GPUDIFF_OK {
			copy(flags, (*[1 << 30]uint8)(unsafe.Pointer(res.pair_flags))[:f.n:f.n])
			C.gpudiff_result_release(b.e.ctx, &res)
		}
		b.e.mu.Unlock()
	}
	for i, ev := range f.evs {
		k := f.pairOf[i]
		if k < 0 || rc != C.GPUDIFF_OK || !f.ok[k] || flags[k]&uint8(ev.which) != 0 {
			ev.enqueue(ev.new)
		}
	}
	if f.jb != nil {
		b.putJSONBuf(f.jb)
	}
	if f.jold != nil {
		f.jold.free()
	}
	if f.cmem != nil {
		C.free(f.cmem)
	}
}

// Store is the device-resident informer snapshot (gpudiff_store_*): the old
// versions stay in HBM, one per slot ((cluster, gvr, namespace, name) -> slot,
// the indexer's key, pkg/syncer/syncer.go:318).
type Store struct {
	e      *Engine
	s      *C.gpudiff_store
	devEnc bool
	// the store's first-sighting rule mirrored (gpudiff.h gpudiff_host_alloc): a slot's first event has its old
	// object encoded, so on a device-encode store that object goes into the upload buffer ahead of the new one; a
	// slot the engine emptied on its own (a conservative deferral) is not mirrored -- such a batch just takes the
	// staging copy, with the same results
	seen map[uint32]bool
}

func (e *Engine) NewStore(maxSlots uint32, spaceBytes uint64, maxEvents uint32) (*Store, error) {
	return e.NewStoreEx(maxSlots, spaceBytes, maxEvents, false)
}

// NewStoreEx with deviceEncode uploads raw JSON and encodes it on the GPU (kernel K0); the
// batcher already keeps each batch's buffers until gpudiff_wait returns and waits in order,
// which is what that mode requires.
func (e *Engine) NewStoreEx(maxSlots uint32, spaceBytes uint64, maxEvents uint32, deviceEncode bool) (*Store, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	var flags C.uint32_t
	if deviceEncode {
		flags = C.GPUDIFF_STORE_DEVICE_ENCODE
	}
	var s *C.gpudiff_store
	if err := errOf(C.gpudiff_store_create_ex(e.ctx, C.uint32_t(maxSlots), C.uint64_t(spaceBytes),
		C.uint32_t(maxEvents), flags, &s)); err != nil {
		return nil, err
	}
	return &Store{e: e, s: s, devEnc: deviceEncode, seen: make(map[uint32]bool)}, nil
}

// Forget is the DeleteFunc side: the slot is empty again.
func (s *Store) Forget(slot uint32) error {
	s.e.mu.Lock()
	defer s.e.mu.Unlock()
	delete(s.seen, slot)
	return errOf(C.gpudiff_store_forget(s.e.ctx, s.s, C.uint32_t(slot)))
}

// WithStore routes the batcher's UpdateStored events through st.
func (b *Batcher) WithStore(st *Store) *Batcher {
	b.store = st
	return b
}

func (b *Batcher) submitStored(evs []event) *flight {
	// events whose objects are not Unstructured never reach the store (its slot
	// state must only see real versions); they are enqueued, as the reference's
	// failed type assertion would (specsyncer.go:20-22) -- in arrival order, when the batch finishes
	f := &flight{evs: evs, pairOf: make([]int, len(evs))}
	good := make([]int, 0, len(evs))
	for i, ev := range evs {
		if _, ok := ev.new.(*unstructured.Unstructured); ok && ev.slot >= 0 {
			f.pairOf[i] = len(good)
			good = append(good, i)
		} else {
			f.pairOf[i] = -1
		}
	}
	n := len(good)
	f.n, f.ok = n, make([]bool, n)
	if n == 0 {
		return f
	}
	ce := (*[1 << 27]C.gpudiff_event)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.gpudiff_event{}))))[:n:n]
	f.cmem = unsafe.Pointer(&ce[0])
	// A device-encode store uploads what it encodes straight from engine-pinned memory when the batch is laid
	// out as gpudiff.h gpudiff_host_alloc says (VERDICT r5 #2): per event, in order, its old object when the slot
	// is new to the store, then its new object.  The other old objects -- read only on a path-table collision --
	// go into a plain buffer of their own.  A host-encode store stages (it uploads encoded blobs).
	st := b.store
	f.jb = b.getJSONBufPinned(b.bytesHint(n), st.devEnc)
	f.jold = newJSONBuf(nil, b.bytesHint(n))
	jb, jold := f.jb, f.jold
	offs := make([]int, 4*n) // new off, len, old off, len (len 0: absent)
	oldIn := make([]bool, n) // the old object sits in jb (else jold)
	for k, i := range good {
		ev := evs[i]
		slot := uint32(ev.slot)
		if !st.seen[slot] {
			if o, l, oko := jb.add(ev.old); oko {
				offs[4*k+2], offs[4*k+3], oldIn[k] = o, l, true
			}
		} else if o, l, oko := jold.add(ev.old); oko {
			offs[4*k+2], offs[4*k+3] = o, l
		}
		st.seen[slot] = true
		if o, l, okn := jb.add(ev.new); okn {
			offs[4*k], offs[4*k+1] = o, l
			f.ok[k] = true
		} else {
			offs[4*k], offs[4*k+1] = jb.raw([]byte("{")) // undecodable: reported dirty, slot emptied
		}
	}
	jb.tail()
	b.noteBytes(len(jb.buf), n)
	for k, i := range good {
		ce[k] = C.gpudiff_event{slot: C.uint32_t(evs[i].slot), pair_id: C.uint32_t(k)}
		ce[k].new_json, ce[k].new_len = jb.at(offs[4*k], offs[4*k+1])
		if oldIn[k] {
			ce[k].old_json, ce[k].old_len = jb.at(offs[4*k+2], offs[4*k+3])
		} else {
			ce[k].old_json, ce[k].old_len = jold.at(offs[4*k+2], offs[4*k+3])
		}
	}
	b.e.mu.Lock()
	f.rc = C.gpudiff_store_submit(b.e.ctx, b.store.s, &ce[0], C.size_t(n), &f.ticket)
	b.e.mu.Unlock()
	return f
}

var errNoEngine = errors.New("gpudiff: engine not initialised")

// Mode selects which of the syncer's two write-path transforms UpsertBodies applies.
type Mode uint32

const (
	// UpsertSpec is upsertIntoDownstream's object (specsyncer.go:94-108).
	UpsertSpec Mode = C.GPUDIFF_UPSERT_SPEC
	// UpsertStatus is updateStatusInUpstream's object (statussyncer.go:44-48).
	UpsertStatus Mode = C.GPUDIFF_UPSERT_STATUS
)

// UpsertBodies returns, for each dirty object, the request body the dynamic
// client would send after the syncer's DeepCopy + SetUID("") +
// SetResourceVersion("") (+ owner-reference filter in UpsertSpec mode): the
// bytes of json.NewEncoder(w).Encode(obj.Object), built by kernel K10 (the
// host path completes what K10 leaves).  bodies[i] is nil when objs[i] is not
// an *unstructured.Unstructured or does not decode; the caller then takes the
// reference path for that object.  The caller splices the live
// resourceVersion in before client.Update (specsyncer.go:122,
// statussyncer.go:56) exactly as today.
func (e *Engine) UpsertBodies(objs []interface{}, mode Mode) ([][]byte, error) {
	n := len(objs)
	if n == 0 {
		return nil, nil
	}
	docs := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	lens := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.size_t(0))))
	defer C.free(docs)
	defer C.free(lens)
	dp := (*[1 << 30]*C.uint8_t)(docs)[:n:n]
	lp := (*[1 << 30]C.size_t)(lens)[:n:n]
	for i, o := range objs {
		dp[i], lp[i] = nil, 0
		if b, ok := jsonOf(o); ok {
			dp[i], lp[i] = cmem(b)
		}
	}
	defer func() {
		for i := range dp {
			C.free(unsafe.Pointer(dp[i]))
		}
	}()
	e.mu.Lock()
	defer e.mu.Unlock()
	var out C.gpudiff_bodies
	if err := errOf(C.gpudiff_upsert_bodies(e.ctx, (**C.uint8_t)(docs), (*C.size_t)(lens), C.size_t(n),
		C.uint32_t(mode), &out)); err != nil {
		return nil, err
	}
	defer C.gpudiff_bodies_release(e.ctx, &out)
	offs := (*[1 << 30]C.uint64_t)(unsafe.Pointer(out.offsets))[: n+1 : n+1]
	st := (*[1 << 30]C.int32_t)(unsafe.Pointer(out.status))[:n:n]
	res := make([][]byte, n)
	for i := 0; i < n; i++ {
		if lp[i] == 0 || st[i] != 0 {
			continue
		}
		res[i] = C.GoBytes(unsafe.Pointer(uintptr(unsafe.Pointer(out.bytes))+uintptr(offs[i])),
			C.int(offs[i+1]-offs[i]))
	}
	return res, nil
}

// OptDeviceEncode opens an engine whose submits send raw JSON to the GPU (kernel K0); DiffAndPlan needs it.
const OptDeviceEncode = uint32(C.GPUDIFF_OPT_DEVICE_ENCODE)

// Write is one API call the syncer's decisions imply (gpudiff_write_plan_get_ex).  For informer
// pairs (PlanInformer) both kinds render the NEW object -- UpdateFunc enqueues newObj
// (specsyncer.go:47-50, statussyncer.go:32-35) and the worker writes it: a spec write is
// upsertIntoDownstream's body (specsyncer.go:86-132), a status write updateStatusInUpstream's
// (statussyncer.go:41-63).  For (upstream A, downstream B) pairs (PlanUpstreamDownstream) the spec
// write renders A and the status write B.
type Write struct {
	Pair int    // index into the olds / news given to DiffAndPlan
	Kind Mode   // UpsertSpec or UpsertStatus
	Noop bool   // the body equals the other document's on the wire in that region (GPUDIFF_SPEC_NOOP / _STATUS_NOOP)
	Body []byte // the request body; nil for a no-op, or when Go cannot decode the object (reference path)
}

// Plan modes (GPUDIFF_PLAN_*): which writes DiffAndPlanMode lists and which document they render.
const (
	PlanInformer           = uint32(C.GPUDIFF_PLAN_INFORMER)            // pairs are (old, new) events; both kinds
	PlanSpec               = uint32(C.GPUDIFF_PLAN_SPEC)                // only spec writes (an upstream informer's batch)
	PlanStatus             = uint32(C.GPUDIFF_PLAN_STATUS)              // only status writes (a downstream informer's batch)
	PlanUpstreamDownstream = uint32(C.GPUDIFF_PLAN_UPSTREAM_DOWNSTREAM) // pairs are (A upstream, B downstream)
)

// DiffAndPlan is DiffAndPlanMode(olds, news, PlanInformer).
func (e *Engine) DiffAndPlan(olds, news [][]byte) ([]uint8, []Write, error) {
	return e.DiffAndPlanMode(olds, news, PlanInformer)
}

// DiffAndPlanMode decides n pairs on the device and renders the writes those decisions imply from
// the JSON still staged in HBM (kernel K10, no second upload): flags[i] are the pair's GPUDIFF_*
// result bits, writes list the spec writes (ascending pair) then the status writes.  The engine must
// have been opened with OptDeviceEncode.  The caller issues each non-no-op write as today (Create,
// then Update with the live resourceVersion on AlreadyExists, specsyncer.go:110-129).
func (e *Engine) DiffAndPlanMode(olds, news [][]byte, mode uint32) ([]uint8, []Write, error) {
	n := len(olds)
	if len(news) != n {
		return nil, nil, errOf(C.GPUDIFF_E_INVAL)
	}
	if n == 0 {
		return nil, nil, nil
	}
	pairs := (*[1 << 28]C.gpudiff_json_pair)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.gpudiff_json_pair{}))))[:n:n]
	defer C.free(unsafe.Pointer(&pairs[0]))
	for i := range olds {
		pa, la := cmem(olds[i])
		pb, lb := cmem(news[i])
		pairs[i] = C.gpudiff_json_pair{old_json: pa, old_len: la, new_json: pb, new_len: lb, pair_id: C.uint32_t(i)}
	}
	defer func() {
		for i := range pairs {
			C.free(unsafe.Pointer(pairs[i].old_json))
			C.free(unsafe.Pointer(pairs[i].new_json))
		}
	}()
	e.mu.Lock()
	defer e.mu.Unlock()
	var ticket C.gpudiff_ticket
	if err := errOf(C.gpudiff_submit(e.ctx, &pairs[0], C.size_t(n), &ticket)); err != nil {
		return nil, nil, err
	}
	var res C.gpudiff_result
	if err := errOf(C.gpudiff_wait(e.ctx, ticket, &res)); err != nil {
		return nil, nil, err
	}
	flags := make([]uint8, n)
	copy(flags, (*[1 << 30]uint8)(unsafe.Pointer(res.pair_flags))[:n:n])
	C.gpudiff_result_release(e.ctx, &res)
	var plan C.gpudiff_write_plan
	if err := errOf(C.gpudiff_write_plan_get_ex(e.ctx, ticket, C.uint32_t(mode), &plan)); err != nil {
		return flags, nil, err
	}
	defer C.gpudiff_write_plan_release(e.ctx, &plan)
	m := int(plan.n)
	writes := make([]Write, m)
	if m == 0 {
		return flags, writes, nil
	}
	idx := (*[1 << 30]C.uint32_t)(unsafe.Pointer(plan.pair_index))[:m:m]
	kind := (*[1 << 30]C.uint8_t)(unsafe.Pointer(plan.kind))[:m:m]
	noop := (*[1 << 30]C.uint8_t)(unsafe.Pointer(plan.noop))[:m:m]
	offs := (*[1 << 30]C.uint64_t)(unsafe.Pointer(plan.bodies.offsets))[: m+1 : m+1]
	st := (*[1 << 30]C.int32_t)(unsafe.Pointer(plan.bodies.status))[:m:m]
	for k := 0; k < m; k++ {
		w := Write{Pair: int(idx[k]), Kind: Mode(kind[k]), Noop: noop[k] != 0}
		if !w.Noop && st[k] == 0 {
			w.Body = C.GoBytes(unsafe.Pointer(uintptr(unsafe.Pointer(plan.bodies.bytes))+uintptr(offs[k])),
				C.int(offs[k+1]-offs[k]))
		}
		writes[k] = w
	}
	return flags, writes, nil
}

// RollupGroup is the status roll-up of one root Deployment
// (pkg/reconciler/deployment/deployment.go:71-91): the int32 sums of its
// leaves' status counters and the index of others[0] (whose
// status.conditions the root copies).
type RollupGroup struct {
	FirstDoc            int
	Members             int
	Replicas            int32
	UpdatedReplicas     int32
	ReadyReplicas       int32
	AvailableReplicas   int32
	UnavailableReplicas int32
}

// Rollup groups are keyed by doc index: DocGroup[i] is the group of docs[i],
// or RollupNone (no kcp.dev/owned-by label) / RollupDecode (Go cannot decode
// the document into an appsv1.Deployment).
const (
	RollupNone   = int(C.GPUDIFF_ROLLUP_NONE)
	RollupDecode = int(C.GPUDIFF_ROLLUP_DECODE)
)

// RollupStatus aggregates every root's status at once from the JSON of the
// cached Deployments (kernels K11 + K12; the host path decides what K11
// leaves): the answer of the splitter's reconcile loop for each root, with
// others[0] fixed to the lowest document index.  Groups are in order of first
// appearance.
func (e *Engine) RollupStatus(docs [][]byte) ([]RollupGroup, []int, error) {
	n := len(docs)
	if n == 0 {
		return nil, nil, nil
	}
	dptr := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	lens := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.size_t(0))))
	defer C.free(dptr)
	defer C.free(lens)
	dp := (*[1 << 30]*C.uint8_t)(dptr)[:n:n]
	lp := (*[1 << 30]C.size_t)(lens)[:n:n]
	for i, b := range docs {
		dp[i], lp[i] = cmem(b)
	}
	defer func() {
		for i := range dp {
			C.free(unsafe.Pointer(dp[i]))
		}
	}()
	e.mu.Lock()
	defer e.mu.Unlock()
	var out C.gpudiff_rollup
	if err := errOf(C.gpudiff_rollup_status(e.ctx, (**C.uint8_t)(dptr), (*C.size_t)(lens), C.size_t(n),
		&out)); err != nil {
		return nil, nil, err
	}
	defer C.gpudiff_rollup_release(e.ctx, &out)
	dg := (*[1 << 30]C.int32_t)(unsafe.Pointer(out.doc_group))[:n:n]
	docGroup := make([]int, n)
	for i := range dg {
		docGroup[i] = int(dg[i])
	}
	ng := int(out.n_groups)
	groups := make([]RollupGroup, ng)
	if ng > 0 {
		gs := (*[1 << 28]C.gpudiff_rollup_group)(unsafe.Pointer(out.groups))[:ng:ng]
		for i, g := range gs {
			groups[i] = RollupGroup{FirstDoc: int(g.first_doc), Members: int(g.n_members),
				Replicas: int32(g.sums[0]), UpdatedReplicas: int32(g.sums[1]), ReadyReplicas: int32(g.sums[2]),
				AvailableReplicas: int32(g.sums[3]), UnavailableReplicas: int32(g.sums[4])}
		}
	}
	return groups, docGroup, nil
}

// Update classification actions (GPUDIFF_NEG_*), the queue actions of
// pkg/reconciler/apiresource/controller.go:159-166.
const (
	NegIgnore  = int32(C.GPUDIFF_NEG_IGNORE)  // dropped (:264, :283)
	NegSpec    = int32(C.GPUDIFF_NEG_SPEC)    // SpecChanged
	NegStatus  = int32(C.GPUDIFF_NEG_STATUS)  // StatusOnlyChanged
	NegMeta    = int32(C.GPUDIFF_NEG_META)    // AnnotationOrLabelsOnlyChanged
	NegCreated = int32(C.GPUDIFF_NEG_CREATED) // Created (no old object)
	NegDecode  = int32(C.GPUDIFF_NEG_DECODE)  // a side not valid JSON / not an object, or a field read that fails Go's typed decode
)

// The typed object of an event (toQueueElementType, controller.go:185-236).
const (
	KindAPIResource = uint8(C.GPUDIFF_NEG_KIND_API) // *APIResourceImport, *NegotiatedAPIResource
	KindCRD         = uint8(C.GPUDIFF_NEG_KIND_CRD) // *apiextensionsv1.CustomResourceDefinition
)

// ClassifyUpdates is the batch form of the "Update" branch of
// Controller.enqueue (controller.go:253-283) for APIResourceImport /
// NegotiatedAPIResource JSON: one action per (olds[i], news[i]); olds[i] == nil
// means no old object.  Kernels K13 + K14, host path for K13's deferrals.
func (e *Engine) ClassifyUpdates(olds, news [][]byte) ([]int32, error) {
	return e.ClassifyUpdatesKinds(nil, olds, news)
}

// ClassifyUpdatesKinds is ClassifyUpdates with each event's kind (KindAPIResource
// or KindCRD; nil: all KindAPIResource), so one batch can carry the events of
// all three informers the controller watches.
func (e *Engine) ClassifyUpdatesKinds(kinds []uint8, olds, news [][]byte) ([]int32, error) {
	n := len(news)
	if n == 0 {
		return nil, nil
	}
	if len(olds) != n || (kinds != nil && len(kinds) != n) {
		return nil, errOf(C.GPUDIFF_E_INVAL)
	}
	var kp *C.uint8_t
	if kinds != nil {
		kp = (*C.uint8_t)(C.CBytes(kinds))
		defer C.free(unsafe.Pointer(kp))
	}
	ptrSz := C.size_t(unsafe.Sizeof(uintptr(0)))
	lenSz := C.size_t(unsafe.Sizeof(C.size_t(0)))
	optr, olen := C.malloc(C.size_t(n)*ptrSz), C.malloc(C.size_t(n)*lenSz)
	nptr, nlen := C.malloc(C.size_t(n)*ptrSz), C.malloc(C.size_t(n)*lenSz)
	defer C.free(optr)
	defer C.free(olen)
	defer C.free(nptr)
	defer C.free(nlen)
	op := (*[1 << 30]*C.uint8_t)(optr)[:n:n]
	ol := (*[1 << 30]C.size_t)(olen)[:n:n]
	np := (*[1 << 30]*C.uint8_t)(nptr)[:n:n]
	nl := (*[1 << 30]C.size_t)(nlen)[:n:n]
	for i := 0; i < n; i++ {
		op[i], ol[i] = nil, 0
		if olds[i] != nil { // present, even when empty: a non-NULL pointer
			op[i], ol[i] = (*C.uint8_t)(C.CBytes(append(olds[i][:len(olds[i]):len(olds[i])], 0))), C.size_t(len(olds[i]))
		}
		np[i], nl[i] = cmem(news[i])
	}
	defer func() {
		for i := 0; i < n; i++ {
			C.free(unsafe.Pointer(op[i]))
			C.free(unsafe.Pointer(np[i]))
		}
	}()
	actions := make([]int32, n)
	e.mu.Lock()
	defer e.mu.Unlock()
	rc := C.gpudiff_classify_updates_kinds(e.ctx, kp, (**C.uint8_t)(optr), (*C.size_t)(olen), (**C.uint8_t)(nptr),
		(*C.size_t)(nlen), C.size_t(n), (*C.int32_t)(unsafe.Pointer(&actions[0])))
	if err := errOf(rc); err != nil {
		return nil, err
	}
	return actions, nil
}

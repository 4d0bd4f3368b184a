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
	"errors"
	"fmt"
	"sync"
	"time"
	"unsafe"

	"k8s.io/apimachinery/pkg/apis/meta/v1/unstructured"
)

// Engine owns one gpudiff context (one GPU, one stream).  A context is not
// reentrant, so every call goes through mu; the Batcher is the intended
// single submitter.
type Engine struct {
	mu  sync.Mutex
	ctx *C.gpudiff_ctx
}

func errOf(rc C.int) error {
	if rc == C.GPUDIFF_OK {
		return nil
	}
	return fmt.Errorf("gpudiff: %s (%d)", C.GoString(C.gpudiff_strerror(rc)), int(rc))
}

// Open creates an engine on HIP device `device` (-1 = current).
func Open(device int) (*Engine, error) {
	var opts C.gpudiff_opts
	opts.device = C.int32_t(device)
	var ctx *C.gpudiff_ctx
	if err := errOf(C.gpudiff_open(&opts, &ctx)); err != nil {
		return nil, err
	}
	return &Engine{ctx: ctx}, nil
}

func (e *Engine) Close() {
	e.mu.Lock()
	defer e.mu.Unlock()
	if e.ctx != nil {
		C.gpudiff_close(e.ctx)
		e.ctx = nil
	}
}

func jsonOf(obj interface{}) ([]byte, bool) {
	u, ok := obj.(*unstructured.Unstructured)
	if !ok || u == nil {
		return nil, false
	}
	b, err := u.MarshalJSON()
	if err != nil {
		return nil, false
	}
	return b, true
}

func cbytes(b []byte) (*C.uint8_t, C.size_t) {
	if len(b) == 0 {
		return nil, 0
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0])), C.size_t(len(b))
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
}

// Batcher collects UpdateFunc events from all informers (MPSC) and decides
// them in one gpudiff_submit per window; dirty events call their enqueue
// (Controller.AddToQueue, syncer.go:222-224) in arrival order.
type Batcher struct {
	e        *Engine
	ch       chan event
	maxBatch int
	window   time.Duration
}

func NewBatcher(e *Engine, maxBatch int, window time.Duration) *Batcher {
	b := &Batcher{e: e, ch: make(chan event, 4*maxBatch), maxBatch: maxBatch, window: window}
	go b.loop()
	return b
}

// Update replaces `if !deepEqual...(old, new) { c.AddToQueue(gvr, new) }`.
func (b *Batcher) Update(oldObj, newObj interface{}, which Which, enqueue func(obj interface{})) {
	b.ch <- event{oldObj, newObj, which, enqueue}
}

func (b *Batcher) loop() {
	var pending []event
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
		if len(pending) > 0 {
			b.flush(pending)
			pending = pending[:0]
		}
		timer.Reset(b.window)
	}
}

func (b *Batcher) flush(evs []event) {
	n := len(evs)
	pairs := (*[1 << 28]C.gpudiff_json_pair)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.gpudiff_json_pair{}))))[:n:n]
	defer C.free(unsafe.Pointer(&pairs[0]))
	keep := make([][]byte, 0, 2*n)
	bad := make([]bool, n)
	for i, ev := range evs {
		a, ok1 := jsonOf(ev.old)
		c, ok2 := jsonOf(ev.new)
		if !ok1 || !ok2 {
			bad[i] = true
			a, c = []byte("{}"), []byte("{}")
		}
		keep = append(keep, a, c)
		pa, la := cbytes(a)
		pc, lc := cbytes(c)
		pairs[i] = C.gpudiff_json_pair{old_json: pa, old_len: la, new_json: pc, new_len: lc,
			pair_id: C.uint32_t(i)}
	}
	b.e.mu.Lock()
	var ticket C.gpudiff_ticket
	rc := C.gpudiff_submit(b.e.ctx, &pairs[0], C.size_t(n), &ticket)
	var res C.gpudiff_result
	if rc == C.GPUDIFF_OK {
		rc = C.gpudiff_wait(b.e.ctx, ticket, &res)
	}
	flags := make([]uint8, n)
	if rc == C.GPUDIFF_OK {
		copy(flags, (*[1 << 30]uint8)(unsafe.Pointer(res.pair_flags))[:n:n])
		C.gpudiff_result_release(b.e.ctx, &res)
	}
	b.e.mu.Unlock()
	for i, ev := range evs {
		// device or encode failure: conservative, like the reference's type
		// assertion failure -> enqueue
		if rc != C.GPUDIFF_OK || bad[i] || flags[i]&uint8(ev.which) != 0 {
			ev.enqueue(ev.new)
		}
	}
	_ = keep
}

var errNoEngine = errors.New("gpudiff: engine not initialised")

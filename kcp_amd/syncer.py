"""Host-side mirror of the reference syncer's handler interface, with the
change-detection predicates answered by the GPU engine.

Reference (sttts/kcp):
  type HandlersProvider func(c *Controller, gvr) cache.ResourceEventHandlerFuncs
                                                   pkg/syncer/syncer.go:68
  NewSpecSyncer handlers   Add/Update/Delete       pkg/syncer/specsyncer.go:43-55
  NewStatusSyncer handlers Update only             pkg/syncer/statussyncer.go:29-39
  Controller.AddToQueue(gvr, obj)                  pkg/syncer/syncer.go:222-224

`deep_equal_apart_from_status` / `deep_equal_status` are the one-pair drop-ins
(same names, argument meaning and error behaviour as the Go predicates: a
pair that cannot be decoded is "not equal").  `UpdateBatcher` is the batched
form the Go shim's batcher goroutine implements: UpdateFunc events are
collected and decided in one gpudiff_submit; dirty ones reach AddToQueue in
arrival order with the same decision the synchronous predicate would give.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional, Tuple

from . import gpudiff as G

_default_engine: Optional[G.Engine] = None


def default_engine() -> G.Engine:
    global _default_engine
    if _default_engine is None:
        _default_engine = G.Engine(device=G.DEVICE_CURRENT)
    return _default_engine


def deep_equal_apart_from_status(old_obj: Any, new_obj: Any, engine: Optional[G.Engine] = None) -> bool:
    """specsyncer.go:17-41 on the GPU."""
    if old_obj is None or new_obj is None:
        return False  # failed type assertion in the reference -> "differs"
    return (engine or default_engine()).spec_equal(old_obj, new_obj)


def deep_equal_status(old_obj: Any, new_obj: Any, engine: Optional[G.Engine] = None) -> bool:
    """statussyncer.go:15-27 on the GPU (asymmetric: new must have status)."""
    if old_obj is None or new_obj is None:
        return False
    return (engine or default_engine()).status_equal(old_obj, new_obj)


@dataclass
class ResourceEventHandlerFuncs:
    """client-go cache.ResourceEventHandlerFuncs [3P]: nil funcs are no-ops."""
    add_func: Optional[Callable[[Any], None]] = None
    update_func: Optional[Callable[[Any, Any], None]] = None
    delete_func: Optional[Callable[[Any], None]] = None

    def on_add(self, obj):
        if self.add_func:
            self.add_func(obj)

    def on_update(self, old, new):
        if self.update_func:
            self.update_func(old, new)

    def on_delete(self, obj):
        if self.delete_func:
            self.delete_func(obj)


@dataclass
class Controller:
    """The consumer side of the gate: AddToQueue (syncer.go:222-224)."""
    queue: List[Tuple[str, Any]] = field(default_factory=list)

    def add_to_queue(self, gvr: str, obj: Any):
        self.queue.append((gvr, obj))


SPEC, STATUS = G.SPEC_DIRTY, G.STATUS_DIRTY


class UpdateBatcher:
    """Collects UpdateFunc events and decides them in one GPU batch.

    `flush()` submits the pending events (also triggered by `max_batch`);
    each event's predicate bit (SPEC or STATUS) decides whether its new object
    goes to its controller's AddToQueue, in arrival order."""

    def __init__(self, engine: Optional[G.Engine] = None, max_batch: int = 4096,
                 decide: Optional[Callable[[List[Tuple[Any, Any]]], List[int]]] = None):
        self.engine = engine
        self.max_batch = max_batch
        self._decide = decide  # test seam: returns per-pair flag bits
        self.pending: List[Tuple[Controller, str, Any, Any, int]] = []

    def update(self, controller: Controller, gvr: str, old, new, bit: int):
        self.pending.append((controller, gvr, old, new, bit))
        if len(self.pending) >= self.max_batch:
            self.flush()

    def _flags(self, pairs) -> List[int]:
        if self._decide is not None:
            return list(self._decide(pairs))
        eng = self.engine or default_engine()
        return eng.diff_pairs(pairs).pair_flags.tolist()

    def flush(self):
        if not self.pending:
            return
        batch, self.pending = self.pending, []
        pairs = [(old, new) for (_, _, old, new, _) in batch]
        flags = self._flags(pairs)
        for (ctl, gvr, _old, new, bit), f in zip(batch, flags):
            if f & bit:  # !deepEqual...(old, new) -> AddToQueue(gvr, new)
                ctl.add_to_queue(gvr, new)


def spec_handlers(c: Controller, gvr: str, batcher: Optional[UpdateBatcher] = None) -> ResourceEventHandlerFuncs:
    """NewSpecSyncer's HandlersProvider (specsyncer.go:44-54)."""
    if batcher is None:
        def update(old, new):
            if not deep_equal_apart_from_status(old, new):
                c.add_to_queue(gvr, new)
    else:
        def update(old, new):
            batcher.update(c, gvr, old, new, SPEC)
    return ResourceEventHandlerFuncs(add_func=lambda obj: c.add_to_queue(gvr, obj), update_func=update,
                                     delete_func=lambda obj: c.add_to_queue(gvr, obj))


def status_handlers(c: Controller, gvr: str, batcher: Optional[UpdateBatcher] = None) -> ResourceEventHandlerFuncs:
    """NewStatusSyncer's HandlersProvider (statussyncer.go:30-38): Update only."""
    if batcher is None:
        def update(old, new):
            if not deep_equal_status(old, new):
                c.add_to_queue(gvr, new)
    else:
        def update(old, new):
            batcher.update(c, gvr, old, new, STATUS)
    return ResourceEventHandlerFuncs(update_func=update)

"""Multi-GPU layer: logical-cluster sharding and the one collective.

The reference runs one independent syncer per logical cluster
(pkg/reconciler/cluster/cluster.go:125-138), each with its own informers and
queue (pkg/syncer/syncer.go:88-132), so pairs shard by logical cluster with no
data-path exchange.  The north star's single collective -- an all-gather of
per-rank dirty counts and dirty pair IDs so every rank holds the node-wide
dirty sets -- is `gather_dirty`, written against torch.distributed so the same
code runs over RCCL/xGMI ("nccl" backend on ROCm) on GPUs and over gloo on CPU
in the tests.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np


def lpt_assign(cluster_weights: Sequence[int], world: int) -> np.ndarray:
    """Greedy LPT bin-packing of clusters onto `world` ranks: heaviest cluster
    first onto the least-loaded rank (ties: lower cluster id, lower rank).
    Returns owner rank per cluster.  Same rule as gpudiff_synth_open."""
    w = np.asarray(cluster_weights, dtype=np.int64)
    order = sorted(range(len(w)), key=lambda c: (-int(w[c]), c))
    load = [0] * world
    owner = np.zeros(len(w), dtype=np.int32)
    for c in order:
        r = min(range(world), key=lambda k: (load[k], k))
        owner[c] = r
        load[r] += int(w[c])
    return owner


def shard_pairs(cluster_of_pair: Sequence[int], world: int) -> List[np.ndarray]:
    """Pair indices per rank (batch order kept within a rank)."""
    cl = np.asarray(cluster_of_pair, dtype=np.int64)
    ids, counts = np.unique(cl, return_counts=True)
    owner_of = dict(zip(ids.tolist(), lpt_assign(counts, world).tolist()))
    owners = np.array([owner_of[c] for c in cl.tolist()], dtype=np.int32)
    return [np.nonzero(owners == r)[0] for r in range(world)]


def gather_dirty(counts, fill, rank: int, world: int, dist, device=None, trim: bool = True):
    """All-gather of the per-rank dirty counts, then of the spec- and
    status-dirty pair IDs (padded to the largest count).

    counts: int32 tensor [8] (n_spec, n_status, ...) on `device`;
    fill(col, buf, n): writes this rank's n IDs of list `col` (0 spec,
    1 status) into the int32 tensor `buf` (the GPU path copies straight from
    HBM with gpudiff_dbatch_export).  Returns (spec_all, status_all): 1-D
    tensors in rank order if `trim`, else the padded [world, max] gathers and
    the host count matrix."""
    import torch

    dev = device if device is not None else counts.device
    allc = torch.empty(world * counts.numel(), dtype=counts.dtype, device=dev)
    dist.all_gather_into_tensor(allc, counts)
    cc = allc.view(world, -1).cpu()
    out = []
    for col in (0, 1):
        mx = max(1, int(cc[:, col].max()))
        buf = torch.zeros(mx, dtype=torch.int32, device=dev)
        fill(col, buf, int(cc[rank, col]))
        allb = torch.empty(world * mx, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(allb, buf)
        allb = allb.view(world, mx)
        out.append(torch.cat([allb[r, :int(cc[r, col])] for r in range(world)]) if trim else allb)
    return (out[0], out[1]) if trim else (out[0], out[1], cc)


def tensor_fill(spec_ids, status_ids):
    """fill() for gather_dirty over ID tensors already in memory."""
    def fill(col, buf, n):
        if n:
            buf[:n] = (spec_ids if col == 0 else status_ids)[:n]
    return fill


class DirtyGather:
    """The per-step collective with ONE all-gather per step: each rank packs
    [counts int32[8] (n_spec, n_status, ...) | spec-dirty IDs (capacity
    cap_spec) | status-dirty IDs (capacity cap_status)] into one preallocated
    int32 buffer and the buffers are all-gathered in a single RCCL call (one
    collective latency instead of three: at N = 8 the step's diff pass is
    ~1 ms, so per-call latency matters).  The capacities start at a value agreed
    before the timed steps (`agree_capacity`: the all-gathered maximum of a
    first pass's counts).

    A changing dirty count (a real watch stream) is handled inside the step
    (`depth` = 1, the default): after the gather, the gathered counts -- 32 B
    per rank, identical on every rank -- are read back (one small D2H copy on
    the stream, waited by an event, not a device synchronisation), and if any
    rank's count exceeded its capacity every rank grows its buffers to the
    gathered maximum (x `grow`) and redoes that step's gather from the same
    results, so the node-wide sets are always exact.  `n_regrows` counts the
    redone steps.

    Pipelining (`depth` > 1): the all-gather is issued asynchronously
    (async_op=True) on the backend's own stream, so step s's collective runs
    while step s+1's diff pass streams on the compute stream.  Step s writes
    send buffer s % depth; before a buffer is refilled the compute stream
    waits (device-side, `work.wait()`) for the collective that last read it.
    There the counts are not read back per step (that would serialise the
    pipeline); instead a running maximum of every step's gathered counts is
    kept on the device and `check()` reports a capacity overflow in ANY step
    -- the IDs of such a step were truncated and `result()` refuses them.
    `finish()` joins the outstanding collectives; it belongs inside the timed
    region."""

    def __init__(self, world: int, cap_spec: int, cap_status: int, device, dist, depth: int = 1,
                 grow: float = 1.25, bind=None, slot=None):
        """bind(send, cap_spec, cap_status): optional -- the engine writes each step's counts and IDs into
        the send buffer itself (gpudiff_dbatch_bind_gather, from its compaction kernel), so a step needs no
        export copies; call begin_step() before the step's diff so the binding points at that step's
        buffer.  fill_counts / fill_ids are then used only to re-export after a capacity regrow.

        slot(k): optional, depth 1 only -- LOOKAHEAD: step s's gathered counts are checked only after step
        s + 1's diff and collective are enqueued (finish() checks the last step), so the host never waits
        between steps and the GPU always has the next pass queued.  The engine alternates result slots by
        step (gpudiff_dbatch_result_slot, set by begin_step), so a capacity regrow found late still exports
        step s's complete lists from its slot, re-gathers it, and re-gathers step s + 1 from the other."""
        import numpy as np
        import torch
        self.world, self.dist, self.device = world, dist, device
        self.depth = max(1, int(depth))
        self.grow = max(1.0, float(grow))
        self.bind = bind
        self.n_steps = 0
        self.n_regrows = 0
        self.maxc = torch.zeros((world, 2), dtype=torch.int32, device=device)
        self.maxc_host = np.zeros((world, 2), dtype=np.int64)  # depth 1: the counts read back every step
        self.slot = slot if self.depth == 1 else None
        self.pending = None  # lookahead: the step whose gathered counts are not checked yet
        self.gathered = []  # tests (trace): (step, capacities, gathered rows) of every lookahead gather
        self.trace = False
        self._alloc(cap_spec, cap_status)

    def _alloc(self, cap_spec: int, cap_status: int):
        import torch
        self.cap = (max(1, int(cap_spec)), max(1, int(cap_status)))
        self.width = 8 + self.cap[0] + self.cap[1]
        self.sends = [torch.zeros(self.width, dtype=torch.int32, device=self.device) for _ in range(self.depth)]
        self.alls = [torch.zeros(self.world * self.width, dtype=torch.int32, device=self.device)
                     for _ in range(self.depth)]
        self.works = [None] * self.depth
        self.used = [False] * self.depth
        pinned = torch.device(self.device).type == "cuda"
        self.host_counts = torch.zeros((self.world, 2), dtype=torch.int32, pin_memory=pinned)
        # lookahead: per step parity, the gathered counts (pinned), their event and the capacities they had
        self.la_counts = [torch.zeros((self.world, 2), dtype=torch.int32, pin_memory=pinned) for _ in range(2)]
        self.la_events = [torch.cuda.Event() if pinned else None for _ in range(2)]
        self.la_caps = [self.cap, self.cap]
        self._select(0)

    def _select(self, b: int):
        self.send, self.all = self.sends[b], self.alls[b]
        self.counts = self.send[:8]
        self.buf = [self.send[8:8 + self.cap[0]], self.send[8 + self.cap[0]:]]
        if self.bind is not None:
            self.bind(self.send, self.cap[0], self.cap[1])

    def begin_step(self):
        """Before the step's diff (with `bind` or `slot`): select this step's send buffer (after the
        collective that last read it) and point the engine's binding at it; with `slot`, the result slot
        this step's diff writes."""
        b = self.n_steps % self.depth
        self._join(b)
        if self.bind is not None:
            self._select(b)
        if self.slot is not None:
            self.slot(self.n_steps % 2)

    def _gather_lookahead(self, k: int, step: int = -1):
        """all-gather of the send buffer, then this step's gathered counts copied to pinned slot k behind an
        event (read later by _check)"""
        self.dist.all_gather_into_tensor(self.all, self.send)
        self.la_counts[k].copy_(self._gathered_counts(0), non_blocking=True)
        self.la_caps[k] = self.cap
        if self.la_events[k] is not None:
            self.la_events[k].record()
        if self.trace:  # synchronises: tests only
            self.gathered.append((step, self.cap, self.all.view(self.world, self.width).cpu().clone()))

    def _check(self, s: int, fill_counts, fill_ids):
        """Lookahead: step s's gathered counts (its collective finished long before: step s + 1's pass was
        queued behind it).  A capacity exceeded on any rank -- the same on every rank, so all redo it
        together -- grows the buffers and re-gathers step s from its result slot, then the in-flight step
        s + 1 (whose send buffer was filled under the old capacities) from the other."""
        k = s % 2
        if self.la_events[k] is not None:
            self.la_events[k].synchronize()
        hc = self.la_counts[k].clone()
        cap = self.la_caps[k]
        self.maxc_host = self.maxc_host.clip(min=hc.numpy())
        if not bool((hc[:, 0] > cap[0]).any() or (hc[:, 1] > cap[1]).any()):
            return
        ms, mt = int(hc[:, 0].max()), int(hc[:, 1].max())
        self._alloc(max(self.cap[0], int(ms * self.grow) + 1), max(self.cap[1], int(mt * self.grow) + 1))
        redo = [s] + ([s + 1] if self.pending == s + 1 else [])
        for t in redo:
            self.slot(t % 2)
            fill_counts(self.counts)
            for col in (0, 1):
                fill_ids(col, self.buf[col])
            self._gather_lookahead(t % 2, t)
        self.n_regrows += 1
        if self.pending == s + 1:  # its re-gather may still exceed the grown capacity: checked as usual
            self.slot((s + 2) % 2)

    @staticmethod
    def agree_capacity(counts, world: int, dist, slack: float = 1.0):
        """All-gathered max of (n_spec, n_status) over ranks (host values; untimed)."""
        import torch
        allc = torch.empty(world * counts.numel(), dtype=counts.dtype, device=counts.device)
        dist.all_gather_into_tensor(allc, counts)
        cc = allc.view(world, -1).cpu()
        return int(cc[:, 0].max() * slack) + 1, int(cc[:, 1].max() * slack) + 1

    def _gathered_counts(self, b: int):
        return self.alls[b].view(self.world, self.width)[:, :2]

    def _read_counts(self):
        """The gathered (n_spec, n_status) of the current buffer on the host: a 8 B x world copy on the
        current stream, waited by an event (the host waits for this step's gather only)."""
        import torch
        self.host_counts.copy_(self._gathered_counts(0), non_blocking=True)
        if self.host_counts.is_pinned():
            ev = torch.cuda.Event()
            ev.record()
            ev.synchronize()
        return self.host_counts

    def step(self, fill_counts, fill_ids):
        """fill_counts(tensor[8]) and fill_ids(col, tensor[cap]) write this
        rank's values into its slots of the send buffer on the device (the GPU
        path: gpudiff_dbatch_export straight from HBM, ordered on the stream
        before the collective).  Both may be called again within one step (a
        capacity regrow re-exports the same results).  With `bind` the engine
        has written them already (begin_step before the diff) and they run only
        after a regrow."""
        import torch
        b = self.n_steps % self.depth
        if self.bind is None:
            self._join(b)  # the collective that last read this buffer
            self._select(b)
            fill_counts(self.counts)
            for col in (0, 1):
                fill_ids(col, self.buf[col])
        if self.slot is not None:  # lookahead (depth 1)
            s = self.n_steps
            self._gather_lookahead(s % 2, s)
            prev, self.pending = self.pending, s
            self.used[0] = True
            self.n_steps += 1
            if prev is not None:
                self._check(prev, fill_counts, fill_ids)
            self._fills = (fill_counts, fill_ids)
            return
        if self.depth > 1:
            self.works[b] = self.dist.all_gather_into_tensor(self.all, self.send, async_op=True)
        else:
            self.dist.all_gather_into_tensor(self.all, self.send)
            hc = self._read_counts()
            if bool((hc[:, 0] > self.cap[0]).any() or (hc[:, 1] > self.cap[1]).any()):
                # every rank sees the same gathered counts, so all take this branch together
                ms, mt = int(hc[:, 0].max()), int(hc[:, 1].max())
                self._alloc(max(self.cap[0], int(ms * self.grow) + 1), max(self.cap[1], int(mt * self.grow) + 1))
                fill_counts(self.counts)
                for col in (0, 1):
                    fill_ids(col, self.buf[col])
                self.dist.all_gather_into_tensor(self.all, self.send)
                self.n_regrows += 1
                hc = self._read_counts()
            # the running maximum on the host: the counts are here already (no device kernel per step)
            np_hc = hc.numpy()
            self.maxc_host = self.maxc_host.clip(min=np_hc)
        self.used[b] = True
        self.n_steps += 1

    def _join(self, b: int):
        """Device-side wait for buffer b's outstanding collective, then fold its gathered counts into the
        running maximum (ordered after the wait on the current stream)."""
        import torch
        if self.works[b] is not None:
            self.works[b].wait()
            self.works[b] = None
            torch.maximum(self.maxc, self._gathered_counts(b), out=self.maxc)

    def finish(self):
        """Join every outstanding collective (the compute stream waits for them); with lookahead, check the
        last step's counts (and regrow it if needed)."""
        for b in range(self.depth):
            self._join(b)
        if self.slot is not None and self.pending is not None:
            s, self.pending = self.pending, None
            self._check(s, *self._fills)

    def _rows(self):
        return self.all.view(self.world, self.width)

    def check(self):
        """-> (ok, host count matrix [world, 8] of the last step); ok only if no
        rank exceeded its capacity in ANY step since the buffers were last sized
        (the device-side running maximum of the gathered counts)."""
        import torch
        self.finish()
        mx = self.maxc.cpu()
        if self.depth == 1:
            mx = torch.maximum(mx, torch.from_numpy(self.maxc_host).to(mx.dtype))
        ok = bool((mx[:, 0] <= self.cap[0]).all() and (mx[:, 1] <= self.cap[1]).all())
        cc = self._rows()[:, :8].cpu()
        return ok, cc

    def result(self):
        """Node-wide (spec IDs, status IDs) of the last step, in rank order
        (host sync; after the timed steps)."""
        import torch
        ok, cc = self.check()
        if not ok:
            raise RuntimeError("dirty-ID capacity exceeded: %s / %s > %s" % (
                self.maxc.cpu().tolist(), self.maxc_host.tolist(), self.cap))
        rows = self._rows()
        spec = torch.cat([rows[r, 8:8 + int(cc[r, 0])] for r in range(self.world)])
        stat = torch.cat([rows[r, 8 + self.cap[0]:8 + self.cap[0] + int(cc[r, 1])] for r in range(self.world)])
        return spec, stat


class PipelinedGather:
    """The per-step collective for TWO diff passes in flight: two contexts, each on its own stream, diff a
    batch and its view (gpudiff_dbatch_create_view) on alternate steps, so pass s + 1's decision kernel
    fills the CUs pass s's tail frees while pass s's compaction, joins and collective run beside it.

    Pass p = s % 2 owns send / gathered buffer p, bound to its batch (gpudiff_dbatch_bind_gather: the
    engine's compaction writes [8 counts | spec IDs | status IDs] there), and its all-gather runs on its
    stream (torch's ProcessGroupNCCL orders the collective after the current stream's work and the stream
    after the collective; the communicator serialises collectives in issue order, the same on every
    rank).  Step s's gathered counts are copied to pinned memory behind an event and checked only after
    step s + 1 is queued; a capacity exceeded on any rank (every rank sees the same counts) grows both
    buffers and re-gathers step s from batch s % 2 -- its lists stay until step s + 2 -- and the in-flight
    step s + 1 from the other, each on its own stream.  Replaced buffers are kept alive until finish(), as
    a collective still queued may read them.

    comm_device = cpu (the gloo rehearsal of this path on one GPU, where RCCL refuses two ranks per device):
    the send buffers stay on the GPU -- the engines still write them from their compaction -- and each
    step's buffer is staged into a pinned host tensor on its pass's stream after that pass, then gathered
    by gloo on the host.  Binding, views, lookahead and regrow are the RCCL path's; only the transport
    differs (and the host waits for pass s before gathering it, so the rehearsal's timings are not the
    node's)."""

    def __init__(self, world: int, cap_spec: int, cap_status: int, device, dist, streams, binds,
                 grow: float = 1.25, comm_device=None):
        import numpy as np
        import torch
        self.world, self.dist, self.device = world, dist, device
        self.host = comm_device is not None and torch.device(comm_device).type == "cpu"
        self.streams, self.binds = list(streams), list(binds)
        self.grow = max(1.0, float(grow))
        self.n_steps = 0
        self.n_regrows = 0
        self.pending = None
        self.maxc_host = np.zeros((world, 2), dtype=np.int64)
        self.hc = [torch.zeros((world, 2), dtype=torch.int32, pin_memory=True) for _ in range(2)]
        self.ev = [torch.cuda.Event() for _ in range(2)]
        self.graveyard = []
        self.gathered = []  # (step, rank-0 rows [world, 8] as gathered) -- every gather, regrows included
        self.trace = False
        self._alloc(cap_spec, cap_status)

    def _alloc(self, cap_spec: int, cap_status: int):
        import torch
        if getattr(self, "sends", None) is not None:
            self.graveyard += self.sends + self.alls
        self.cap = (max(1, int(cap_spec)), max(1, int(cap_status)))
        self.width = 8 + self.cap[0] + self.cap[1]
        self.sends, self.alls = [], []
        # gloo: the host mirrors the collective reads and writes (the send buffers stay device memory)
        self.hsends = [torch.zeros(self.width, dtype=torch.int32, pin_memory=True) for _ in range(2)] \
            if self.host else None
        for p in range(2):
            with torch.cuda.stream(self.streams[p]):
                self.sends.append(torch.zeros(self.width, dtype=torch.int32, device=self.device))
                self.alls.append(torch.zeros(self.world * self.width, dtype=torch.int32,
                                             device="cpu" if self.host else self.device))
            self.binds[p](self.sends[p], self.cap[0], self.cap[1])
        self.caps_at = [self.cap, self.cap]

    def _views(self, p: int):
        s = self.sends[p]
        return s[:8], [s[8:8 + self.cap[0]], s[8 + self.cap[0]:]]

    def _gather(self, p: int, step: int = -1):
        import torch
        if self.host:
            # pass p's send buffer (written by its compaction, on its stream) -> pinned host -> gloo
            with torch.cuda.stream(self.streams[p]):
                self.hsends[p].copy_(self.sends[p], non_blocking=True)
            self.streams[p].synchronize()
            self.dist.all_gather_into_tensor(self.alls[p], self.hsends[p])
            self.hc[p].copy_(self.alls[p].view(self.world, self.width)[:, :2])
            self.ev[p].record(self.streams[p])  # already complete: keeps _check's wait uniform
        else:
            with torch.cuda.stream(self.streams[p]):
                self.dist.all_gather_into_tensor(self.alls[p], self.sends[p])
                self.hc[p].copy_(self.alls[p].view(self.world, self.width)[:, :2], non_blocking=True)
                self.ev[p].record()
        self.caps_at[p] = self.cap
        if self.trace:  # tests: what each gather delivered (synchronises; never in a timed run)
            self.streams[p].synchronize()
            rows = self.alls[p].view(self.world, self.width)
            self.gathered.append((step, self.cap, rows.cpu().clone()))

    def step(self, fill_counts, fill_ids):
        """After step s's diff was enqueued on pass s % 2's context.  fill_counts(p, t) / fill_ids(p, col,
        buf) re-export pass p's results (used only after a regrow)."""
        s = self.n_steps
        self._gather(s % 2, s)
        prev, self.pending = self.pending, s
        self.n_steps += 1
        self._fills = (fill_counts, fill_ids)
        if prev is not None:
            self._check(prev)

    def _check(self, s: int):
        import torch
        p = s % 2
        self.ev[p].synchronize()
        hc = self.hc[p].clone()
        cap = self.caps_at[p]
        self.maxc_host = self.maxc_host.clip(min=hc.numpy())
        if not bool((hc[:, 0] > cap[0]).any() or (hc[:, 1] > cap[1]).any()):
            return
        ms, mt = int(hc[:, 0].max()), int(hc[:, 1].max())
        self._alloc(max(self.cap[0], int(ms * self.grow) + 1), max(self.cap[1], int(mt * self.grow) + 1))
        fill_counts, fill_ids = self._fills
        for t in [s] + ([s + 1] if self.pending == s + 1 else []):
            q = t % 2
            counts, bufs = self._views(q)
            with torch.cuda.stream(self.streams[q]):
                fill_counts(q, counts)
                for col in (0, 1):
                    fill_ids(q, col, bufs[col])
            self._gather(q, t)
        self.n_regrows += 1

    def finish(self):
        """Check the last step (inside the timed region: it waits for the last collective)."""
        import torch
        if self.pending is not None:
            s, self.pending = self.pending, None
            self._check(s)
            self.ev[s % 2].synchronize()
        for st in self.streams:
            torch.cuda.current_stream().wait_stream(st)

    def check(self):
        ok = bool((self.maxc_host[:, 0] <= self.cap[0]).all() and (self.maxc_host[:, 1] <= self.cap[1]).all())
        p = (self.n_steps - 1) % 2
        cc = self.alls[p].view(self.world, self.width)[:, :8].cpu()
        return ok, cc

    def result(self):
        """Node-wide (spec IDs, status IDs) of the last step, in rank order."""
        import torch
        ok, cc = self.check()
        if not ok:
            raise RuntimeError("dirty-ID capacity exceeded: %s > %s" % (self.maxc_host.tolist(), self.cap))
        rows = self.alls[(self.n_steps - 1) % 2].view(self.world, self.width)
        spec = torch.cat([rows[r, 8:8 + int(cc[r, 0])] for r in range(self.world)])
        stat = torch.cat([rows[r, 8 + self.cap[0]:8 + self.cap[0] + int(cc[r, 1])] for r in range(self.world)])
        return spec, stat

    @property
    def depth(self):
        return 2

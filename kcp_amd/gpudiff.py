"""ctypes binding of libgpudiff.so (include/gpudiff.h).

This is the Python host side above the C-ABI.  It holds no diff logic: every
decision is made by the HIP kernels behind the C-ABI.  If the shared library
is missing the import fails loudly (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
import json
import os
from dataclasses import dataclass
from typing import Any, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import buildinfo

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgpudiff.so")

ABI_VERSION = 6  # GPUDIFF_ABI_VERSION of include/gpudiff.h
OK = 0
E_INVAL, E_NOMEM, E_DEVICE, E_NODEVICE, E_CAPACITY, E_STATE, E_DECODE, E_NOTFOUND = range(-1, -9, -1)

SPEC_DIRTY, STATUS_DIRTY, DECODE_ERROR, SPEC_NOOP, STATUS_NOOP = 0x1, 0x2, 0x4, 0x8, 0x10
PATH_CHANGED, PATH_ADDED, PATH_REMOVED, PATH_STATUS_ABSENT = 0, 1, 2, 3
PATH_REGION_STATUS = 0x80
OPT_TIMING = 0x1
OPT_DEVICE_ENCODE = 0x2000000
OPT_ARENA_SHIFT = 21  # test hook: 4 bits, the K2 wave arenas shrunk 2^k-fold (forces the deferred K4 path)
DEVICE_CURRENT, DEVICE_NONE = -1, -2

PATH_HASH_BITS = 32  # GPUDIFF_PATH_HASH_BITS: segment keys and reported path hashes
OBJ_HAS_STATUS, OBJ_DECODE_ERR, OBJ_FRESH, OBJ_SEED_SHIFT = 0x1, 0x2, 0x4, 8
STORE_DEVICE_ENCODE = 0x1
EXPORT_COUNTS, EXPORT_SPEC_IDS, EXPORT_STATUS_IDS, EXPORT_DIRTY_IDS, EXPORT_FLAGS = range(5)


class GpuDiffError(RuntimeError):
    def __init__(self, code: int, where: str):
        self.code = code
        super().__init__("%s: %s (%d)" % (where, _lib.gpudiff_strerror(code).decode(), code))


class Opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("encode_threads", C.c_uint32), ("stream", C.c_void_p),
                ("flags", C.c_uint32), ("path_hash_bits", C.c_uint32)]


class JsonPair(C.Structure):
    _fields_ = [("old_json", C.c_void_p), ("old_len", C.c_size_t), ("new_json", C.c_void_p),
                ("new_len", C.c_size_t), ("pair_id", C.c_uint32), ("cluster_id", C.c_uint32)]


# numpy mirror of gpudiff_json_pair (zero-copy pair tables over one JSON buffer)
JSON_PAIR_DTYPE = np.dtype([("old_json", "<u8"), ("old_len", "<u8"), ("new_json", "<u8"), ("new_len", "<u8"),
                            ("pair_id", "<u4"), ("cluster_id", "<u4")])
assert JSON_PAIR_DTYPE.itemsize == C.sizeof(JsonPair)


def json_pair_array(buf: np.ndarray, offs: np.ndarray, ids=None, clusters=None) -> np.ndarray:
    """Pair table over one contiguous JSON buffer: pair i's old object is
    buf[offs[2i]:offs[2i+1]], its new one buf[offs[2i+1]:offs[2i+2]].  The
    buffer must outlive every submit of the table."""
    n = (len(offs) - 1) // 2
    base = buf.ctypes.data
    o = offs.astype(np.uint64)
    arr = np.zeros(n, dtype=JSON_PAIR_DTYPE)
    arr["old_json"] = base + o[0:2 * n:2]
    arr["old_len"] = o[1:2 * n + 1:2] - o[0:2 * n:2]
    arr["new_json"] = base + o[1:2 * n + 1:2]
    arr["new_len"] = o[2:2 * n + 2:2] - o[1:2 * n + 1:2]
    arr["pair_id"] = np.arange(n, dtype=np.uint32) if ids is None else ids
    arr["cluster_id"] = 0 if clusters is None else clusters
    return arr


ZC_SLACK = 32  # gpudiff.h gpudiff_host_alloc: a document's staged span is len + 32 rounded up to 16


def zero_copy_layout(lens: np.ndarray):
    """Offsets of documents laid out for gpudiff_submit's zero-copy upload (gpudiff.h gpudiff_host_alloc): each
    at a 16-B aligned offset, followed by its staged span; returns (offsets, bytes the buffer needs)."""
    span = (lens.astype(np.uint64) + ZC_SLACK + 15) & ~np.uint64(15)
    offs = np.zeros(lens.size, np.uint64)
    np.cumsum(span[:-1], out=offs[1:])
    return offs, int(offs[-1] + span[-1]) + ZC_SLACK if lens.size else ZC_SLACK


class PinnedJson:
    """A gpudiff_host_alloc buffer holding JSON pairs in the zero-copy layout, with its pair table: what the
    syncer batcher produces when it renders a flush straight into engine-pinned memory.
    Free it (or the engine) when done; every submit of `pairs` must be waited first."""

    def __init__(self, eng: "Engine", buf: np.ndarray, offs: np.ndarray, ids=None, clusters=None):
        n = (len(offs) - 1) // 2
        o = offs.astype(np.int64)
        lens = np.diff(o)
        doffs, nbytes = zero_copy_layout(lens)
        p = C.c_void_p()
        _chk(_lib.gpudiff_host_alloc(eng.ctx, nbytes, C.byref(p)), "gpudiff_host_alloc")
        self.eng, self.ptr, self.nbytes = eng, p.value, nbytes
        dst = np.ctypeslib.as_array(C.cast(self.ptr, C.POINTER(C.c_uint8)), (nbytes,))
        src = np.ascontiguousarray(buf)
        for k in range(2 * n):  # the render step of the batcher (untimed in the benches)
            a, ln, d = int(o[k]), int(lens[k]), int(doffs[k])
            dst[d:d + ln] = src[a:a + ln]
        self.pairs = np.zeros(n, dtype=JSON_PAIR_DTYPE)
        self.pairs["old_json"] = self.ptr + doffs[0:2 * n:2]
        self.pairs["old_len"] = lens[0:2 * n:2]
        self.pairs["new_json"] = self.ptr + doffs[1:2 * n:2]
        self.pairs["new_len"] = lens[1:2 * n:2]
        self.pairs["pair_id"] = np.arange(n, dtype=np.uint32) if ids is None else ids
        self.pairs["cluster_id"] = 0 if clusters is None else clusters

    def free(self):
        if self.ptr:
            _chk(_lib.gpudiff_host_free(self.eng.ctx, self.ptr), "gpudiff_host_free")
            self.ptr = None


class PinnedDocs:
    """Documents in one gpudiff_host_alloc buffer, each at a 16-B aligned offset followed by its staged span (the
    zero-copy layout of gpudiff.h gpudiff_host_alloc): what a watch-stream reader produces when it writes each
    event's JSON straight into engine-pinned memory.  `ptrs[i]` is document i's address.  Free it (or the engine)
    once every submit that reads it has been waited."""

    def __init__(self, eng: "Engine", lens):
        lens = np.asarray(lens, dtype=np.uint64)
        self.offs, self.nbytes = zero_copy_layout(lens)
        self.lens = lens
        p = C.c_void_p()
        _chk(_lib.gpudiff_host_alloc(eng.ctx, self.nbytes, C.byref(p)), "gpudiff_host_alloc")
        self.eng, self.ptr = eng, p.value
        self.view = np.ctypeslib.as_array(C.cast(self.ptr, C.POINTER(C.c_uint8)), (self.nbytes,))
        self.ptrs = self.offs + np.uint64(self.ptr)

    @classmethod
    def of_bytes(cls, eng: "Engine", docs):
        docs = [bytes(d) for d in docs]
        pd = cls(eng, [len(d) for d in docs])
        for o, d in zip(pd.offs.tolist(), docs):
            pd.view[o:o + len(d)] = np.frombuffer(d, np.uint8)
        return pd

    @classmethod
    def of_ranges(cls, eng: "Engine", buf: np.ndarray, starts, lens):
        """Document i = buf[starts[i] : starts[i] + lens[i]] (the render step; untimed in the benches)."""
        pd = cls(eng, lens)
        src = np.ascontiguousarray(buf)
        for o, a, n in zip(pd.offs.tolist(), np.asarray(starts).tolist(), np.asarray(lens).tolist()):
            pd.view[o:o + n] = src[a:a + n]
        return pd

    def free(self):
        if self.ptr and self.eng.ctx:
            _chk(_lib.gpudiff_host_free(self.eng.ctx, self.ptr), "gpudiff_host_free")
        self.ptr = None


class PairRow(C.Structure):
    _fields_ = [("off_a", C.c_uint64), ("off_b", C.c_uint64),
                ("spec_l_a", C.c_uint32), ("spec_l_b", C.c_uint32),
                ("spec_ar_a", C.c_uint32), ("spec_ar_b", C.c_uint32),
                ("stat_l_a", C.c_uint32), ("stat_l_b", C.c_uint32),
                ("stat_ar_a", C.c_uint32), ("stat_ar_b", C.c_uint32),
                ("flags_a", C.c_uint32), ("flags_b", C.c_uint32),
                ("pair_id", C.c_uint32), ("cluster_id", C.c_uint32)]


ROW_DTYPE = np.dtype([("off_a", "<u8"), ("off_b", "<u8"), ("spec_l_a", "<u4"), ("spec_l_b", "<u4"),
                      ("spec_ar_a", "<u4"), ("spec_ar_b", "<u4"), ("stat_l_a", "<u4"), ("stat_l_b", "<u4"),
                      ("stat_ar_a", "<u4"), ("stat_ar_b", "<u4"), ("flags_a", "<u4"), ("flags_b", "<u4"),
                      ("pair_id", "<u4"), ("cluster_id", "<u4")])
assert ROW_DTYPE.itemsize == 64


class Event(C.Structure):
    _fields_ = [("slot", C.c_uint32), ("pair_id", C.c_uint32), ("cluster_id", C.c_uint32), ("reserved", C.c_uint32),
                ("new_json", C.c_void_p), ("new_len", C.c_size_t), ("old_json", C.c_void_p), ("old_len", C.c_size_t)]


class StoreStats(C.Structure):
    _fields_ = [("max_slots", C.c_uint64), ("live_slots", C.c_uint64), ("space_bytes", C.c_uint64),
                ("used_bytes", C.c_uint64), ("live_bytes", C.c_uint64), ("compactions", C.c_uint64),
                ("events", C.c_uint64), ("old_encoded", C.c_uint64), ("reseeded", C.c_uint64),
                ("collisions_unresolved", C.c_uint64), ("last_batch_bytes", C.c_uint64), ("deferred", C.c_uint64),
                ("host_submit_ms", C.c_float), ("h2d_ms", C.c_float), ("encode_ms", C.c_float),
                ("link_ms", C.c_float), ("submit_wait_ms", C.c_float), ("submit_docs_ms", C.c_float),
                ("submit_copy_ms", C.c_float), ("submit_enqueue_ms", C.c_float), ("finish_ms", C.c_float),
                ("timing_batches", C.c_uint32), ("zero_copy_batches", C.c_uint32), ("space_conservative", C.c_uint64)]


class ObjInfo(C.Structure):
    _fields_ = [("status", C.c_int32), ("oflags", C.c_uint32), ("spec_l", C.c_uint32), ("spec_ar", C.c_uint32),
                ("stat_l", C.c_uint32), ("stat_ar", C.c_uint32), ("off", C.c_uint64), ("bytes", C.c_uint64),
                ("n_tab", C.c_uint32), ("reserved", C.c_uint32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


TOK_OK, TOK_SYNTAX, TOK_NUMBER, TOK_KEY, TOK_STRING, TOK_HASH, TOK_DEPTH, TOK_SIZE, TOK_SPACE, TOK_FLOAT, TOK_WIDE, \
    TOK_FIELD, TOK_LIST = range(13)
ROLLUP_NONE, ROLLUP_DECODE = -1, -2

UPSERT_SPEC, UPSERT_STATUS = 0, 1
# gpudiff_write_plan_get_ex modes: which writes, rendered from which document of a pair
PLAN_INFORMER, PLAN_SPEC, PLAN_STATUS, PLAN_UPSTREAM_DOWNSTREAM = 0x0, 0x1, 0x2, 0x4
BODY_DEVICE, BODY_HOST = 0, 1


class Bodies(C.Structure):
    _fields_ = [("n", C.c_size_t), ("offsets", C.c_void_p), ("bytes", C.c_void_p), ("status", C.c_void_p),
                ("source", C.c_void_p), ("k10_status", C.c_void_p), ("n_host", C.c_size_t),
                ("internal", C.c_void_p)]


class WritePlanC(C.Structure):
    _fields_ = [("n", C.c_size_t), ("pair_index", C.c_void_p), ("kind", C.c_void_p), ("noop", C.c_void_p),
                ("bodies", Bodies), ("internal", C.c_void_p)]


class WBatchStats(C.Structure):
    _fields_ = [("n_docs", C.c_uint64), ("json_bytes", C.c_uint64), ("body_bytes", C.c_uint64),
                ("scratch_bytes", C.c_uint64), ("out_cap_bytes", C.c_uint64), ("k10_ms", C.c_double),
                ("runs", C.c_uint64)]


class RollupGroup(C.Structure):
    _fields_ = [("first_doc", C.c_uint32), ("n_members", C.c_uint32), ("sums", C.c_int32 * 5),
                ("reserved", C.c_uint32)]


class Rollup(C.Structure):
    _fields_ = [("n_docs", C.c_size_t), ("doc_group", C.c_void_p), ("n_groups", C.c_size_t), ("groups", C.c_void_p),
                ("k11_status", C.c_void_p), ("n_host", C.c_size_t), ("host_grouped", C.c_uint32),
                ("internal", C.c_void_p)]


class RBatchStats(C.Structure):
    _fields_ = [("n_docs", C.c_uint64), ("json_bytes", C.c_uint64), ("scratch_bytes", C.c_uint64),
                ("k11_ms", C.c_double), ("k12_ms", C.c_double), ("runs", C.c_uint64)]


class NBatchStats(C.Structure):
    _fields_ = [("n_pairs", C.c_uint64), ("json_bytes", C.c_uint64), ("scratch_bytes", C.c_uint64),
                ("n_host", C.c_uint64), ("k13_ms", C.c_double), ("k14_ms", C.c_double), ("runs", C.c_uint64)]


class HBatchInfo(C.Structure):
    _fields_ = [("n_pairs", C.c_size_t), ("rows", C.c_void_p), ("pool", C.c_void_p), ("pool_bytes", C.c_uint64),
                ("total_leaves", C.c_uint64), ("n_decode_errors", C.c_uint64), ("n_reseeded", C.c_uint64)]


class Result(C.Structure):
    _fields_ = [("n_pairs", C.c_size_t), ("pair_flags", C.c_void_p),
                ("n_spec_dirty", C.c_size_t), ("spec_dirty_ids", C.c_void_p),
                ("n_status_dirty", C.c_size_t), ("status_dirty_ids", C.c_void_p),
                ("n_dirty", C.c_size_t), ("dirty_ids", C.c_void_p), ("path_offsets", C.c_void_p),
                ("n_paths", C.c_size_t), ("path_hashes", C.c_void_p), ("path_kinds", C.c_void_p),
                ("internal_", C.c_void_p)]


class DeviceView(C.Structure):
    _fields_ = [("pair_flags", C.c_void_p), ("spec_dirty_ids", C.c_void_p), ("status_dirty_ids", C.c_void_p),
                ("dirty_ids", C.c_void_p), ("counts", C.c_void_p)]


class BatchStats(C.Structure):
    _fields_ = [("n_pairs", C.c_uint64), ("pool_bytes", C.c_uint64), ("total_leaves", C.c_uint64),
                ("compare_bytes", C.c_uint64), ("value_bytes", C.c_uint64)]


class Timings(C.Structure):
    _fields_ = [("compare_ms", C.c_float), ("compact_ms", C.c_float),
                ("join_ms", C.c_float), ("emit_ms", C.c_float), ("total_ms", C.c_float),
                ("n_passes", C.c_uint32), ("k2_launches", C.c_uint32)]


# (name, restype, argtypes) for every symbol of include/gpudiff.h
_P = C.c_void_p
SIGNATURES = [
    ("gpudiff_strerror", C.c_char_p, [C.c_int]),
    ("gpudiff_abi_version", C.c_int, []),
    ("gpudiff_build_id", C.c_char_p, []),
    ("gpudiff_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("gpudiff_open", C.c_int, [C.POINTER(Opts), C.POINTER(_P)]),
    ("gpudiff_close", None, [_P]),
    ("gpudiff_encode_pairs", C.c_int, [_P, C.POINTER(JsonPair), C.c_size_t, C.POINTER(_P)]),
    ("gpudiff_hbatch_info_get", C.c_int, [_P, C.POINTER(HBatchInfo)]),
    ("gpudiff_hbatch_free", None, [_P, _P]),
    ("gpudiff_dbatch_create", C.c_int, [_P, C.c_uint64, C.c_uint64, C.POINTER(_P)]),
    ("gpudiff_dbatch_append", C.c_int, [_P, _P, _P]),
    ("gpudiff_dbatch_reset", C.c_int, [_P, _P]),
    ("gpudiff_dbatch_stats_get", C.c_int, [_P, C.POINTER(BatchStats)]),
    ("gpudiff_dbatch_device_view", C.c_int, [_P, C.POINTER(DeviceView)]),
    ("gpudiff_dbatch_read_pool", C.c_int, [_P, _P, C.c_uint64, C.c_void_p, C.c_uint64]),
    ("gpudiff_dbatch_export", C.c_int, [_P, _P, C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64]),
    ("gpudiff_dbatch_free", None, [_P, _P]),
    ("gpudiff_dbatch_bind_gather", C.c_int, [_P, _P, C.c_void_p, C.c_uint32, C.c_uint32]),
    ("gpudiff_dbatch_result_slot", C.c_int, [_P, _P, C.c_uint32]),
    ("gpudiff_dbatch_create_view", C.c_int, [_P, _P, C.POINTER(_P)]),
    ("gpudiff_cluster_bytes", C.c_int, [C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p]),
    ("gpudiff_shard_lpt", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]),
    ("gpudiff_diff", C.c_int, [_P, _P, C.POINTER(C.c_uint64)]),
    ("gpudiff_wait", C.c_int, [_P, C.c_uint64, C.POINTER(Result)]),
    ("gpudiff_result_release", None, [_P, C.POINTER(Result)]),
    ("gpudiff_last_timings", C.c_int, [_P, C.POINTER(Timings)]),
    ("gpudiff_sync", C.c_int, [_P]),
    ("gpudiff_timing_reset", C.c_int, [_P]),
    ("gpudiff_hbatch_create", C.c_int, [_P, C.c_uint64, C.c_size_t, C.c_uint64, C.POINTER(_P), C.POINTER(_P),
                                        C.POINTER(_P)]),
    ("gpudiff_hbatch_resize", C.c_int, [_P, _P, C.c_uint64, C.c_size_t, C.c_uint64, C.POINTER(_P),
                                        C.POINTER(_P)]),
    ("gpudiff_submit", C.c_int, [_P, C.POINTER(JsonPair), C.c_size_t, C.POINTER(C.c_uint64)]),
    ("gpudiff_store_create", C.c_int, [_P, C.c_uint32, C.c_uint64, C.c_uint32, C.POINTER(_P)]),
    ("gpudiff_store_create_ex", C.c_int, [_P, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    ("gpudiff_store_submit", C.c_int, [_P, _P, C.POINTER(Event), C.c_size_t, C.POINTER(C.c_uint64)]),
    ("gpudiff_store_forget", C.c_int, [_P, _P, C.c_uint32]),
    ("gpudiff_store_stats_get", C.c_int, [_P, C.POINTER(StoreStats)]),
    ("gpudiff_submit_stats_get", C.c_int, [_P, C.POINTER(StoreStats)]),
    ("gpudiff_host_alloc", C.c_int, [_P, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("gpudiff_host_free", C.c_int, [_P, C.c_void_p]),
    ("gpudiff_store_free", None, [_P, _P]),
    ("gpudiff_encode_objects", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_uint32),
                                         C.c_size_t, C.c_void_p, C.c_uint64, C.POINTER(ObjInfo)]),
    ("gpudiff_encode_object_host", C.c_int, [C.c_char_p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64,
                                             C.POINTER(ObjInfo)]),
    ("gpudiff_k0_profile", C.c_int, [_P, C.c_int, C.POINTER(C.c_uint64)]),
    ("gpudiff_k2_profile", C.c_int, [_P, C.c_void_p, C.c_uint32]),
    ("gpudiff_upsert_bodies", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t, C.c_uint32,
                                        C.POINTER(Bodies)]),
    ("gpudiff_bodies_release", None, [_P, C.POINTER(Bodies)]),
    ("gpudiff_write_plan_get", C.c_int, [_P, C.c_uint64, C.POINTER(WritePlanC)]),
    ("gpudiff_write_plan_get_ex", C.c_int, [_P, C.c_uint64, C.c_uint32, C.POINTER(WritePlanC)]),
    ("gpudiff_write_plan_release", None, [_P, C.POINTER(WritePlanC)]),
    ("gpudiff_wbatch_create", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t, C.c_uint32,
                                        C.POINTER(_P)]),
    ("gpudiff_wbatch_run", C.c_int, [_P, _P]),
    ("gpudiff_wbatch_fetch", C.c_int, [_P, _P, C.POINTER(Bodies)]),
    ("gpudiff_wbatch_stats_get", C.c_int, [_P, C.POINTER(WBatchStats)]),
    ("gpudiff_wbatch_free", None, [_P, _P]),
    ("gpudiff_upsert_body_host", C.c_int, [C.c_char_p, C.c_size_t, C.c_uint32, C.c_void_p, C.c_size_t,
                                           C.POINTER(C.c_size_t)]),
    ("gpudiff_rbatch_create", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t,
                                        C.POINTER(_P)]),
    ("gpudiff_rbatch_run", C.c_int, [_P, _P]),
    ("gpudiff_rbatch_fetch", C.c_int, [_P, _P, C.POINTER(Rollup)]),
    ("gpudiff_rbatch_stats_get", C.c_int, [_P, C.POINTER(RBatchStats)]),
    ("gpudiff_rbatch_free", None, [_P, _P]),
    ("gpudiff_rollup_status", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t,
                                        C.POINTER(Rollup)]),
    ("gpudiff_rollup_release", None, [_P, C.POINTER(Rollup)]),
    ("gpudiff_rollup_doc_host", C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_int32), C.c_void_p, C.c_size_t,
                                          C.POINTER(C.c_size_t)]),
    ("gpudiff_nbatch_create", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_void_p),
                                        C.POINTER(C.c_size_t), C.c_size_t, C.POINTER(_P)]),
    ("gpudiff_nbatch_run", C.c_int, [_P, _P]),
    ("gpudiff_nbatch_fetch", C.c_int, [_P, _P, C.POINTER(C.c_int32)]),
    ("gpudiff_nbatch_stats_get", C.c_int, [_P, C.POINTER(NBatchStats)]),
    ("gpudiff_nbatch_free", None, [_P, _P]),
    ("gpudiff_nbatch_create_kinds", C.c_int, [_P, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                              C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t, C.POINTER(_P)]),
    ("gpudiff_classify_updates", C.c_int, [_P, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_void_p),
                                           C.POINTER(C.c_size_t), C.c_size_t, C.POINTER(C.c_int32)]),
    ("gpudiff_classify_updates_kinds", C.c_int, [_P, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                                 C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t,
                                                 C.POINTER(C.c_int32)]),
    ("gpudiff_classify_updates_host_kinds", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                                      C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_size_t,
                                                      C.c_uint32, C.POINTER(C.c_int32)]),
    ("gpudiff_negotiate_pair_host_kind", C.c_int, [C.c_uint32, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                                   C.POINTER(C.c_int32)]),
    ("gpudiff_classify_updates_host", C.c_int, [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_void_p),
                                                C.POINTER(C.c_size_t), C.c_size_t, C.c_uint32, C.POINTER(C.c_int32)]),
    ("gpudiff_negotiate_pair_host", C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                              C.POINTER(C.c_int32)]),
    ("gpudiff_spec_equal", C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]),
    ("gpudiff_status_equal", C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]),
    ("gpudiff_resolve_path", C.c_int, [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_uint64, C.c_uint8,
                                       C.c_uint32, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
]


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError("libgpudiff.so not built (run `python kcp_amd/build.py`); there is no CPU fallback")
    from . import _hiprt
    _hiprt.preload()  # share torch's HIP runtime instead of mapping a second one
    lib = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    # the structures above and the meaning of unchanged symbols (e.g. gpudiff_write_plan_get's default
    # mode, ABI 4) follow this ABI: a library built from other headers is refused, not half-used
    got = lib.gpudiff_abi_version()
    if got != ABI_VERSION:
        raise ImportError("%s has ABI %d, this binding needs %d (rebuild with kcp_amd/build.py)"
                          % (LIB_PATH, got, ABI_VERSION))
    # ...and a library built from other sources than the ones shipped beside it is refused too: the ID is a
    # content hash of every source, header and build flag (kcp_amd/buildinfo.py), never an mtime
    global BUILD_ID, BUILD_VERIFIED
    BUILD_ID = lib.gpudiff_build_id().decode()
    if buildinfo.sources_present():
        want = buildinfo.source_id()
        if BUILD_ID != want:
            raise ImportError("%s was built from other sources (build ID %s, the shipped sources hash to %s): "
                              "rebuild with kcp_amd/build.py" % (LIB_PATH, BUILD_ID, want))
        BUILD_VERIFIED = True
    return lib


BUILD_ID = ""          # gpudiff_build_id() of the loaded library
BUILD_VERIFIED = False  # True when it equals the shipped sources' content hash
_lib = _load()


def lib() -> C.CDLL:
    return _lib


def _chk(rc: int, where: str):
    if rc != OK:
        raise GpuDiffError(rc, where)


def device_count() -> int:
    n = C.c_int(0)
    _chk(_lib.gpudiff_device_count(C.byref(n)), "gpudiff_device_count")
    return n.value


def cluster_bytes(rows: np.ndarray, n_clusters: int) -> np.ndarray:
    """Σ B_pair per logical cluster of encoded rows (ROW_DTYPE): the bytes K2 streams for each cluster's
    pairs -- the shard weight of SURVEY.md §8(e) (gpudiff_cluster_bytes)."""
    rows = np.ascontiguousarray(rows, dtype=ROW_DTYPE)
    out = np.zeros(n_clusters, dtype=np.uint64)
    _chk(_lib.gpudiff_cluster_bytes(rows.ctypes.data, rows.size, n_clusters, out.ctypes.data), "gpudiff_cluster_bytes")
    return out


def shard_lpt(weights, world: int) -> np.ndarray:
    """Owner rank per cluster: greedy LPT by weight (gpudiff_shard_lpt; shard.lpt_assign restates it)."""
    w = np.ascontiguousarray(weights, dtype=np.uint64)
    owner = np.zeros(w.size, dtype=np.int32)
    _chk(_lib.gpudiff_shard_lpt(w.ctypes.data, w.size, world, owner.ctypes.data), "gpudiff_shard_lpt")
    return owner


def to_json_bytes(obj: Union[bytes, bytearray, str, dict]) -> bytes:
    if isinstance(obj, (bytes, bytearray)):
        return bytes(obj)
    if isinstance(obj, str):
        return obj.encode()
    return json.dumps(obj, separators=(",", ":")).encode()


@dataclass
class DiffResult:
    """Host copy of one batch's results (all arrays in batch order)."""
    pair_flags: np.ndarray          # u8 [n_pairs]
    spec_dirty_ids: np.ndarray      # u32
    status_dirty_ids: np.ndarray    # u32
    dirty_ids: np.ndarray           # u32
    path_offsets: np.ndarray        # u32 [n_dirty + 1]
    path_hashes: np.ndarray         # u64
    path_kinds: np.ndarray          # u8

    def paths_of(self, k: int) -> List[Tuple[int, int]]:
        """[(hash, kind)] of the k-th dirty pair."""
        b, e = int(self.path_offsets[k]), int(self.path_offsets[k + 1])
        return list(zip(self.path_hashes[b:e].tolist(), self.path_kinds[b:e].tolist()))


def _arr(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    ct = np.ctypeslib.as_ctypes_type(np.dtype(dtype))
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,)).copy()


class HostBatch:
    def __init__(self, engine: "Engine", handle: int, keep: Any):
        self.engine = engine
        self.h = C.c_void_p(handle)
        self._keep = keep

    def info(self) -> HBatchInfo:
        inf = HBatchInfo()
        _chk(_lib.gpudiff_hbatch_info_get(self.h, C.byref(inf)), "gpudiff_hbatch_info_get")
        return inf

    def rows(self) -> np.ndarray:
        inf = self.info()
        if inf.n_pairs == 0:
            return np.zeros(0, dtype=ROW_DTYPE)
        buf = (C.c_uint8 * (inf.n_pairs * 64)).from_address(inf.rows)
        return np.frombuffer(bytes(buf), dtype=ROW_DTYPE)

    def pool(self) -> bytes:
        inf = self.info()
        return C.string_at(inf.pool, inf.pool_bytes) if inf.pool_bytes else b""

    def pool_view(self) -> np.ndarray:
        """The pool as a u8 array over the batch's own host memory (no copy; C.string_at takes a C int
        size, so pools over 2 GiB -- config4's 7 GB -- cannot go through pool()).  Valid while the batch
        lives."""
        inf = self.info()
        if not inf.pool_bytes:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array((C.c_uint8 * inf.pool_bytes).from_address(inf.pool))

    def free(self):
        if self.h:
            _lib.gpudiff_hbatch_free(self.engine.ctx, self.h)
            self.h = C.c_void_p(0)

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceBatch:
    def __init__(self, engine: "Engine", pool_bytes: int, max_pairs: int, _view_of: "DeviceBatch" = None):
        self.engine = engine
        h = C.c_void_p()
        if _view_of is None:
            _chk(_lib.gpudiff_dbatch_create(engine.ctx, pool_bytes, max_pairs, C.byref(h)), "gpudiff_dbatch_create")
        else:
            _chk(_lib.gpudiff_dbatch_create_view(engine.ctx, _view_of.h, C.byref(h)), "gpudiff_dbatch_create_view")
        self.base = _view_of  # keeps the base alive while the view lives
        self.h = h

    def view(self, engine: "Engine") -> "DeviceBatch":
        """A batch with its own outputs over this batch's resident pairs, diffed by `engine` (typically a
        second context on its own stream: two passes in flight, gpudiff_dbatch_create_view)."""
        return DeviceBatch(engine, 0, 0, _view_of=self)

    def append(self, hb: HostBatch):
        _chk(_lib.gpudiff_dbatch_append(self.engine.ctx, self.h, hb.h), "gpudiff_dbatch_append")

    def reset(self):
        _chk(_lib.gpudiff_dbatch_reset(self.engine.ctx, self.h), "gpudiff_dbatch_reset")

    def stats(self) -> BatchStats:
        st = BatchStats()
        _chk(_lib.gpudiff_dbatch_stats_get(self.h, C.byref(st)), "gpudiff_dbatch_stats_get")
        return st

    def device_view(self) -> DeviceView:
        v = DeviceView()
        _chk(_lib.gpudiff_dbatch_device_view(self.h, C.byref(v)), "gpudiff_dbatch_device_view")
        return v

    def export(self, what: int, dst_device_ptr: int, max_elems: int, known_count: int = 1 << 62):
        """Async D2D copy of results into caller device memory (ctx stream)."""
        _chk(_lib.gpudiff_dbatch_export(self.engine.ctx, self.h, what, dst_device_ptr, max_elems, known_count),
             "gpudiff_dbatch_export")

    def bind_gather(self, send_device_ptr: int, cap_spec: int, cap_status: int):
        """K3 of every later diff also writes [8 counts | spec IDs | status IDs] into this device buffer
        (gpudiff_dbatch_bind_gather); 0 unbinds."""
        _chk(_lib.gpudiff_dbatch_bind_gather(self.engine.ctx, self.h, send_device_ptr or None, cap_spec, cap_status),
             "gpudiff_dbatch_bind_gather")

    def result_slot(self, slot: int):
        """Select result slot 0 / 1 for later diffs, exports and waits (gpudiff_dbatch_result_slot)."""
        _chk(_lib.gpudiff_dbatch_result_slot(self.engine.ctx, self.h, slot), "gpudiff_dbatch_result_slot")

    def read_pool(self, off: int, nbytes: int) -> bytes:
        buf = C.create_string_buffer(max(nbytes, 1))
        _chk(_lib.gpudiff_dbatch_read_pool(self.engine.ctx, self.h, off, buf, nbytes), "gpudiff_dbatch_read_pool")
        return buf.raw[:nbytes]

    def free(self):
        if self.h:
            _lib.gpudiff_dbatch_free(self.engine.ctx, self.h)
            self.h = C.c_void_p(0)

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class ObjectStore:
    """Device-resident informer snapshot (gpudiff_store_*): submit(events)
    diffs each event's new object against its slot's resident version and
    makes it resident; results come back through Engine.wait(ticket)."""

    def __init__(self, engine: "Engine", max_slots: int, space_bytes: int, max_events: int,
                 device_encode: bool = False):
        self.engine = engine
        self.device_encode = device_encode
        h = C.c_void_p()
        _chk(_lib.gpudiff_store_create_ex(engine.ctx, max_slots, space_bytes, max_events,
                                          STORE_DEVICE_ENCODE if device_encode else 0, C.byref(h)),
             "gpudiff_store_create_ex")
        self.h = h
        self._keep = [None, None]  # inputs of the (at most two) submits in flight
        self._k = 0

    @staticmethod
    def events(items):
        """items: [(slot, new_json, old_json_or_None, pair_id, cluster_id)] -> (Event array, n, keepalive)."""
        n = len(items)
        arr = (Event * max(n, 1))()
        keep = []
        for i, it in enumerate(items):
            slot, new, old = it[0], it[1], it[2]
            nb = to_json_bytes(new)
            cn = C.create_string_buffer(nb, len(nb)) if nb else C.create_string_buffer(1)
            keep.append(cn)
            arr[i].slot = slot
            arr[i].pair_id = it[3] if len(it) > 3 else i
            arr[i].cluster_id = it[4] if len(it) > 4 else 0
            arr[i].new_json = C.cast(cn, C.c_void_p)
            arr[i].new_len = len(nb)
            if old is not None:
                ob = to_json_bytes(old)
                co = C.create_string_buffer(ob, len(ob)) if ob else C.create_string_buffer(1)
                keep.append(co)
                arr[i].old_json = C.cast(co, C.c_void_p)
                arr[i].old_len = len(ob)
        return arr, n, keep

    def submit(self, items, zero_copy: bool = False) -> int:
        """zero_copy (device-encode stores): every event's documents -- its old object when given, then its new one --
        are first written into one gpudiff_host_alloc buffer in the zero-copy layout, which the store uploads with
        no staging copy (old objects the store does not encode are uploaded but never read)."""
        if not zero_copy:
            arr, n, keep = self.events(items)
            return self.submit_raw(arr, n, keep)
        docs = []
        for it in items:
            if it[2] is not None:
                docs.append(to_json_bytes(it[2]))
            docs.append(to_json_bytes(it[1]))
        pd = PinnedDocs.of_bytes(self.engine, docs)
        n = len(items)
        arr = (Event * max(n, 1))()
        k = 0
        for i, it in enumerate(items):
            arr[i].slot = it[0]
            arr[i].pair_id = it[3] if len(it) > 3 else i
            arr[i].cluster_id = it[4] if len(it) > 4 else 0
            if it[2] is not None:
                arr[i].old_json, arr[i].old_len = int(pd.ptrs[k]), int(pd.lens[k])
                k += 1
            arr[i].new_json, arr[i].new_len = int(pd.ptrs[k]), int(pd.lens[k])
            k += 1
        return self.submit_raw(arr, n, pd)

    def submit_raw(self, arr, n, keep=None) -> int:
        t = C.c_uint64()
        _chk(_lib.gpudiff_store_submit(self.engine.ctx, self.h, arr, n, C.byref(t)), "gpudiff_store_submit")
        old = self._keep[self._k]
        if old is not None and isinstance(old[1], PinnedDocs):
            old[1].free()  # its batch was waited before this submit could reuse the ring slot
        self._keep[self._k] = (arr, keep)
        self._k ^= 1
        return t.value

    def forget(self, slot: int):
        _chk(_lib.gpudiff_store_forget(self.engine.ctx, self.h, slot), "gpudiff_store_forget")

    def stats(self) -> StoreStats:
        s = StoreStats()
        _chk(_lib.gpudiff_store_stats_get(self.h, C.byref(s)), "gpudiff_store_stats_get")
        return s

    def free(self):
        if self.h:
            _lib.gpudiff_store_free(self.engine.ctx, self.h)
            self.h = C.c_void_p(0)
        for k in self._keep:
            if k is not None and isinstance(k[1], PinnedDocs):
                k[1].free()
        self._keep = [None, None]

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


NEG_KIND_API, NEG_KIND_CRD = 0, 1  # GPUDIFF_NEG_KIND_*: APIResourceImport/NegotiatedAPIResource, CRD
NEGOUT_BYTES = 1184  # K13's per-document record (kcp_amd/csrc/tokenize.h NegOut)


class Engine:
    """One gpudiff context (one GPU, one stream, one submitting thread)."""

    def __init__(self, device: int = DEVICE_CURRENT, encode_threads: int = 0, stream: Optional[int] = None,
                 timing: bool = False, path_hash_bits: int = PATH_HASH_BITS, flags: int = 0,
                 device_encode: bool = False):
        if stream is not None and not stream:
            # 0 is HIP's null stream, which the engine cannot share: gpudiff_open reads NULL as "create your
            # own (non-blocking) stream", and a non-blocking stream never orders against the null stream --
            # the caller's copies / collectives would race the engine's exports.  Share a real stream:
            # s = torch.cuda.Stream(dev); torch.cuda.set_stream(s); Engine(..., stream=s.cuda_stream)
            raise ValueError("Engine(stream=0): the null stream cannot be shared; make a torch.cuda.Stream current "
                             "and pass its cuda_stream")
        o = Opts(device=device, encode_threads=encode_threads, stream=stream or None,
                 flags=(OPT_TIMING if timing else 0) | (OPT_DEVICE_ENCODE if device_encode else 0) | flags,
                 path_hash_bits=path_hash_bits)
        h = C.c_void_p()
        _chk(_lib.gpudiff_open(C.byref(o), C.byref(h)), "gpudiff_open")
        self.ctx = h
        self.path_hash_bits = min(path_hash_bits or PATH_HASH_BITS, PATH_HASH_BITS)  # the library clamps the same way

    def close(self):
        if self.ctx:
            _lib.gpudiff_close(self.ctx)
            self.ctx = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- encoding
    @staticmethod
    def _pairs(pairs: Sequence[Tuple[Any, Any]], ids: Optional[Sequence[int]] = None,
               clusters: Optional[Sequence[int]] = None):
        n = len(pairs)
        arr = (JsonPair * max(n, 1))()
        keep = []
        for i, (a, b) in enumerate(pairs):
            ab, bb = to_json_bytes(a), to_json_bytes(b)
            ca = C.create_string_buffer(ab, len(ab)) if ab else C.create_string_buffer(1)
            cb = C.create_string_buffer(bb, len(bb)) if bb else C.create_string_buffer(1)
            keep += [ca, cb]
            arr[i].old_json = C.cast(ca, C.c_void_p)
            arr[i].old_len = len(ab)
            arr[i].new_json = C.cast(cb, C.c_void_p)
            arr[i].new_len = len(bb)
            arr[i].pair_id = ids[i] if ids is not None else i
            arr[i].cluster_id = clusters[i] if clusters is not None else 0
        return arr, n, keep

    def encode(self, pairs, ids=None, clusters=None) -> HostBatch:
        arr, n, keep = self._pairs(pairs, ids, clusters)
        h = C.c_void_p()
        _chk(_lib.gpudiff_encode_pairs(self.ctx, arr, n, C.byref(h)), "gpudiff_encode_pairs")
        return HostBatch(self, h.value, None)

    # ---- device
    def device_batch(self, pool_bytes: int, max_pairs: int) -> DeviceBatch:
        return DeviceBatch(self, pool_bytes, max_pairs)

    def diff(self, db: DeviceBatch) -> int:
        t = C.c_uint64()
        _chk(_lib.gpudiff_diff(self.ctx, db.h, C.byref(t)), "gpudiff_diff")
        return t.value

    def wait(self, ticket: int) -> DiffResult:
        r = Result()
        _chk(_lib.gpudiff_wait(self.ctx, ticket, C.byref(r)), "gpudiff_wait")
        self.__dict__.get("_held", {}).pop(ticket, None)
        try:
            out = DiffResult(
                pair_flags=_arr(r.pair_flags, r.n_pairs, np.uint8),
                spec_dirty_ids=_arr(r.spec_dirty_ids, r.n_spec_dirty, np.uint32),
                status_dirty_ids=_arr(r.status_dirty_ids, r.n_status_dirty, np.uint32),
                dirty_ids=_arr(r.dirty_ids, r.n_dirty, np.uint32),
                path_offsets=_arr(r.path_offsets, r.n_dirty + 1, np.uint32),
                path_hashes=_arr(r.path_hashes, r.n_paths, np.uint64),
                path_kinds=_arr(r.path_kinds, r.n_paths, np.uint8))
        finally:
            _lib.gpudiff_result_release(self.ctx, C.byref(r))
        return out

    def sync(self):
        _chk(_lib.gpudiff_sync(self.ctx), "gpudiff_sync")

    def timing_reset(self):
        _chk(_lib.gpudiff_timing_reset(self.ctx), "gpudiff_timing_reset")

    def timings(self) -> Timings:
        t = Timings()
        _chk(_lib.gpudiff_last_timings(self.ctx, C.byref(t)), "gpudiff_last_timings")
        return t

    def submit(self, pairs, ids=None, clusters=None) -> int:
        arr, n, keep = self._pairs(pairs, ids, clusters)
        t = C.c_uint64()
        _chk(_lib.gpudiff_submit(self.ctx, arr, n, C.byref(t)), "gpudiff_submit")
        self._hold(t.value, (arr, keep))
        return t.value

    def _hold(self, ticket, bufs):
        """The caller owns a submit's inputs until gpudiff_wait (the device-encode
        path re-reads deferred pairs there): keep them alive per ticket; the
        submit ring holds at most two batches, older tickets are dropped."""
        held = self.__dict__.setdefault("_held", {})
        held[ticket] = bufs
        for t in sorted(held)[:-2]:
            del held[t]

    def submit_stats(self) -> StoreStats:
        """gpudiff_submit_stats_get: the device-encode submit path's statistics (phase times with timing)."""
        st = StoreStats()
        _chk(_lib.gpudiff_submit_stats_get(self.ctx, C.byref(st)), "gpudiff_submit_stats_get")
        return st

    def submit_array(self, arr: np.ndarray) -> int:
        """gpudiff_submit over a JSON_PAIR_DTYPE table (json_pair_array)."""
        assert arr.dtype == JSON_PAIR_DTYPE and arr.flags["C_CONTIGUOUS"]
        t = C.c_uint64()
        _chk(_lib.gpudiff_submit(self.ctx, arr.ctypes.data_as(C.POINTER(JsonPair)), arr.size, C.byref(t)),
             "gpudiff_submit")
        return t.value

    def write_plan(self, ticket: int, mode: int = PLAN_INFORMER) -> "WritePlan":
        """gpudiff_write_plan_get_ex: the writes for a waited device-encode batch (bodies from HBM).
        mode PLAN_INFORMER (default): pairs are informer (old, new) events, every write renders new;
        | PLAN_UPSTREAM_DOWNSTREAM: pairs are (A upstream, B downstream), spec writes render A;
        | PLAN_SPEC / PLAN_STATUS: only those writes (neither: both)."""
        wp = WritePlanC()
        _chk(_lib.gpudiff_write_plan_get_ex(self.ctx, ticket, mode, C.byref(wp)), "gpudiff_write_plan_get_ex")
        try:
            n = wp.n
            b = wp.bodies
            offs = np.ctypeslib.as_array(C.cast(b.offsets, C.POINTER(C.c_uint64)), (n + 1,)).copy()
            st = _arr(b.status, n, np.int32)
            src = _arr(b.source, n, np.uint8)
            total = int(offs[-1]) if n else 0
            raw = C.string_at(b.bytes, total) if total else b""
            return WritePlan(pair_index=_arr(wp.pair_index, n, np.uint32), kind=_arr(wp.kind, n, np.uint8),
                             noop=_arr(wp.noop, n, np.uint8),
                             bodies=[None if st[i] != OK else raw[int(offs[i]):int(offs[i + 1])] for i in range(n)],
                             source=src, n_host=int(b.n_host))
        finally:
            _lib.gpudiff_write_plan_release(self.ctx, C.byref(wp))

    def diff_pairs(self, pairs, ids=None, clusters=None) -> DiffResult:
        return self.wait(self.submit(pairs, ids, clusters))

    def object_store(self, max_slots: int, space_bytes: int, max_events: int,
                     device_encode: bool = False) -> ObjectStore:
        return ObjectStore(self, max_slots, space_bytes, max_events, device_encode)

    # ---- object encoding (device-store format: blob + path table)
    def encode_objects(self, docs, seeds=None, out_cap: int = 0):
        """Kernel K0 over the documents: [(ObjInfo dict, blob bytes or None)]."""
        docs = [to_json_bytes(x) for x in docs]
        n = len(docs)
        bufs = [C.create_string_buffer(x, len(x)) if x else C.create_string_buffer(1) for x in docs]
        ptrs = (C.c_void_p * max(n, 1))(*[C.cast(b, C.c_void_p) for b in bufs])
        lens = (C.c_size_t * max(n, 1))(*[len(x) for x in docs])
        sd = (C.c_uint32 * max(n, 1))(*(list(seeds) if seeds is not None else [0] * n))
        cap = out_cap or sum(31 * len(x) + 352 for x in docs) + 16  # + a body and a table pad to 128 B each
        out = C.create_string_buffer(cap)
        info = (ObjInfo * max(n, 1))()
        _chk(_lib.gpudiff_encode_objects(self.ctx, ptrs, lens, sd, n, C.cast(out, C.c_void_p), cap, info),
             "gpudiff_encode_objects")
        raw = out.raw
        res = []
        for i in range(n):
            f = info[i]
            res.append((f.as_dict(), raw[f.off:f.off + f.bytes] if f.status == TOK_OK else None))
        return res

    # ---- write path: request bodies of dirty objects
    def upsert_bodies(self, docs, mode: int = UPSERT_SPEC):
        """Kernel K10 (host-completed) over the documents: BodyList."""
        wb = self.wbatch(docs, mode)
        try:
            wb.run()
            return wb.fetch()
        finally:
            wb.close()

    def wbatch(self, docs, mode: int = UPSERT_SPEC) -> "WBatch":
        return WBatch(self, docs, mode)

    # ---- Deployment splitter status roll-up
    def rollup_status(self, docs) -> "RollupResult":
        """Kernels K11 + K12 (host path for K11's deferrals) over cached Deployments."""
        rb = self.rbatch(docs)
        try:
            rb.run()
            return rb.fetch()
        finally:
            rb.close()

    def rbatch(self, docs) -> "RBatch":
        return RBatch(self, docs)

    # ---- API-negotiation update classifier
    def classify_updates(self, pairs, kinds=NEG_KIND_API) -> np.ndarray:
        """Kernels K13 + K14 (host path for K13's deferrals): one NEG_* action per (old or None, new) pair.
        kinds: one NEG_KIND_* for every pair, or a sequence with one per pair."""
        nb = self.nbatch(pairs, kinds)
        try:
            nb.run()
            return nb.fetch()
        finally:
            nb.close()

    def nbatch(self, pairs, kinds=NEG_KIND_API) -> "NBatch":
        return NBatch(self, pairs, kinds)

    def k0_profile(self, enable: bool = True):
        """K0 per-phase wall-clock ticks (100 MHz) summed over waves since the last call."""
        out = (C.c_uint64 * 8)()
        _chk(_lib.gpudiff_k0_profile(self.ctx, 1 if enable else 0, out), "gpudiff_k0_profile")
        return list(out)

    def k2_profile(self, dev_ptr: int, cap_waves: int):
        """Run K2's timeline build and record its per-wave timeline into device memory (12 u64 per wave); 0 stops
        recording and returns the context to the default build."""
        _chk(_lib.gpudiff_k2_profile(self.ctx, dev_ptr or None, cap_waves), "gpudiff_k2_profile")

    # ---- single pair drop-ins
    def spec_equal(self, old, new) -> bool:
        a, b = to_json_bytes(old), to_json_bytes(new)
        eq = C.c_int()
        rc = _lib.gpudiff_spec_equal(self.ctx, a, len(a), b, len(b), C.byref(eq))
        if rc not in (OK, E_DECODE):
            _chk(rc, "gpudiff_spec_equal")
        return bool(eq.value)

    def status_equal(self, old, new) -> bool:
        a, b = to_json_bytes(old), to_json_bytes(new)
        eq = C.c_int()
        rc = _lib.gpudiff_status_equal(self.ctx, a, len(a), b, len(b), C.byref(eq))
        if rc not in (OK, E_DECODE):
            _chk(rc, "gpudiff_status_equal")
        return bool(eq.value)


def _doc_arrays(docs):
    docs = [to_json_bytes(x) for x in docs]
    n = len(docs)
    bufs = [C.create_string_buffer(x, len(x)) if x else C.create_string_buffer(1) for x in docs]
    ptrs = (C.c_void_p * max(n, 1))(*[C.cast(b, C.c_void_p) for b in bufs])
    lens = (C.c_size_t * max(n, 1))(*[len(x) for x in docs])
    return docs, bufs, ptrs, lens


@dataclass
class WritePlan:
    """The writes of one diffed batch (gpudiff_write_plan): spec writes, then
    status writes, each rendered from the document the plan mode names (informer
    pairs: new); no-op writes carry no body."""
    pair_index: np.ndarray
    kind: np.ndarray               # UPSERT_SPEC / UPSERT_STATUS
    noop: np.ndarray
    bodies: List[Optional[bytes]]  # b"" for no-op writes, None = undecodable
    source: np.ndarray
    n_host: int


@dataclass
class BodyList:
    bodies: List[Optional[bytes]]  # None = Go decode error (no write)
    source: np.ndarray             # BODY_DEVICE / BODY_HOST
    k10_status: np.ndarray         # K10's TOK_* per document
    n_host: int


class WBatch:
    """Documents resident in HBM for K10 (gpudiff_wbatch_*)."""

    def __init__(self, eng: "Engine", docs, mode: int = UPSERT_SPEC):
        self.eng = eng
        self.docs, self._bufs, ptrs, lens = _doc_arrays(docs)
        h = C.c_void_p()
        _chk(_lib.gpudiff_wbatch_create(eng.ctx, ptrs, lens, len(self.docs), mode, C.byref(h)),
             "gpudiff_wbatch_create")
        self.h = h

    def run(self):
        _chk(_lib.gpudiff_wbatch_run(self.eng.ctx, self.h), "gpudiff_wbatch_run")

    def fetch(self) -> BodyList:
        b = Bodies()
        _chk(_lib.gpudiff_wbatch_fetch(self.eng.ctx, self.h, C.byref(b)), "gpudiff_wbatch_fetch")
        try:
            n = b.n
            offs = np.ctypeslib.as_array(C.cast(b.offsets, C.POINTER(C.c_uint64)), (n + 1,)).copy()
            st = np.ctypeslib.as_array(C.cast(b.status, C.POINTER(C.c_int32)), (max(n, 1),))[:n].copy()
            src = np.ctypeslib.as_array(C.cast(b.source, C.POINTER(C.c_uint8)), (max(n, 1),))[:n].copy()
            k10 = np.ctypeslib.as_array(C.cast(b.k10_status, C.POINTER(C.c_int32)), (max(n, 1),))[:n].copy()
            total = int(offs[-1]) if n else 0
            raw = C.string_at(b.bytes, total) if total else b""
            bodies = [None if st[i] != OK else raw[int(offs[i]):int(offs[i + 1])] for i in range(n)]
            return BodyList(bodies, src, k10, int(b.n_host))
        finally:
            _lib.gpudiff_bodies_release(self.eng.ctx, C.byref(b))

    def stats(self) -> WBatchStats:
        st = WBatchStats()
        _chk(_lib.gpudiff_wbatch_stats_get(self.h, C.byref(st)), "gpudiff_wbatch_stats_get")
        return st

    def close(self):
        if self.h:
            _lib.gpudiff_wbatch_free(self.eng.ctx, self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class RollupResult:
    """deployment.go:41-91 over a batch: per document its group (or ROLLUP_NONE /
    ROLLUP_DECODE); per group (ascending first_doc) the int32 status sums."""
    doc_group: np.ndarray          # int32 [n]
    first_doc: np.ndarray          # uint32 [groups]: others[0]
    n_members: np.ndarray          # uint32 [groups]
    sums: np.ndarray               # int32 [groups, 5]
    k11_status: np.ndarray         # K11's TOK_* per document
    n_host: int
    host_grouped: bool

    def as_dict(self):
        return {"doc_group": self.doc_group.tolist(),
                "groups": [{"first_doc": int(f), "n_members": int(m), "sums": [int(x) for x in s]}
                           for f, m, s in zip(self.first_doc, self.n_members, self.sums)]}


class RBatch:
    """Cached Deployments resident in HBM for K11/K12 (gpudiff_rbatch_*)."""

    def __init__(self, eng: "Engine", docs):
        self.eng = eng
        self.docs, self._bufs, ptrs, lens = _doc_arrays(docs)
        h = C.c_void_p()
        _chk(_lib.gpudiff_rbatch_create(eng.ctx, ptrs, lens, len(self.docs), C.byref(h)), "gpudiff_rbatch_create")
        self.h = h

    def run(self):
        _chk(_lib.gpudiff_rbatch_run(self.eng.ctx, self.h), "gpudiff_rbatch_run")

    def fetch(self) -> RollupResult:
        r = Rollup()
        _chk(_lib.gpudiff_rbatch_fetch(self.eng.ctx, self.h, C.byref(r)), "gpudiff_rbatch_fetch")
        try:
            n, g = r.n_docs, r.n_groups
            if n:
                dg = np.ctypeslib.as_array(C.cast(r.doc_group, C.POINTER(C.c_int32)), (n,)).copy()
                k11 = np.ctypeslib.as_array(C.cast(r.k11_status, C.POINTER(C.c_int32)), (n,)).copy()
            else:
                dg = np.zeros(0, np.int32)
                k11 = np.zeros(0, np.int32)
            if g:
                raw = np.frombuffer(C.string_at(r.groups, 32 * g), dtype=np.uint32).reshape(g, 8)
            else:
                raw = np.zeros((0, 8), np.uint32)
            return RollupResult(dg, raw[:, 0].copy(), raw[:, 1].copy(), raw[:, 2:7].view(np.int32).copy(), k11,
                                int(r.n_host), bool(r.host_grouped))
        finally:
            _lib.gpudiff_rollup_release(self.eng.ctx, C.byref(r))

    def stats(self) -> RBatchStats:
        st = RBatchStats()
        _chk(_lib.gpudiff_rbatch_stats_get(self.h, C.byref(st)), "gpudiff_rbatch_stats_get")
        return st

    def close(self):
        if self.h:
            _lib.gpudiff_rbatch_free(self.eng.ctx, self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _kinds_array(kinds, n):
    """NEG_KIND_* per pair as a uint8 array (kept alive by the caller), from one kind or a sequence"""
    if isinstance(kinds, (int, np.integer)):
        arr = np.full(max(n, 1), int(kinds), np.uint8)
    else:
        arr = np.ascontiguousarray(np.asarray(kinds, np.uint8))
        if arr.size != n:
            raise ValueError("kinds: %d entries for %d pairs" % (arr.size, n))
        if n == 0:
            arr = np.zeros(1, np.uint8)
    return arr


class NBatch:
    """(old, new) pairs of APIResourceImport / NegotiatedAPIResource / CustomResourceDefinition JSON resident
    in HBM for K13/K14 (gpudiff_nbatch_*); old None = no old object; kinds: NEG_KIND_* (one, or per pair)."""

    def __init__(self, eng: "Engine", pairs, kinds=None):
        if kinds is None:
            kinds = NEG_KIND_API
        self.eng = eng
        pairs = list(pairs)
        self.n = len(pairs)
        olds = [None if a is None else to_json_bytes(a) for a, _ in pairs]
        _, self._nb, nptrs, nlens = _doc_arrays([b for _, b in pairs])
        _, self._ob, optrs, olens = _doc_arrays([a if a is not None else b"" for a in olds])
        for i, a in enumerate(olds):
            if a is None:
                optrs[i] = None
        self._kinds = _kinds_array(kinds, self.n)
        h = C.c_void_p()
        _chk(_lib.gpudiff_nbatch_create_kinds(eng.ctx, self._kinds.ctypes.data, optrs, olens, nptrs, nlens, self.n,
                                              C.byref(h)), "gpudiff_nbatch_create_kinds")
        self.h = h

    def run(self):
        _chk(_lib.gpudiff_nbatch_run(self.eng.ctx, self.h), "gpudiff_nbatch_run")

    def fetch(self) -> np.ndarray:
        out = np.zeros(max(self.n, 1), np.int32)
        _chk(_lib.gpudiff_nbatch_fetch(self.eng.ctx, self.h, out.ctypes.data_as(C.POINTER(C.c_int32))),
             "gpudiff_nbatch_fetch")
        return out[:self.n]

    def stats(self) -> NBatchStats:
        st = NBatchStats()
        _chk(_lib.gpudiff_nbatch_stats_get(self.h, C.byref(st)), "gpudiff_nbatch_stats_get")
        return st

    def close(self):
        if self.h:
            _lib.gpudiff_nbatch_free(self.eng.ctx, self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def negotiate_pair_host(old, new, kind: int = None) -> int:
    """The classifier's host path (Go-exact) for one pair; old None = no old object; kind NEG_KIND_*."""
    a = None if old is None else to_json_bytes(old)
    b = to_json_bytes(new)
    act = C.c_int32()
    if kind is None:
        _chk(_lib.gpudiff_negotiate_pair_host(a, 0 if a is None else len(a), b, len(b), C.byref(act)),
             "gpudiff_negotiate_pair_host")
    else:
        _chk(_lib.gpudiff_negotiate_pair_host_kind(kind, a, 0 if a is None else len(a), b, len(b), C.byref(act)),
             "gpudiff_negotiate_pair_host_kind")
    return int(act.value)


class HostPairs:
    """(old, new) JSON pairs held in C memory for the classifier's host path
    (gpudiff_classify_updates_host); old None = no old object."""

    def __init__(self, pairs, kinds=None):
        pairs = list(pairs)
        self.n = len(pairs)
        self._kinds = None if kinds is None else _kinds_array(kinds, self.n)
        olds = [None if a is None else to_json_bytes(a) for a, _ in pairs]
        _, self._nb, self.nptrs, self.nlens = _doc_arrays([b for _, b in pairs])
        _, self._ob, self.optrs, self.olens = _doc_arrays([a if a is not None else b"" for a in olds])
        for i, a in enumerate(olds):
            if a is None:
                self.optrs[i] = None

    def classify(self, threads: int = 1) -> np.ndarray:
        out = np.zeros(max(self.n, 1), np.int32)
        if self._kinds is None:
            _chk(_lib.gpudiff_classify_updates_host(self.optrs, self.olens, self.nptrs, self.nlens, self.n, threads,
                                                    out.ctypes.data_as(C.POINTER(C.c_int32))),
                 "gpudiff_classify_updates_host")
        else:
            _chk(_lib.gpudiff_classify_updates_host_kinds(self._kinds.ctypes.data, self.optrs, self.olens, self.nptrs,
                                                          self.nlens, self.n, threads,
                                                          out.ctypes.data_as(C.POINTER(C.c_int32))),
                 "gpudiff_classify_updates_host_kinds")
        return out[:self.n]


def rollup_doc_host(doc):
    """The roll-up host path for one document: ([5 x int32], owned-by bytes or None), or None when Go
    cannot decode it."""
    b = to_json_bytes(doc)
    v = (C.c_int32 * 5)()
    n = C.c_size_t()
    buf = C.create_string_buffer(max(1, len(b)))
    rc = _lib.gpudiff_rollup_doc_host(b, len(b), v, C.cast(buf, C.c_void_p), len(b) + 1, C.byref(n))
    if rc == E_DECODE:
        return None
    if rc == E_CAPACITY:  # a decoded label never outgrows ~3x its JSON text
        buf = C.create_string_buffer(n.value)
        rc = _lib.gpudiff_rollup_doc_host(b, len(b), v, C.cast(buf, C.c_void_p), n.value, C.byref(n))
    _chk(rc, "gpudiff_rollup_doc_host")
    label = None if n.value == C.c_size_t(-1).value else buf.raw[:n.value]
    return list(v), label


def upsert_body_host(doc, mode: int = UPSERT_SPEC) -> Optional[bytes]:
    """The host path (Go-exact): the request body, or None on a Go decode error."""
    b = to_json_bytes(doc)
    n = C.c_size_t()
    rc = _lib.gpudiff_upsert_body_host(b, len(b), mode, None, 0, C.byref(n))
    if rc == E_DECODE:
        return None
    if rc not in (OK, E_CAPACITY):
        _chk(rc, "gpudiff_upsert_body_host")
    out = C.create_string_buffer(max(1, n.value))
    _chk(_lib.gpudiff_upsert_body_host(b, len(b), mode, C.cast(out, C.c_void_p), n.value, C.byref(n)),
         "gpudiff_upsert_body_host")
    return out.raw[:n.value]


def resolve_path(old, new, path_hash: int, path_kind: int, path_hash_bits: int = PATH_HASH_BITS) -> str:
    a, b = to_json_bytes(old), to_json_bytes(new)
    buf = C.create_string_buffer(4096)
    n = C.c_size_t()
    _chk(_lib.gpudiff_resolve_path(a, len(a), b, len(b), path_hash, path_kind, path_hash_bits, buf, 4096,
                                   C.byref(n)), "gpudiff_resolve_path")
    if n.value >= 4096:
        buf = C.create_string_buffer(n.value + 1)
        _chk(_lib.gpudiff_resolve_path(a, len(a), b, len(b), path_hash, path_kind, path_hash_bits, buf,
                                       n.value + 1, C.byref(n)), "gpudiff_resolve_path")
    return buf.value.decode("utf-8", "replace")


def encode_object_host(doc, seed: int = 0, path_hash_bits: int = PATH_HASH_BITS):
    """Host encoder (the Go-exact path) in the device-store format: (ObjInfo dict, blob bytes or None)."""
    b = to_json_bytes(doc)
    info = ObjInfo()
    _chk(_lib.gpudiff_encode_object_host(b, len(b), seed, path_hash_bits, None, 0, C.byref(info)),
         "gpudiff_encode_object_host")
    if info.status != TOK_OK:
        return info.as_dict(), None
    out = C.create_string_buffer(max(1, info.bytes))
    _chk(_lib.gpudiff_encode_object_host(b, len(b), seed, path_hash_bits, C.cast(out, C.c_void_p), info.bytes,
                                         C.byref(info)), "gpudiff_encode_object_host")
    return info.as_dict(), out.raw[:info.bytes]


# ------------------------------------------------------------------ decoding helpers (tests / tooling)

TAB_INDEX = 1 << 63
TAB_NONE = 0xFFFFFFFF


def decode_path_table(blob: bytes, info: dict):
    """Path table of a device-store blob (include/gpudiff_format.h) -> [(hash,
    parent hash, component)], component ('K', key bytes) or ('I', index), in
    table order; None for a blob stored without a valid table."""
    n = info["n_tab"]
    if n == TAB_NONE:
        return None
    base = blob_body(info["spec_l"], info["spec_ar"], info["stat_l"], info["stat_ar"])
    if not n:
        return []
    hs = np.frombuffer(blob, "<u8", n, base)
    phs = np.frombuffer(blob, "<u8", n, base + 8 * n)
    cs = np.frombuffer(blob, "<u8", n, base + 16 * n)
    keys = base + 24 * n
    out = []
    for h, ph, c in zip(hs.tolist(), phs.tolist(), cs.tolist()):
        if c & TAB_INDEX:
            comp = ("I", c & 0xFFFFFFFF)
        else:
            ko, kl = c & 0xFFFFFFFF, c >> 32
            comp = ("K", blob[keys + ko:keys + ko + kl])
        out.append((h, ph, comp))
    return out


def decode_segment(pool: bytes, off: int, L: int, arena: int):
    """Canonical segment -> list of (key, val, meta, value_bytes).  A long
    string's first 8 bytes sit in its value slot, its tail in the arena at a
    4-byte aligned offset (include/gpudiff_format.h)."""
    vals = np.frombuffer(pool, dtype="<u8", count=L, offset=off) if L else np.zeros(0, "<u8")
    keys = np.frombuffer(pool, dtype="<u4", count=L, offset=off + 8 * L) if L else np.zeros(0, "<u4")
    metas = np.frombuffer(pool, dtype="<u4", count=L, offset=off + 12 * L) if L else np.zeros(0, "<u4")
    head = 16 * L
    ar = off + head
    out = []
    for k, v, m in zip(keys.tolist(), vals.tolist(), metas.tolist()):
        tag, ln = m & 7, m >> 3
        if tag == 5 and ln > 8:
            vb = int(v).to_bytes(8, "little") + bytes(pool[ar:ar + ln - 8])
            ar += (ln - 8 + 3) & ~3
        elif tag == 5:
            vb = int(v).to_bytes(8, "little")[:ln]
        elif tag in (3, 4):
            vb = int(v).to_bytes(8, "little")
        else:
            vb = b""
        out.append((k, v, m, vb))
    assert ((ar - off - head + 15) & ~15) == arena, (ar, off, head, arena)
    return out


BLOB_ALIGN = 128  # GPUDIFF_BLOB_ALIGN


def blob_body(sl: int, sar: int, tl: int, tar: int) -> int:
    """Both segments zero padded to 128 B (gpudiff_blob_body): a store blob's path table starts here."""
    return (segment_bytes(sl, sar) + segment_bytes(tl, tar) + BLOB_ALIGN - 1) & ~(BLOB_ALIGN - 1)


def segment_bytes(L: int, arena: int) -> int:
    """vals u64 | keys u32 | metas u32 per leaf, then the arena (include/gpudiff_format.h)."""
    return 16 * L + arena

"""ctypes wrapper of oracle/_build/liboracle.so -- the C++ restatement of the
reference predicates (TEST INFRASTRUCTURE / CPU BASELINE ONLY)."""
import ctypes as C
import os

import numpy as np

from . import build as _build

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = _build.LIB if os.path.exists(_build.LIB) else _build.build()
        l = C.CDLL(path)
        l.oracle_load.restype = C.c_void_p
        l.oracle_load.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.POINTER(C.c_char_p),
                                  C.POINTER(C.c_size_t), C.c_size_t]
        l.oracle_free.restype = None
        l.oracle_free.argtypes = [C.c_void_p]
        l.oracle_tree_paths.restype = C.c_long
        l.oracle_tree_paths.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        l.oracle_tree_check.restype = C.c_long
        l.oracle_tree_check.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        l.oracle_csr_run.restype = C.c_double
        l.oracle_csr_run.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_double, C.c_void_p,
                                     C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
        l.oracle_csr_paths.restype = C.c_long
        l.oracle_csr_paths.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_size_t]
        l.oracle_decide.restype = C.c_double
        l.oracle_decide.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_double, C.POINTER(C.c_double)]
        l.oracle_docs_load.restype = C.c_void_p
        l.oracle_docs_load.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t]
        l.oracle_docs_free.restype = None
        l.oracle_docs_free.argtypes = [C.c_void_p]
        l.oracle_upsert_body.restype = C.c_long
        l.oracle_upsert_body.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_char_p, C.c_size_t]
        l.oracle_upsert_run.restype = C.c_double
        l.oracle_upsert_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.POINTER(C.c_double),
                                        C.POINTER(C.c_uint64)]
        l.oracle_rollup_load.restype = C.c_void_p
        l.oracle_rollup_load.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t]
        l.oracle_rollup_free.restype = None
        l.oracle_rollup_free.argtypes = [C.c_void_p]
        l.oracle_rollup_run.restype = C.c_int
        l.oracle_rollup_run.argtypes = [C.c_void_p, C.c_int, C.c_double, C.POINTER(C.c_double), C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t)]
        _lib = l
    return _lib


class DecodedPairs:
    """Pairs decoded once (untimed) into the oracle's Go-like value trees."""

    def __init__(self, pairs):
        n = len(pairs)
        self.n = n
        A = (C.c_char_p * n)(*[a for a, _ in pairs])
        B = (C.c_char_p * n)(*[b for _, b in pairs])
        AL = (C.c_size_t * n)(*[len(a) for a, _ in pairs])
        BL = (C.c_size_t * n)(*[len(b) for _, b in pairs])
        self.h = lib().oracle_load(A, AL, B, BL, n)

    def decide(self, threads=1, min_seconds=0.0):
        """-> (flags u8[n], sweeps, seconds)"""
        flags = np.zeros(self.n, dtype=np.uint8)
        sec = C.c_double()
        sweeps = lib().oracle_decide(self.h, flags.ctypes.data_as(C.c_void_p), threads, min_seconds,
                                     C.byref(sec))
        return flags, sweeps, sec.value

    def paths(self, seeds, cap=None):
        """Field-path diff over the decoded trees (checker, untimed): (offsets
        u32[n_dirty + 1], hashes u64, kinds u8) in gpudiff_result layout; pair i
        hashed under seeds[i] (the encoder's per-pair seed)."""
        seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
        cap = cap or max(1024, 64 * self.n)
        while True:
            offs = np.zeros(self.n + 1, np.uint32)
            hs = np.zeros(cap, np.uint64)
            ks = np.zeros(cap, np.uint8)
            m = lib().oracle_tree_paths(self.h, seeds.ctypes.data, offs.ctypes.data, hs.ctypes.data, ks.ctypes.data,
                                        cap)
            if m >= 0:
                flags, _, _ = self.decide()
                nd = int(np.count_nonzero(flags & 3))
                return offs[:nd + 1], hs[:m], ks[:m]
            cap *= 4

    def close(self):
        if self.h:
            lib().oracle_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DecodedDocs:
    """Documents decoded once (untimed) for the write-path restatement
    (DeepCopy + upsert transform + json.Marshal)."""

    def __init__(self, docs):
        n = len(docs)
        self.n = n
        D = (C.c_char_p * max(n, 1))(*docs)
        L = (C.c_size_t * max(n, 1))(*[len(d) for d in docs])
        self.h = lib().oracle_docs_load(D, L, n)

    def body(self, i, mode=0):
        n = lib().oracle_upsert_body(self.h, i, mode, None, 0)
        if n < 0:
            return None
        buf = C.create_string_buffer(n)
        lib().oracle_upsert_body(self.h, i, mode, buf, n)
        return buf.raw[:n]

    def run(self, mode=0, threads=1, min_seconds=0.0):
        """-> (sweeps, seconds, body bytes per sweep)"""
        sec = C.c_double()
        nb = C.c_uint64()
        sw = lib().oracle_upsert_run(self.h, mode, threads, min_seconds, C.byref(sec), C.byref(nb))
        return sw, sec.value, nb.value

    def close(self):
        if self.h:
            lib().oracle_docs_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RollupDocs:
    """Cached Deployments (JSON) for the roll-up restatement (oracle/rollup_ref.cpp):
    typed-field decode + group by owned-by + int32 sums, decode timed."""

    def __init__(self, docs):
        n = len(docs)
        self.n = n
        D = (C.c_char_p * max(n, 1))(*docs)
        L = (C.c_size_t * max(n, 1))(*[len(d) for d in docs])
        self.h = lib().oracle_rollup_load(D, L, n)

    def run(self, threads=1, min_seconds=0.0):
        """-> (sweeps, seconds, result dict like rollup_oracle.rollup without owned_by)"""
        n = self.n
        dg = np.zeros(max(n, 1), np.int32)
        first = np.zeros(max(n, 1), np.uint32)
        cnt = np.zeros(max(n, 1), np.uint32)
        sums = np.zeros(max(5 * n, 1), np.int32)
        ng = C.c_size_t()
        sec = C.c_double()
        sw = lib().oracle_rollup_run(self.h, threads, min_seconds, C.byref(sec), dg.ctypes.data, first.ctypes.data,
                                     cnt.ctypes.data, sums.ctypes.data, C.byref(ng))
        g = ng.value
        res = {"doc_group": dg[:n].tolist(),
               "groups": [{"first_doc": int(first[i]), "n_members": int(cnt[i]), "sums": sums[5 * i:5 * i + 5].tolist()}
                          for i in range(g)]}
        return sw, sec.value, res

    def close(self):
        if self.h:
            lib().oracle_rollup_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def tree_check(buf: np.ndarray, offs: np.ndarray, seeds: np.ndarray, threads: int = 16, cap: int = 0):
    """Decisions and changed paths of n pairs given as JSON (buf u8, offs u64[2n+1] as
    Population.json_range returns), by the tree-walk restatement with its own decoder: (flags u8[n],
    offsets u32[n_dirty + 1], hashes u64, kinds u8).  TEST INFRASTRUCTURE (tools/full_tree_check.py)."""
    n = (len(offs) - 1) // 2
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
    cap = cap or max(1024, 8 * n)
    while True:
        flags = np.zeros(max(n, 1), np.uint8)
        o = np.zeros(n + 1, np.uint32)
        hs = np.zeros(cap, np.uint64)
        ks = np.zeros(cap, np.uint8)
        m = lib().oracle_tree_check(buf.ctypes.data, offs.ctypes.data, n, seeds.ctypes.data, threads,
                                    flags.ctypes.data, o.ctypes.data, hs.ctypes.data, ks.ctypes.data, cap)
        if m >= 0:
            nd = int(np.count_nonzero(flags[:n] & 3))
            return flags[:n], o[:nd + 1], hs[:m], ks[:m]
        cap *= 4


class CsrPairs:
    """The build's canonical CSR encoding of a batch (a host batch's pool and
    rows) for the CPU merge over CSR ("cpu-csr", oracle/csr_ref.cpp)."""

    def __init__(self, pool: bytes, rows: np.ndarray):
        # bytes, or a u8 array (HostBatch.pool_view: pools over 2 GiB)
        pool = pool if isinstance(pool, np.ndarray) else np.frombuffer(pool, dtype=np.uint8)
        self.pool = pool if pool.size else np.zeros(16, np.uint8)
        self.rows = np.ascontiguousarray(rows)
        self.n = len(rows)

    def run(self, threads=1, min_seconds=0.0):
        """-> (flags u8[n], sweeps, seconds, paths per sweep); decisions and changed paths timed"""
        flags = np.zeros(max(self.n, 1), np.uint8)
        sec = C.c_double()
        npth = C.c_uint64()
        sw = lib().oracle_csr_run(self.pool.ctypes.data, self.rows.ctypes.data, self.n, threads, min_seconds,
                                  flags.ctypes.data, C.byref(sec), C.byref(npth))
        return flags[:self.n], sw, sec.value, npth.value

    def paths(self, cap=None):
        """-> (flags u8[n], offsets u32[n_dirty + 1], hashes u64, kinds u8)"""
        cap = cap or max(1024, 64 * self.n)
        while True:
            flags = np.zeros(max(self.n, 1), np.uint8)
            offs = np.zeros(self.n + 1, np.uint32)
            hs = np.zeros(cap, np.uint64)
            ks = np.zeros(cap, np.uint8)
            m = lib().oracle_csr_paths(self.pool.ctypes.data, self.rows.ctypes.data, self.n, flags.ctypes.data,
                                       offs.ctypes.data, hs.ctypes.data, ks.ctypes.data, cap)
            if m >= 0:
                nd = int(np.count_nonzero(flags[:self.n] & 3))
                return flags[:self.n], offs[:nd + 1], hs[:m], ks[:m]
            cap *= 4


def csr_paths_ptr(pool_ptr: int, rows: np.ndarray, threads: int = 8):
    """The CPU merge's changed-path CSR of a host batch read in place (pool_ptr = the batch's host pool,
    rows = its pair rows), split over threads (ctypes drops the GIL): (flags u8[n], offsets
    u32[n_dirty + 1], hashes u64, kinds u8) in gpudiff_result layout.  Checker only (bench.py's
    full-size path parity, untimed)."""
    from concurrent.futures import ThreadPoolExecutor
    rows = np.ascontiguousarray(rows)
    n = len(rows)
    T = max(1, min(threads, n // 4096 + 1))
    cuts = [n * t // T for t in range(T + 1)]

    def one(t):
        sub = rows[cuts[t]:cuts[t + 1]]
        m = len(sub)
        cap = max(1024, 16 * m)
        while True:
            flags = np.zeros(max(m, 1), np.uint8)
            offs = np.zeros(m + 1, np.uint32)
            hs = np.zeros(cap, np.uint64)
            ks = np.zeros(cap, np.uint8)
            k = lib().oracle_csr_paths(pool_ptr, sub.ctypes.data, m, flags.ctypes.data, offs.ctypes.data,
                                       hs.ctypes.data, ks.ctypes.data, cap)
            if k >= 0:
                nd = int(np.count_nonzero(flags[:m] & 3))
                return flags[:m], offs[:nd + 1], hs[:k], ks[:k]
            cap *= 4
    with ThreadPoolExecutor(T) as ex:
        parts = list(ex.map(one, range(T)))
    flags = np.concatenate([p[0] for p in parts]) if n else np.zeros(0, np.uint8)
    offs, base = [np.zeros(1, np.uint64)], 0
    for p in parts:
        offs.append(p[1][1:].astype(np.uint64) + base)
        base += int(p[1][-1])
    return (flags, np.concatenate(offs), np.concatenate([p[2] for p in parts]),
            np.concatenate([p[3] for p in parts]))

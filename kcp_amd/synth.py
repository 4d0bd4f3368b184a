"""ctypes binding of libgpudiff_synth.so (include/gpudiff_synth.h): seeded
synthetic populations for bench.py and tests.  Not part of the drop-in."""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import gpudiff as G

_HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH_PATH = os.path.join(_HERE, "libgpudiff_synth.so")

SPEC_MUT, STATUS_MUT, B_HAS_STATUS = 0x1, 0x2, 0x4


class SynthCfg(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_pairs", C.c_uint64), ("n_clusters", C.c_uint32),
                ("mutate_frac", C.c_float), ("w_configmap", C.c_float), ("w_secret", C.c_float),
                ("w_deployment", C.c_float), ("w_crd", C.c_float), ("w_deep", C.c_float),
                ("crd_leaves", C.c_uint32)]


_P = C.c_void_p
_SIGS = [
    ("gpudiff_synth_open", C.c_int, [C.POINTER(SynthCfg), C.c_int, C.c_int, C.POINTER(_P)]),
    ("gpudiff_synth_open_ex", C.c_int, [C.POINTER(SynthCfg), C.c_int, C.c_int, C.c_void_p, C.POINTER(_P)]),
    ("gpudiff_synth_build_id", C.c_char_p, []),
    ("gpudiff_synth_cluster_sizes", C.c_int, [C.POINTER(SynthCfg), C.c_void_p]),
    ("gpudiff_synth_cluster_bytes", C.c_int, [C.POINTER(SynthCfg), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]),
    ("gpudiff_synth_local_ids", C.c_int, [_P, C.c_void_p]),
    ("gpudiff_synth_close", None, [_P]),
    ("gpudiff_synth_local_pairs", C.c_uint64, [_P]),
    ("gpudiff_synth_local_clusters", C.c_uint64, [_P]),
    ("gpudiff_synth_global_index", C.c_uint64, [_P, C.c_uint64]),
    ("gpudiff_synth_encode", C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint32, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint64)]),
    ("gpudiff_synth_copy_out", C.c_int, [_P, _P, _P, _P]),
    ("gpudiff_synth_json_range", C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint32, C.POINTER(_P), _P, _P]),
    ("gpudiff_synth_free_buf", None, [_P]),
    ("gpudiff_synth_json", C.c_int, [_P, C.c_uint64, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t), C.c_char_p,
                                     C.c_size_t, C.POINTER(C.c_size_t)]),
]

from . import _hiprt  # noqa: E402

_hiprt.preload()
_lib = C.CDLL(SYNTH_PATH)
for _n, _r, _a in _SIGS:
    getattr(_lib, _n).restype = _r
    getattr(_lib, _n).argtypes = _a
# the generator must come from the same sources as the engine it feeds (kcp_amd/buildinfo.py)
from .gpudiff import BUILD_ID as _ENGINE_BUILD_ID  # noqa: E402

if _lib.gpudiff_synth_build_id().decode() != _ENGINE_BUILD_ID:
    raise ImportError("%s has build ID %s, libgpudiff.so %s: rebuild with kcp_amd/build.py"
                      % (SYNTH_PATH, _lib.gpudiff_synth_build_id().decode(), _ENGINE_BUILD_ID))

# SURVEY.md §8(d) populations
CONFIGS = {
    # name: (n_pairs, n_clusters, mix cm/secret/deploy/crd/deep, seed offset)
    "config1": (10_000, 1, (0, 0, 1, 0, 0), 1),
    "config2": (1_000_000, 10_000, (0.5, 0.5, 0, 0, 0), 2),
    "config3": (10_000_000, 100_000, (0.2, 0.2, 0.4, 0.2, 0), 3),
    "config4": (100_000, 1_000, (0, 0, 0, 0, 1), 4),
}
BASE_SEED = 20211004


def make_cfg(name: str, n_pairs: int = 0, n_clusters: int = 0, mutate_frac: float = 0.05) -> SynthCfg:
    n, c, mix, off = CONFIGS[name]
    return SynthCfg(seed=BASE_SEED + off, n_pairs=n_pairs or n, n_clusters=n_clusters or c,
                    mutate_frac=mutate_frac, w_configmap=mix[0], w_secret=mix[1], w_deployment=mix[2],
                    w_crd=mix[3], w_deep=mix[4], crd_leaves=200)


@dataclass
class Chunk:
    hb: G.HostBatch
    truth: np.ndarray  # u8 ground-truth bits per pair
    pool_bytes: int
    leaves: int


def cluster_sizes(cfg: SynthCfg) -> np.ndarray:
    """Pairs per logical cluster of the population (u64 [n_clusters])."""
    out = np.zeros(cfg.n_clusters, dtype=np.uint64)
    if _lib.gpudiff_synth_cluster_sizes(C.byref(cfg), out.ctypes.data) != 0:
        raise RuntimeError("gpudiff_synth_cluster_sizes failed")
    return out


def cluster_bytes(cfg: SynthCfg, stride: int = 1, offset: int = 0, threads: int = 16) -> np.ndarray:
    """Exact Σ B_pair per logical cluster (u64 [n_clusters]) for the clusters c % stride == offset (zeros
    elsewhere): their pairs are encoded on the host and gpudiff_pair_compare_bytes summed by cluster.
    Ranks split the work (stride = world, offset = rank) and sum the vectors."""
    out = np.zeros(cfg.n_clusters, dtype=np.uint64)
    if _lib.gpudiff_synth_cluster_bytes(C.byref(cfg), stride, offset, threads, out.ctypes.data) != 0:
        raise RuntimeError("gpudiff_synth_cluster_bytes failed")
    return out


class Population:
    """One rank's shard (LPT by logical cluster) of a synthetic population: clusters packed by
    `cluster_weight` (Σ B_pair, `cluster_bytes`) or, if None, by pair count."""

    def __init__(self, cfg: SynthCfg, world: int = 1, rank: int = 0, cluster_weight=None):
        h = C.c_void_p()
        wt = None
        if cluster_weight is not None:
            wt = np.ascontiguousarray(cluster_weight, dtype=np.uint64)
            assert wt.size == cfg.n_clusters
        rc = _lib.gpudiff_synth_open_ex(C.byref(cfg), world, rank, None if wt is None else wt.ctypes.data,
                                        C.byref(h))
        if rc != 0:
            raise RuntimeError("gpudiff_synth_open failed (%d)" % rc)
        self.h = h
        self.cfg = cfg
        self.n = int(_lib.gpudiff_synth_local_pairs(h))
        self.n_clusters = int(_lib.gpudiff_synth_local_clusters(h))

    def close(self):
        if self.h:
            _lib.gpudiff_synth_close(self.h)
            self.h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def local_ids(self) -> np.ndarray:
        """Global pair index (= the pair_id the encoder writes) of every local pair, u32 [n]."""
        out = np.zeros(max(self.n, 1), dtype=np.uint32)
        if _lib.gpudiff_synth_local_ids(self.h, out.ctypes.data) != 0:
            raise RuntimeError("gpudiff_synth_local_ids failed")
        return out[:self.n]

    def global_index(self, i: int) -> int:
        return int(_lib.gpudiff_synth_global_index(self.h, i))

    def chunk(self, engine: G.Engine, first: int, n: int, threads: int = 16,
              reuse: "G.HostBatch | None" = None) -> Chunk:
        """Encodes local pairs [first, first+n) into a host batch (pinned on a
        GPU engine).  `reuse` recycles a staging batch (waits for its last H2D
        copy; reallocates only when it is too small)."""
        pb, lv = C.c_uint64(), C.c_uint64()
        rc = _lib.gpudiff_synth_encode(self.h, first, n, threads, C.byref(pb), C.byref(lv))
        if rc != 0:
            raise RuntimeError("gpudiff_synth_encode failed")
        pool = C.c_void_p()
        rows = C.c_void_p()
        if reuse is not None:
            G._chk(G._lib.gpudiff_hbatch_resize(engine.ctx, reuse.h, pb.value, n, lv.value, C.byref(pool),
                                                C.byref(rows)), "gpudiff_hbatch_resize")
            hb = reuse
        else:
            hbh = C.c_void_p()
            G._chk(G._lib.gpudiff_hbatch_create(engine.ctx, pb.value, n, lv.value, C.byref(hbh), C.byref(pool),
                                                C.byref(rows)), "gpudiff_hbatch_create")
            hb = G.HostBatch(engine, hbh.value, None)
        truth = np.zeros(n, dtype=np.uint8)
        _lib.gpudiff_synth_copy_out(self.h, pool, rows, truth.ctypes.data_as(C.c_void_p))
        return Chunk(hb, truth, pb.value, lv.value)

    def json_range(self, first: int, n: int, threads: int = 16):
        """JSON of local pairs [first, first+n) in one buffer: (u8 buffer, u64
        offsets [2n+1] with A_i at [offs[2i], offs[2i+1]) and B_i after it,
        u8 ground-truth bits [n])."""
        offs = np.zeros(2 * n + 1, dtype=np.uint64)
        truth = np.zeros(max(n, 1), dtype=np.uint8)
        p = C.c_void_p()
        rc = _lib.gpudiff_synth_json_range(self.h, first, n, threads, C.byref(p), offs.ctypes.data,
                                           truth.ctypes.data)
        if rc != 0:
            raise RuntimeError("gpudiff_synth_json_range failed (%d)" % rc)
        try:
            total = int(offs[-1])
            buf = np.empty(max(total, 1), dtype=np.uint8)
            if total:
                C.memmove(buf.ctypes.data, p, total)
        finally:
            _lib.gpudiff_synth_free_buf(p)
        return buf, offs, truth[:n]

    def json_pair(self, i: int):
        al, bl = C.c_size_t(), C.c_size_t()
        _lib.gpudiff_synth_json(self.h, i, None, 0, C.byref(al), None, 0, C.byref(bl))
        a = C.create_string_buffer(al.value + 1)
        b = C.create_string_buffer(bl.value + 1)
        rc = _lib.gpudiff_synth_json(self.h, i, a, al.value + 1, C.byref(al), b, bl.value + 1, C.byref(bl))
        if rc != 0:
            raise RuntimeError("gpudiff_synth_json failed")
        return a.raw[:al.value], b.raw[:bl.value]

    def expected_flags(self, truth: np.ndarray) -> np.ndarray:
        """Ground-truth decision bits: spec dirty iff a spec mutation was
        applied; status dirty iff B has no status key (statussyncer.go:22-26)
        or a status mutation was applied."""
        f = np.zeros(truth.shape, dtype=np.uint8)
        f |= np.where(truth & SPEC_MUT, G.SPEC_DIRTY, 0).astype(np.uint8)
        st = ((truth & STATUS_MUT) != 0) | ((truth & B_HAS_STATUS) == 0)
        f |= np.where(st, G.STATUS_DIRTY, 0).astype(np.uint8)
        return f


# ------------------------------------------------------------------ roll-up population

_DEP_TMPL = ('{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"annotations":{"deployment.kubernetes.io/'
             'revision":"1"},"clusterName":"%s","creationTimestamp":"2021-10-04T15:09:37Z","generation":%d,'
             '"labels":{%s},"name":"%s","namespace":"%s","resourceVersion":"%d","uid":"%08x-5ac9-4f5e-9d3e-'
             '%012x"},"spec":{"progressDeadlineSeconds":600,"replicas":%d,"revisionHistoryLimit":10,"selector":'
             '{"matchLabels":{"app":"%s"}},"strategy":{"rollingUpdate":{"maxSurge":"25%%","maxUnavailable":"25%%"},'
             '"type":"RollingUpdate"},"template":{"metadata":{"creationTimestamp":null,"labels":{"app":"%s"}},'
             '"spec":{"containers":[{"image":"quay.io/kcp-dev/%s:v%d","imagePullPolicy":"IfNotPresent","name":'
             '"%s","resources":{},"terminationMessagePath":"/dev/termination-log","terminationMessagePolicy":'
             '"File"}],"dnsPolicy":"ClusterFirst","restartPolicy":"Always","schedulerName":"default-scheduler",'
             '"securityContext":{},"terminationGracePeriodSeconds":30}}},"status":{"availableReplicas":%d,'
             '"conditions":[{"lastTransitionTime":"2021-10-04T15:09:51Z","lastUpdateTime":"2021-10-04T15:09:51Z",'
             '"message":"Deployment has minimum availability.","reason":"MinimumReplicasAvailable","status":"True",'
             '"type":"Available"},{"lastTransitionTime":"2021-10-04T15:09:37Z","lastUpdateTime":'
             '"2021-10-04T15:09:51Z","message":"ReplicaSet \\"%s-66b6c48dd5\\" has successfully progressed.",'
             '"reason":"NewReplicaSetAvailable","status":"True","type":"Progressing"}],"observedGeneration":%d,'
             '"readyReplicas":%d,"replicas":%d,"unavailableReplicas":%d,"updatedReplicas":%d}}')


def rollup_population(n_roots: int, leaves_per_root: int = 4, seed: int = 20211004 + 6, shuffle: bool = True):
    """Cached Deployments as the splitter's informer holds them: per root one
    Deployment without an owned-by label and `leaves_per_root` leaves labelled
    kcp.dev/cluster=<cluster>, kcp.dev/owned-by=<root> (deployment.go:127-160),
    with seeded status counters; API-server JSON (sorted keys, no whitespace).
    Returns (docs, roots): roots[i] = index of root i's own document."""
    rng = np.random.default_rng(seed)
    n = n_roots * (1 + leaves_per_root)
    st = rng.integers(0, 50, size=(n, 5)).tolist()
    order = rng.permutation(n).tolist() if shuffle else list(range(n))
    docs = [b""] * n
    roots = [0] * n_roots
    k = 0
    for r in range(n_roots):
        name = "web-%07d" % r
        ns = "ns-%04d" % (r % 997)
        lc = "lc-%05d" % (r % 100000)
        for j in range(1 + leaves_per_root):
            idx = order[k]
            s = st[k]
            k += 1
            if j == 0:
                labels = '"app":"%s"' % name
                dname = name
                roots[r] = idx
            else:
                labels = '"app":"%s","kcp.dev/cluster":"cluster-%d","kcp.dev/owned-by":"%s"' % (name, j, name)
                dname = "%s--cluster-%d" % (name, j)
            docs[idx] = (_DEP_TMPL % (lc, 1 + (r & 3), labels, dname, ns, 1000 + idx, idx, r, s[0], name, name,
                                      name, 1 + (r & 7), name, s[3], name, 1 + (r & 3), s[2], s[0], s[4],
                                      s[1])).encode()
    return docs, roots


def negotiate_population(n_pairs: int, seed: int = 20211004 + 7, variants: bool = True):
    """(old, new) Update pairs of APIResourceImport / NegotiatedAPIResource JSON
    for the API-negotiation classifier (pkg/reconciler/apiresource/controller.go:
    238-295), API-server shaped (~1.3 KB: metadata with the kcp labels, a spec
    with the columnDefinitions of a CommonAPIResourceSpec, 1-3 status
    conditions).  Event mix: 15% resync (same resourceVersion), 20% generation
    bump, 25% status change (condition status / reason / time / added), 15%
    annotation change, 15% label change only, 10% nothing but resourceVersion.
    With `variants`, 2% of the new objects carry a condition time written in
    another zone (the same instant) and 0.5% a fold-case metadata key (a
    document the device leaves to the host path).  Returns (pairs, expected
    actions as designed by the generator)."""
    rng = np.random.default_rng(seed)
    kinds = ("APIResourceImport", "NegotiatedAPIResource")
    cols = ",".join('{"name":"%s","type":"string","format":"","description":"%s column","priority":0,'
                    '"jsonPath":".spec.%s"}' % (c, c, c) for c in ("Ready", "Phase", "Location", "Age"))

    def doc(kind, name, rv, gen, labels, ann, conds, meta_key="metadata"):
        lab = ",".join('"%s":"%s"' % kv for kv in labels)
        an = ",".join('"%s":"%s"' % kv for kv in ann)
        cs = ",".join('{"type":"%s","status":"%s","lastTransitionTime":"%s","reason":"%s","message":"%s"}' % c
                      for c in conds)
        return ('{"apiVersion":"apiresource.kcp.dev/v1alpha1","kind":"%s","%s":{"name":"%s","clusterName":"admin",'
                '"uid":"5f0c%08x-8d1e-4c1b-9a61-0d1f2e3c4b5a","resourceVersion":"%d","generation":%d,'
                '"creationTimestamp":"2021-10-04T15:09:37Z","labels":{%s},"annotations":{%s}},'
                '"spec":{"groupVersion":{"group":"apps","version":"v1"},"plural":"%ss","singular":"%s",'
                '"kind":"Widget","scope":"Namespaced","location":"us-east1","schemaUpdateStrategy":"UpdateUnpublished",'
                '"columnDefinitions":[%s]},"status":{"conditions":[%s]}}' % (
                    kind, meta_key, name, rv & 0xFFFFFFFF, rv, gen, lab, an, name, name, cols, cs)).encode()

    pairs, want = [], []
    u = rng.random(n_pairs)
    v = rng.random(n_pairs)
    for i in range(n_pairs):
        kind = kinds[i & 1]
        name = "widget%07d" % i
        rv = 1000 + 7 * i
        gen = 1 + (i % 5)
        labels = [("kcp.dev/cluster", "lc-%05d" % (i % 10000)), ("app", "w%d" % (i % 97))]
        ann = [("kcp.dev/schema", "v%d" % (i % 3))]
        ts = "2021-10-%02dT%02d:%02d:%02dZ" % (1 + i % 28, i % 24, i % 60, (7 * i) % 60)
        conds = [("Compatible", "True", ts, "Compatible", "schema is compatible")]
        if i % 3:
            conds.append(("Available", "True", ts, "Published", "negotiated"))
        old = doc(kind, name, rv, gen, labels, ann, conds)
        x = u[i]
        nrv, ngen, nlab, nann, ncond = rv + 1, gen, labels, ann, list(conds)
        if x < 0.15:
            nrv, exp = rv, 0
        elif x < 0.35:
            ngen, exp = gen + 1, 1
        elif x < 0.60:
            c = ncond[0]
            y = v[i]
            if y < 0.4:
                ncond[0] = (c[0], "False", c[2], "Incompatible", c[4])
            elif y < 0.7:
                ncond[0] = (c[0], c[1], "2021-11-01T00:00:00Z", c[3], c[4])
            else:
                ncond.append(("Enforced", "True", ts, "Enforced", "enforced"))
            exp = 2
        elif x < 0.75:
            nann, exp = [("kcp.dev/schema", "v%d" % (i % 3 + 10))], 3
        elif x < 0.90:
            nlab, exp = labels[:1] + [("app", "moved")], 0   # the missing `!`: differing labels are ignored
        else:
            exp = 3                                           # equal labels: AnnotationOrLabelsOnlyChanged
        meta_key = "metadata"
        if variants and exp in (0, 3) and nrv != rv:
            y = v[i]
            if y < 0.02:  # the same instant, another zone
                c = ncond[0]
                hh = int(c[2][11:13])
                day = int(c[2][8:10])
                ncond[0] = (c[0], c[1], "2021-10-%02dT%02d:%s+01:00" % (day + (hh + 1) // 24, (hh + 1) % 24, c[2][14:19]),
                            c[3], c[4])
            elif y > 0.995:
                meta_key = "Metadata"
        new = doc(kind, name, nrv, ngen, nlab, nann, ncond, meta_key)
        pairs.append((old, new))
        want.append(exp)
    return pairs, np.asarray(want, np.int32)


def crd_population(n_pairs: int, seed: int = 20211004 + 8, n_props: int = 12):
    """(old, new) Update pairs of CustomResourceDefinition JSON (kind
    GPUDIFF_NEG_KIND_CRD; the third kind of controller.go:186-199), API-server
    shaped: metadata with kcp labels, a spec with one served version whose
    openAPIV3Schema has `n_props` properties (~3 KB at the default), status
    {conditions: NamesAccepted + Established, acceptedNames {plural, singular,
    kind, listKind, shortNames?, categories?}, storedVersions}.  Event mix: 15%
    resync, 20% generation bump (a schema edit), 25% status change (a condition,
    an accepted name, a short name / category added, a stored version
    appended), 15% annotation change, 15% label change only, 10% nothing but
    resourceVersion.  Returns (pairs, expected actions as designed)."""
    rng = np.random.default_rng(seed)

    def doc(name, rv, gen, labels, ann, conds, names, stored, nprops):
        lab = ",".join('"%s":"%s"' % kv for kv in labels)
        an = ",".join('"%s":"%s"' % kv for kv in ann)
        cs = ",".join('{"type":"%s","status":"%s","lastTransitionTime":"%s","reason":"%s","message":"%s"}' % c
                      for c in conds)
        props = ",".join('"field%02d":{"type":"string","description":"field %d of %s","maxLength":%d}'
                         % (k, k, name, 64 + k) for k in range(nprops))
        nm = '"plural":"%s","singular":"%s","kind":"%s","listKind":"%sList"' % (
            names["plural"], names["singular"], names["kind"], names["kind"])
        if names.get("shortNames") is not None:
            nm += ',"shortNames":[%s]' % ",".join('"%s"' % x for x in names["shortNames"])
        if names.get("categories") is not None:
            nm += ',"categories":[%s]' % ",".join('"%s"' % x for x in names["categories"])
        sv = ",".join('"%s"' % v for v in stored)
        return ('{"apiVersion":"apiextensions.k8s.io/v1","kind":"CustomResourceDefinition","metadata":{"name":'
                '"%ss.example.dev","clusterName":"admin","uid":"7a1c%08x-8d1e-4c1b-9a61-0d1f2e3c4b5a",'
                '"resourceVersion":"%d","generation":%d,"creationTimestamp":"2021-10-04T15:09:37Z","labels":{%s},'
                '"annotations":{%s}},"spec":{"group":"example.dev","names":{%s},"scope":"Namespaced","versions":'
                '[{"name":"v1","served":true,"storage":true,"schema":{"openAPIV3Schema":{"type":"object",'
                '"properties":{"spec":{"type":"object","properties":{%s}},"status":{"type":"object",'
                '"x-kubernetes-preserve-unknown-fields":true}}}},"subresources":{"status":{}}}],'
                '"conversion":{"strategy":"None"}},"status":{"conditions":[%s],"acceptedNames":{%s},'
                '"storedVersions":[%s]}}' % (name, rv & 0xFFFFFFFF, rv, gen, lab, an, nm, props, cs, nm, sv)).encode()

    pairs, want = [], []
    u = rng.random(n_pairs)
    v = rng.random(n_pairs)
    for i in range(n_pairs):
        name = "widget%07d" % i
        rv = 5000 + 11 * i
        gen = 1 + (i % 4)
        labels = [("kcp.dev/cluster", "lc-%05d" % (i % 10000)), ("app", "w%d" % (i % 97))]
        ann = [("kcp.dev/schema", "v%d" % (i % 3))]
        ts = "2021-10-%02dT%02d:%02d:%02dZ" % (1 + i % 28, i % 24, i % 60, (7 * i) % 60)
        conds = [("NamesAccepted", "True", ts, "NoConflicts", "no conflicts found"),
                 ("Established", "True", ts, "InitialNamesAccepted", "the initial names have been accepted")]
        names = {"plural": name + "s", "singular": name, "kind": "W%07d" % i}
        if i % 3 == 0:
            names["shortNames"] = ["w%d" % i]
        if i % 5 == 0:
            names["categories"] = ["all"]
        stored = ["v1"] if i % 4 else ["v1beta1", "v1"]
        nprops = n_props
        old = doc(name, rv, gen, labels, ann, conds, names, stored, nprops)
        x = u[i]
        nrv, ngen, nlab, nann, ncond, nnames, nstored = rv + 1, gen, labels, ann, list(conds), dict(names), stored
        if x < 0.15:
            nrv, exp = rv, 0
        elif x < 0.35:
            ngen, nprops, exp = gen + 1, n_props + 1, 1
        elif x < 0.60:
            y = v[i]
            if y < 0.3:
                c = ncond[1]
                ncond[1] = (c[0], "False", "2021-11-01T00:00:00Z", "Terminating", "the object is being deleted")
            elif y < 0.5:
                nnames["kind"] = "X%07d" % i
            elif y < 0.7:
                nnames["shortNames"] = list(names.get("shortNames") or []) + ["x%d" % i]
            elif y < 0.85:
                nnames["categories"] = list(names.get("categories") or []) + ["kcp"]
            else:
                nstored = stored + ["v2"]
            exp = 2
        elif x < 0.75:
            nann, exp = [("kcp.dev/schema", "v%d" % (i % 3 + 10))], 3
        elif x < 0.90:
            nlab, exp = labels[:1] + [("app", "moved")], 0   # the missing `!`: differing labels are ignored
        else:
            exp = 3                                           # equal labels: AnnotationOrLabelsOnlyChanged
        new = doc(name, nrv, ngen, nlab, nann, ncond, nnames, nstored, nprops)
        pairs.append((old, new))
        want.append(exp)
    return pairs, np.asarray(want, np.int32)

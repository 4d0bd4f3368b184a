"""Seeded synthetic object populations (small scale, pure Python) shaped like
SURVEY.md §8(d) configs 1-4: Deployments (contrib/examples/deployment.yaml
shape), ConfigMaps/Secrets, medium and deep CRDs.  B = A with the metadata the
predicates ignore rewritten, plus seeded mutations on a fraction of pairs."""
import base64
import copy
import json
import random

from tests.golden.kat_cases import BASE, J

SEED = 20211004


def _s(rnd, lo, hi, alphabet="abcdefghijklmnopqrstuvwxyz0123456789-"):
    return "".join(rnd.choice(alphabet) for _ in range(rnd.randint(lo, hi)))


def _meta(rnd, i, cluster, nlabels=4, nann=2):
    return {
        "name": "obj-%d" % i, "namespace": "ns-%d" % (i % 17),
        "uid": "%08x-0000-4000-8000-%012x" % (rnd.getrandbits(32), i),
        "resourceVersion": str(rnd.randint(1, 10 ** 7)),
        "creationTimestamp": "2021-10-04T15:09:37Z",
        "clusterName": "lc-%05d" % cluster,
        "labels": {"kcp.dev/cluster": "lc-%05d" % cluster,
                   **{"l%d" % k: _s(rnd, 1, 12) for k in range(nlabels - 1)}},
        "annotations": {"a%d" % k: _s(rnd, 4, 40) for k in range(nann)},
    }


def configmap(rnd, i, cluster, secret=False):
    data = {}
    for k in range(8):
        v = _s(rnd, 64, 512, "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 _-.")
        data[_s(rnd, 8, 24)] = base64.b64encode(v.encode()).decode() if secret else v
    o = {"apiVersion": "v1", "kind": "Secret" if secret else "ConfigMap", "metadata": _meta(rnd, i, cluster),
         "data": data}
    if secret:
        o["type"] = "Opaque"
    return o


def deployment(rnd, i, cluster):
    o = copy.deepcopy(BASE)
    o["metadata"] = _meta(rnd, i, cluster, 2, 1)
    o["spec"]["replicas"] = rnd.randint(1, 10)
    o["spec"]["template"]["spec"]["containers"][0]["image"] = "busybox:1.%d" % rnd.randint(20, 36)
    return o


def _crd_tree(rnd, depth, budget):
    if depth <= 0 or budget[0] <= 0 or rnd.random() < 0.25:
        budget[0] -= 1
        c = rnd.random()
        if c < 0.3:
            return rnd.randint(-1000, 10 ** 6)
        if c < 0.4:
            return rnd.random() * 100
        if c < 0.5:
            return rnd.random() < 0.5
        if c < 0.55:
            return None
        return _s(rnd, 0, 60)
    if rnd.random() < 0.5:
        return [_crd_tree(rnd, depth - 1, budget) for _ in range(rnd.randint(0, 5))]
    return {_s(rnd, 2, 10): _crd_tree(rnd, depth - 1, budget) for _ in range(rnd.randint(0, 5))}


def crd(rnd, i, cluster, leaves=200, depth=6):
    spec = {}
    budget = [leaves // 2]
    while budget[0] > 0:
        spec[_s(rnd, 3, 10)] = _crd_tree(rnd, depth, budget)
    conds = [{"type": "C%d" % k, "status": rnd.choice(["True", "False"]), "reason": _s(rnd, 5, 20),
              "lastTransitionTime": "2021-10-04T15:10:00Z", "observedGeneration": k}
             for k in range(max(1, leaves // 20))]
    return {"apiVersion": "example.kcp.dev/v1", "kind": "Widget", "metadata": _meta(rnd, i, cluster),
            "spec": spec, "status": {"conditions": conds, "phase": "Ready"}}


def _leaf_paths(x, path=()):
    if isinstance(x, dict) and x:
        for k, v in x.items():
            yield from _leaf_paths(v, path + (k,))
    elif isinstance(x, list) and x:
        for k, v in enumerate(x):
            yield from _leaf_paths(v, path + (k,))
    else:
        yield path


def _get(o, path):
    for p in path:
        o = o[p]
    return o


def mutate(rnd, o):
    """One semantic mutation (always changes spec or status)."""
    kind = o.get("kind")
    c = rnd.random()
    if kind in ("ConfigMap", "Secret"):
        if c < 0.70:
            k = rnd.choice(sorted(o["data"]))
            o["data"][k] = o["data"][k] + "x"
        elif c < 0.85:
            labs = o["metadata"]["labels"]
            if rnd.random() < 0.5 and len(labs) > 1:
                del labs[rnd.choice(sorted(k for k in labs if k != "kcp.dev/cluster"))]
            else:
                labs["new-%d" % rnd.randint(0, 99)] = "v"
        elif c < 0.95:
            o["metadata"]["annotations"]["a0"] += "!"
        else:
            if rnd.random() < 0.5:
                o["data"]["zz-added"] = "1"
            else:
                del o["data"][rnd.choice(sorted(o["data"]))]
        return o
    if kind == "Deployment":
        if c < 0.4:
            o["spec"]["replicas"] += 1
        elif c < 0.6:
            o["spec"]["template"]["spec"]["containers"][0]["image"] += "-rc"
        elif c < 0.8:
            o["status"]["readyReplicas"] = o["status"]["readyReplicas"] - 1
        elif c < 0.9:
            o["spec"]["replicas"] = float(o["spec"]["replicas"])  # int -> float retype
        else:
            o["status"]["conditions"].reverse()
        return o
    # CRD: list insert/delete mid-array, retype, value edit
    lists = [p for p in _leaf_paths(o["spec"])]
    arrs = []

    def find_lists(x, path=()):
        if isinstance(x, list) and len(x) >= 2:
            arrs.append(path)
        if isinstance(x, dict):
            for k, v in x.items():
                find_lists(v, path + (k,))
        elif isinstance(x, list):
            for k, v in enumerate(x):
                find_lists(v, path + (k,))

    find_lists(o["spec"])
    if c < 0.3 and arrs:
        a = _get(o["spec"], rnd.choice(arrs))
        if rnd.random() < 0.5:
            a.insert(len(a) // 2, "inserted")
        else:
            del a[len(a) // 2]
    elif c < 0.45:
        o["status"]["conditions"][0]["status"] = "Unknown"
    elif c < 0.55:
        o["status"]["conditions"].insert(1, {"type": "New", "status": "True"})
    else:
        p = rnd.choice(lists) if lists else None
        if p:
            parent = _get(o["spec"], p[:-1]) if len(p) > 1 else o["spec"]
            v = parent[p[-1]]
            if isinstance(v, bool) or v is None:
                parent[p[-1]] = "changed"
            elif isinstance(v, int):
                parent[p[-1]] = float(v) if rnd.random() < 0.5 else v + 1
            elif isinstance(v, float):
                parent[p[-1]] = v + 1.0
            elif isinstance(v, str):
                parent[p[-1]] = v + "~"
            else:
                parent[p[-1]] = 1
        else:
            o["spec"]["added"] = 1
    return o


def _noise(rnd, o):
    m = o.get("metadata")
    if isinstance(m, dict):
        m["uid"] = "ffffffff-0000-4000-8000-%012x" % rnd.getrandbits(40)
        m["resourceVersion"] = str(rnd.randint(1, 10 ** 7))
        m["managedFields"] = [{"manager": "syncer", "operation": "Update"}]
    return o


def make_pairs(n, seed=SEED, mix=(("cm", 0.25), ("secret", 0.25), ("deploy", 0.3), ("crd", 0.2)),
               mutate_frac=0.05, clusters=100, crd_leaves=200, pretty_frac=0.1):
    """Returns (pairs [(A_json, B_json)], cluster ids, mutated flags)."""
    rnd = random.Random(seed)
    kinds = [k for k, _ in mix]
    weights = [w for _, w in mix]
    pairs, cl, muts = [], [], []
    for i in range(n):
        c = rnd.randrange(clusters)
        k = rnd.choices(kinds, weights)[0]
        if k == "cm":
            a = configmap(rnd, i, c)
        elif k == "secret":
            a = configmap(rnd, i, c, True)
        elif k == "deploy":
            a = deployment(rnd, i, c)
        else:
            a = crd(rnd, i, c, crd_leaves)
        b = _noise(rnd, copy.deepcopy(a))
        m = rnd.random() < mutate_frac
        if m:
            b = mutate(rnd, b)
        aj = json.dumps(a, separators=(",", ":")).encode()
        bj = (json.dumps(b, indent=1, sort_keys=True) if rnd.random() < pretty_frac
              else json.dumps(b, separators=(",", ":"))).encode()
        pairs.append((aj, bj))
        cl.append(c)
        muts.append(m)
    return pairs, cl, muts


def deep_pairs(seed=41, n_pairs=24, sizes=(1500, 3000, 6000)):
    """Pairs whose joins cover thousands of keys: list inserts / deletes (every later index path
    changes), single value changes, key renames, status list inserts and equal pairs."""
    rnd = random.Random(seed)
    pairs = []
    for i in range(n_pairs):
        n = rnd.choice(sizes)
        a = {"apiVersion": "v1", "kind": "Deep", "metadata": {"name": "d%d" % i},
             "spec": {"items": ["v%05d-%s" % (j, "x" * (j % 13)) for j in range(n)],
                      "map": {"k%05d" % j: j for j in range(n // 2)}},
             "status": {"conds": [{"type": "C%d" % j, "ok": j % 2 == 0} for j in range(n // 4)]}}
        b = json.loads(json.dumps(a))
        op = i % 6
        if op == 0:
            b["spec"]["items"].insert(rnd.randrange(n), "inserted")
        elif op == 1:
            del b["spec"]["items"][rnd.randrange(n)]
        elif op == 2:
            b["spec"]["map"]["k%05d" % rnd.randrange(n // 2)] = -1
        elif op == 3:
            b["spec"]["map"]["znew"] = 1
            del b["spec"]["map"]["k00000"]
        elif op == 4:
            b["status"]["conds"].insert(3, {"type": "X"})
        pairs.append((J(a), J(b)))
    return pairs


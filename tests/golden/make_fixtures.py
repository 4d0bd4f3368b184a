#!/usr/bin/env python3
"""Generate the committed golden fixtures (SURVEY.md §8(c) "Golden vectors /
fixtures to commit" (ii)-(iii) and the per-config subsets).

Run in the build container (it reads /root/reference, which the GPU box does
not have); the outputs are data only:

  tests/golden/manifests.json.gz  pairs built from the reference's own data
        files -- contrib/examples/deployment.yaml (trailing space kept),
        contrib/demo/deployment.yaml, contrib/examples/pod.yaml and
        cluster.yaml, and ≤64 KB subtrees of contrib/crds/apps/apps_deployments.yaml
        as deep-object seeds -- each with seeded edits of the kinds the syncer
        sees (ignored metadata churn, spec/label/annotation edits, status
        changes, status removal, list insert/delete, int<->float retype).
  tests/golden/config{1,2,3,4}.json.gz  pairs sampled from the seeded
        synthetic populations bench.py runs (kcp_amd.synth), half of them
        mutated pairs.

Expected outputs come from the Python oracle (oracle/gpudiff_oracle.py):
the reference has no tests or expected outputs for this path (SURVEY.md
§8(c)), so these fixtures pin the oracle against regressions and give the
HIP path and the C++ restatement a fixed target; they are not an independent
check of the oracle (the KAT table is).

usage: python tests/golden/make_fixtures.py [--ref /root/reference]
"""
import argparse
import base64
import copy
import gzip
import json
import os
import random
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import gpudiff_oracle as O  # noqa: E402

FORMAT = 1


def J(obj) -> bytes:
    return json.dumps(obj, separators=(",", ":"), ensure_ascii=False).encode()


def expect(a: bytes, b: bytes) -> dict:
    r = O.diff_pair(a, b)
    return dict(spec_dirty=r["spec_dirty"], status_dirty=r["status_dirty"], decode_error=r["decode_error"],
                seed=r["seed"],
                paths=[["%016x" % h, kind | (0x80 if region else 0), O.render_path(p)]
                       for (h, region, kind, p) in r["paths"]])


def record(name: str, a: bytes, b: bytes) -> dict:
    return dict(name=name, a=base64.b64encode(a).decode(), b=base64.b64encode(b).decode(), expect=expect(a, b))


def write(path: str, source: str, pairs: list):
    doc = dict(format=FORMAT, source=source, generator="tests/golden/make_fixtures.py", n=len(pairs), pairs=pairs)
    with gzip.GzipFile(path, "wb", mtime=0) as f:
        f.write(json.dumps(doc, separators=(",", ":"), sort_keys=True).encode())
    print("wrote %s: %d pairs, %d bytes" % (os.path.relpath(path, ROOT), len(pairs), os.path.getsize(path)))


# ------------------------------------------------------------------ manifests
def load_yaml(ref, rel):
    with open(os.path.join(ref, rel)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def served(obj, cluster="us-east1", owner="example", rv="1001"):
    """What an informer cache holds for the manifest: server-set metadata and
    the kcp labels (pkg/reconciler/deployment/deployment.go:138-139)."""
    o = copy.deepcopy(obj)
    md = o.setdefault("metadata", {})
    md.setdefault("namespace", "default")
    md["uid"] = "6f1d2c3e-0000-4000-8000-%012d" % random.randrange(10 ** 12)
    md["resourceVersion"] = rv
    md["creationTimestamp"] = "2021-10-04T15:09:37Z"
    md["generation"] = 1
    md["clusterName"] = "admin"
    md.setdefault("labels", {}).update({"kcp.dev/cluster": cluster, "kcp.dev/owned-by": owner})
    return o


def churn(o):
    """Metadata the predicates ignore (specsyncer.go:30-35 skips metadata)."""
    o = copy.deepcopy(o)
    md = o["metadata"]
    md["uid"] = "0a0a0a0a-0000-4000-8000-000000000002"
    md["resourceVersion"] = str(int(md.get("resourceVersion", "1")) + 17)
    md["managedFields"] = [{"manager": "syncer", "operation": "Update", "apiVersion": o.get("apiVersion", "v1")}]
    md["creationTimestamp"] = "2021-10-05T00:00:00Z"
    return o


def deployment_status(replicas):
    return {"observedGeneration": 1, "replicas": replicas, "updatedReplicas": replicas,
            "readyReplicas": replicas, "availableReplicas": replicas,
            "conditions": [
                {"type": "Available", "status": "True", "reason": "MinimumReplicasAvailable",
                 "message": "Deployment has minimum availability.",
                 "lastUpdateTime": "2021-10-04T15:10:01Z", "lastTransitionTime": "2021-10-04T15:10:01Z"},
                {"type": "Progressing", "status": "True", "reason": "NewReplicaSetAvailable",
                 "message": "ReplicaSet \"example-5d59d67564\" has successfully progressed.",
                 "lastUpdateTime": "2021-10-04T15:10:01Z", "lastTransitionTime": "2021-10-04T15:09:37Z"}]}


def edits_for(o, rnd):
    """(name, new object) edits of one served object."""
    out = [("identical", copy.deepcopy(o)), ("metadata-churn", churn(o))]
    b = churn(o)
    b["metadata"]["labels"]["app"] = "edited"
    out.append(("label-add", b))
    b = churn(o)
    b["metadata"].setdefault("annotations", {})["kcp.dev/note"] = "x" * 40
    out.append(("annotation-add", b))
    b = churn(o)
    b["metadata"]["labels"]["kcp.dev/cluster"] = 7  # non-string label value: GetLabels -> nil
    out.append(("label-nonstring", b))
    if "spec" in o:
        b = churn(o)
        b["spec"]["kcpFixtureKey"] = None  # top-level null inside spec is a real leaf
        out.append(("spec-null-leaf", b))
        b = churn(o)
        del b["spec"]
        out.append(("spec-removed", b))
    if "status" in o:
        b = churn(o)
        del b["status"]
        out.append(("status-removed", b))
        b = churn(o)
        b["status"] = None
        out.append(("status-null", b))
    return out


def deployment_pairs(ref, rel, rnd):
    pairs = []
    for base in load_yaml(ref, rel):
        a = served(base)
        reps = a["spec"].get("replicas", 1)
        a["status"] = deployment_status(reps)
        for name, b in edits_for(a, rnd):
            pairs.append(record("%s:%s" % (rel, name), J(a), J(b)))
        b = churn(a)
        b["spec"]["replicas"] = reps + 1
        pairs.append(record("%s:replicas" % rel, J(a), J(b)))
        b = churn(a)
        b["spec"]["replicas"] = float(reps)  # int64 -> float64 retype: Semantic.DeepEqual false
        pairs.append(record("%s:replicas-float" % rel, J(a), J(b)))
        b = churn(a)
        c = b["spec"]["template"]["spec"]["containers"][0]
        c["image"] = c["image"] + "-patched"
        pairs.append(record("%s:image" % rel, J(a), J(b)))
        if "command" in c:
            b = churn(a)
            cc = b["spec"]["template"]["spec"]["containers"][0]["command"]
            cc[-1] = cc[-1].rstrip(" \n") + "\n"  # drop the trailing space of the literal block
            pairs.append(record("%s:command-trailing-space" % rel, J(a), J(b)))
            b = churn(a)
            b["spec"]["template"]["spec"]["containers"][0]["command"].insert(1, "-x")
            pairs.append(record("%s:command-insert" % rel, J(a), J(b)))
        b = churn(a)
        b["status"]["readyReplicas"] = reps - 1
        b["status"]["conditions"][0]["status"] = "False"
        pairs.append(record("%s:status-edit" % rel, J(a), J(b)))
        b = churn(a)
        b["status"]["conditions"].reverse()
        pairs.append(record("%s:conditions-reversed" % rel, J(a), J(b)))
        b = churn(a)
        b["status"]["conditions"] = []
        pairs.append(record("%s:conditions-empty" % rel, J(a), J(b)))
        # formatting of the old side's bytes never matters (decoded trees are compared)
        pairs.append(record("%s:pretty-printed-old" % rel, json.dumps(a, indent=2).encode(), J(churn(a))))
    return pairs


def plain_pairs(ref, rel, rnd):
    pairs = []
    for base in load_yaml(ref, rel):
        a = served(base)
        for name, b in edits_for(a, rnd):
            pairs.append(record("%s:%s" % (rel, name), J(a), J(b)))
    return pairs


def subtrees(node, path, out, lo, hi):
    """Collect dict subtrees whose JSON size is in [lo, hi] bytes."""
    if isinstance(node, dict):
        n = len(J(node))
        if lo <= n <= hi:
            out.append((path, node))
        for k, v in node.items():
            subtrees(v, path + (k,), out, lo, hi)
    elif isinstance(node, list):
        for i, v in enumerate(node):
            subtrees(v, path + (i,), out, lo, hi)


def leaf_paths(node, path=()):
    if isinstance(node, dict) and node:
        for k, v in node.items():
            yield from leaf_paths(v, path + (k,))
    elif isinstance(node, list) and node:
        for i, v in enumerate(node):
            yield from leaf_paths(v, path + (i,))
    else:
        yield path


def list_paths(node, path=()):
    if isinstance(node, list):
        if len(node) >= 3:
            yield path
        for i, v in enumerate(node):
            yield from list_paths(v, path + (i,))
    elif isinstance(node, dict):
        for k, v in node.items():
            yield from list_paths(v, path + (k,))


def get(node, path):
    for p in path:
        node = node[p]
    return node


def crd_pairs(ref, rel, rnd, count):
    crd = load_yaml(ref, rel)[0]
    found = []
    subtrees(crd, (), found, 8 << 10, 64 << 10)
    rnd.shuffle(found)
    pairs = []
    for k, (path, sub) in enumerate(found[:count]):
        a = served({"apiVersion": "fixtures.kcp.dev/v1", "kind": "SchemaSlice",
                    "metadata": {"name": "slice-%d" % k}, "spec": sub,
                    "status": {"source": "/".join(map(str, path)),
                               "items": [{"i": i, "ok": i % 3 == 0} for i in range(64)]}})
        leaves = [p for p in leaf_paths(a["spec"]) if p]
        for e in range(6):
            b = churn(a)
            kind = e % 6
            if kind == 0:  # one description / leaf edit deep inside
                p = rnd.choice(leaves)
                parent = get(b["spec"], p[:-1])
                v = parent[p[-1]]
                parent[p[-1]] = (v + " (edited)") if isinstance(v, str) else [v]
            elif kind == 1:  # list delete mid-array: every later index shifts
                lps = list(list_paths(b["spec"]))
                if lps:
                    lst = get(b["spec"], rnd.choice(lps))
                    del lst[len(lst) // 2]
            elif kind == 2:  # list insert at the front
                lps = list(list_paths(b["spec"]))
                if lps:
                    get(b["spec"], rnd.choice(lps)).insert(0, "inserted")
            elif kind == 3:  # status list shift
                del b["status"]["items"][5]
            elif kind == 4:  # status removed
                del b["status"]
            pairs.append(record("%s:%s:edit%d" % (rel, "/".join(map(str, path[-3:])), kind), J(a), J(b)))
    return pairs


# ------------------------------------------------------------------ synthetic configs
def config_pairs(name, n_clean, n_dirty, scan):
    from kcp_amd import synth as S
    pop = S.Population(S.make_cfg(name))
    n = pop.n
    clean, dirty = [], []
    step = max(1, n // scan)
    for i in range(0, n, step):
        a, b = pop.json_pair(i)
        r = O.diff_pair(a, b)
        spec_or_status_change = r["spec_dirty"] or any(k != O.KIND_STATUS_ABSENT for (_, _, k, _) in r["paths"])
        bucket = dirty if spec_or_status_change else clean
        want = n_dirty if bucket is dirty else n_clean
        if len(bucket) < want:
            bucket.append(dict(name="%s:%d" % (name, pop.global_index(i)),
                               a=base64.b64encode(a).decode(), b=base64.b64encode(b).decode(),
                               expect=dict(spec_dirty=r["spec_dirty"], status_dirty=r["status_dirty"],
                                           decode_error=r["decode_error"], seed=r["seed"],
                                           paths=[["%016x" % h, kind | (0x80 if region else 0), O.render_path(p)]
                                                  for (h, region, kind, p) in r["paths"]])))
        if len(clean) >= n_clean and len(dirty) >= n_dirty:
            break
    pop.close()
    return clean + dirty


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    rnd = random.Random(20211004)
    random.seed(20211004)
    todo = args.only.split(",") if args.only else ["manifests", "config1", "config2", "config3", "config4"]
    if "manifests" in todo:
        pairs = []
        pairs += deployment_pairs(args.ref, "contrib/examples/deployment.yaml", rnd)
        pairs += deployment_pairs(args.ref, "contrib/demo/deployment.yaml", rnd)
        pairs += plain_pairs(args.ref, "contrib/examples/pod.yaml", rnd)
        pairs += plain_pairs(args.ref, "contrib/examples/cluster.yaml", rnd)
        pairs += crd_pairs(args.ref, "contrib/crds/apps/apps_deployments.yaml", rnd, 6)
        write(os.path.join(HERE, "manifests.json.gz"),
              "reference data files contrib/examples/{deployment,pod,cluster}.yaml, contrib/demo/deployment.yaml, "
              "contrib/crds/apps/apps_deployments.yaml subtrees (8-64 KB), with seeded edits", pairs)
    sizes = {"config1": (100, 100, 4000), "config2": (100, 100, 8000), "config3": (100, 100, 8000),
             "config4": (15, 15, 1000)}
    for name in ("config1", "config2", "config3", "config4"):
        if name in todo:
            nc, nd, scan = sizes[name]
            write(os.path.join(HERE, "%s.json.gz" % name),
                  "kcp_amd.synth population %s (bench workload generator), evenly spaced sample, "
                  "%d unmutated + %d mutated pairs" % (name, nc, nd), config_pairs(name, nc, nd, scan))


if __name__ == "__main__":
    main()

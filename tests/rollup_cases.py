"""Known answers for the Deployment splitter's status roll-up fields
(pkg/reconciler/deployment/deployment.go:41-91), each stating what Go 1.16
encoding/json does when the splitter's informer decodes the document into an
appsv1.Deployment: the five status counters (replicas, updatedReplicas,
readyReplicas, availableReplicas, unavailableReplicas) and the
kcp.dev/owned-by label, or DECODE when the decode fails (the object never
reaches the cache).  Hand-written from the published encoding/json rules
(decode.go object()/literalStore(), fold.go); no reference run exists (no Go).
"""

DECODE = "decode"
O = "kcp.dev/owned-by"


def dep(labels=None, status=None, extra=""):
    import json
    md = {"name": "d", "namespace": "default"}
    if labels is not None:
        md["labels"] = labels
    o = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": md, "spec": {"replicas": 3}}
    if status is not None:
        o["status"] = status
    s = json.dumps(o, separators=(",", ":"))
    return (s[:-1] + extra + "}").encode() if extra else s.encode()


# (name, document bytes, expected: DECODE or (counters, owned-by str or None))
CASES = [
    ("plain leaf", dep({O: "root", "kcp.dev/cluster": "c1"},
                       {"replicas": 5, "updatedReplicas": 5, "readyReplicas": 4, "availableReplicas": 4,
                        "unavailableReplicas": 1}), ([5, 5, 4, 4, 1], "root")),
    ("root (no owned-by)", dep({"app": "x"}, {"replicas": 10}), ([10, 0, 0, 0, 0], None)),
    ("no labels, no status", dep(), ([0, 0, 0, 0, 0], None)),
    ("empty status", dep({O: "r"}, {}), ([0, 0, 0, 0, 0], "r")),
    ("status null (struct: no-op)", dep({O: "r"}, None, ',"status":null'), ([0, 0, 0, 0, 0], "r")),
    ("counter null (int32: no-op)", dep({O: "r"}, {"replicas": None, "readyReplicas": 2}), ([0, 0, 2, 0, 0], "r")),
    ("int32 max / min", dep({O: "r"}, {"replicas": 2147483647, "unavailableReplicas": -2147483648}),
     ([2147483647, 0, 0, 0, -2147483648], "r")),
    ("int32 overflow", dep({O: "r"}, {"replicas": 2147483648}), DECODE),
    ("int32 underflow", dep({O: "r"}, {"replicas": -2147483649}), DECODE),
    ("int64-sized literal", b'{"status":{"replicas":9223372036854775808}}', DECODE),
    ("float literal 3.0", b'{"status":{"replicas":3.0}}', DECODE),
    ("exponent literal 1e2", b'{"status":{"replicas":1e2}}', DECODE),
    ("negative zero", b'{"status":{"replicas":-0}}', ([0, 0, 0, 0, 0], None)),
    ("string counter", b'{"status":{"replicas":"3"}}', DECODE),
    ("bool counter", b'{"status":{"replicas":true}}', DECODE),
    ("object counter", b'{"status":{"replicas":{}}}', DECODE),
    ("status is a list", b'{"status":[]}', DECODE),
    ("status is a string", b'{"status":"x"}', DECODE),
    ("metadata is a list", b'{"metadata":[]}', DECODE),
    ("metadata null", b'{"metadata":null,"status":{"replicas":1}}', ([1, 0, 0, 0, 0], None)),
    ("labels null", b'{"metadata":{"labels":null}}', ([0, 0, 0, 0, 0], None)),
    ("labels empty", b'{"metadata":{"labels":{}}}', ([0, 0, 0, 0, 0], None)),
    ("labels is a list", b'{"metadata":{"labels":[]}}', DECODE),
    ("label value a number", b'{"metadata":{"labels":{"a":1,"kcp.dev/owned-by":"r"}}}', DECODE),
    ("label value null -> \"\"", b'{"metadata":{"labels":{"kcp.dev/owned-by":null}}}', ([0, 0, 0, 0, 0], "")),
    ("owned-by empty string", b'{"metadata":{"labels":{"kcp.dev/owned-by":""}}}', ([0, 0, 0, 0, 0], "")),
    ("owned-by escaped", b'{"metadata":{"labels":{"kcp.dev/owned-by":"r\\u00e9\\/x"}}}',
     ([0, 0, 0, 0, 0], "ré/x")),
    ("owned-by non-ASCII", '{"metadata":{"labels":{"kcp.dev/owned-by":"ré"}}}'.encode(),
     ([0, 0, 0, 0, 0], "ré")),
    ("owned-by invalid UTF-8 -> U+FFFD", b'{"metadata":{"labels":{"kcp.dev/owned-by":"r\xff"}}}',
     ([0, 0, 0, 0, 0], "r�")),
    ("owned-by lone surrogate -> U+FFFD", b'{"metadata":{"labels":{"kcp.dev/owned-by":"\\ud800x"}}}',
     ([0, 0, 0, 0, 0], "�x")),
    ("label key case matters (map)", b'{"metadata":{"labels":{"KCP.dev/owned-by":"r"}}}', ([0, 0, 0, 0, 0], None)),
    ("field names fold: Status/METADATA/Labels/REPLICAS",
     b'{"METADATA":{"Labels":{"kcp.dev/owned-by":"r"}},"Status":{"REPLICAS":2,"readyreplicas":1}}',
     ([2, 0, 1, 0, 0], "r")),
    ("long s folds to s", '{"statuſ":{"replicaſ":4}}'.encode(), ([4, 0, 0, 0, 0], None)),
    ("kelvin sign does not fold to s", '{"status":{"Keplicas":4}}'.encode(), ([0, 0, 0, 0, 0], None)),
    ("long s folds labels", '{"metadata":{"labelſ":{"kcp.dev/owned-by":"r"}}}'.encode(),
     ([0, 0, 0, 0, 0], "r")),
    ("repeated status merges", b'{"status":{"replicas":1,"readyReplicas":7},"status":{"replicas":2}}',
     ([2, 0, 7, 0, 0], None)),
    ("repeated counter last wins", b'{"status":{"replicas":1,"replicas":9}}', ([9, 0, 0, 0, 0], None)),
    ("status then Status merge", b'{"status":{"replicas":1},"Status":{"availableReplicas":3}}',
     ([1, 0, 0, 3, 0], None)),
    ("status, then null keeps", b'{"status":{"replicas":1},"status":null}', ([1, 0, 0, 0, 0], None)),
    ("repeated labels merge", b'{"metadata":{"labels":{"kcp.dev/owned-by":"a"},"labels":{"x":"y"}}}',
     ([0, 0, 0, 0, 0], "a")),
    ("repeated labels override", b'{"metadata":{"labels":{"kcp.dev/owned-by":"a"},"labels":{"kcp.dev/owned-by":"b"}}}',
     ([0, 0, 0, 0, 0], "b")),
    ("labels, then null clears", b'{"metadata":{"labels":{"kcp.dev/owned-by":"a"},"labels":null}}',
     ([0, 0, 0, 0, 0], None)),
    ("repeated metadata merges", b'{"metadata":{"labels":{"kcp.dev/owned-by":"a"}},"metadata":{"name":"n"}}',
     ([0, 0, 0, 0, 0], "a")),
    ("duplicate owned-by last wins", b'{"metadata":{"labels":{"kcp.dev/owned-by":"a","kcp.dev/owned-by":"b"}}}',
     ([0, 0, 0, 0, 0], "b")),
    ("other status fields ignored", b'{"status":{"observedGeneration":4,"conditions":[{"type":"Available"}],'
                                    b'"collisionCount":1,"replicas":2}}', ([2, 0, 0, 0, 0], None)),
    ("nested status not read", b'{"spec":{"status":{"replicas":5}}}', ([0, 0, 0, 0, 0], None)),
    ("whitespace", b' { "status" : { "replicas" : 3 } , "metadata" : { "labels" : { "kcp.dev/owned-by" : "r" } } } ',
     ([3, 0, 0, 0, 0], "r")),
    ("syntax error", b'{"status":{"replicas":3}', DECODE),
    ("trailing data", b'{"status":{}} x', DECODE),
    ("bad literal elsewhere", b'{"spec":{"paused":tru},"status":{}}', DECODE),
    ("leading zero elsewhere", b'{"spec":{"replicas":01}}', DECODE),
    ("bad escape elsewhere", b'{"spec":{"x":"\\q"}}', DECODE),
    ("control char in string", b'{"spec":{"x":"a\x01"}}', DECODE),
    ("top level not an object", b'[1]', DECODE),
    ("huge float elsewhere is fine (typed decode skips it)", b'{"spec":{"x":1e400},"status":{"replicas":1}}',
     ([1, 0, 0, 0, 0], None)),
]

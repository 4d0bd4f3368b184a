"""Known-answer table of SURVEY.md Appendix A.4 as concrete JSON pairs.

Each case is (name, A_json_bytes, B_json_bytes, expected_spec_equal,
expected_status_equal) where an expected value of None means "not pinned by
the table" (the oracle still computes it, and the HIP path must match the
oracle).  A = old/upstream, B = new/downstream.

The base object is contrib/examples/deployment.yaml:1-23 of the reference
(note the trailing newline of the literal block at :21-23) with the server
defaults a kube-apiserver adds and a two-condition status, written out here
as JSON (this is data, not reference source).
"""
import copy
import json

BASE = {
    "apiVersion": "apps/v1",
    "kind": "Deployment",
    "metadata": {
        "name": "example",
        "namespace": "default",
        "uid": "6f1d2c3e-0000-4000-8000-000000000001",
        "resourceVersion": "1001",
        "generation": 1,
        "creationTimestamp": "2021-10-04T15:09:37Z",
        "clusterName": "admin",
        "labels": {"kcp.dev/cluster": "us-east1", "kcp.dev/owned-by": "example"},
        "annotations": {"deployment.kubernetes.io/revision": "1"},
    },
    "spec": {
        "replicas": 3,
        "selector": {"matchLabels": {"app": "nginx"}},
        "template": {
            "metadata": {"labels": {"app": "nginx"}, "creationTimestamp": None},
            "spec": {
                "containers": [{
                    "name": "busybox",
                    "image": "busybox:1.25",
                    "command": ["/bin/sh", "-ec", "echo \"Going to sleep\"\ntail -f /dev/null\n"],
                    "resources": {},
                    "terminationMessagePath": "/dev/termination-log",
                    "terminationMessagePolicy": "File",
                    "imagePullPolicy": "IfNotPresent",
                }],
                "restartPolicy": "Always",
                "terminationGracePeriodSeconds": 30,
                "dnsPolicy": "ClusterFirst",
                "securityContext": {},
                "schedulerName": "default-scheduler",
            },
        },
        "strategy": {"type": "RollingUpdate",
                     "rollingUpdate": {"maxUnavailable": "25%", "maxSurge": "25%"}},
        "revisionHistoryLimit": 10,
        "progressDeadlineSeconds": 600,
    },
    "status": {
        "observedGeneration": 1,
        "replicas": 3,
        "updatedReplicas": 3,
        "readyReplicas": 3,
        "availableReplicas": 3,
        "conditions": [
            {"type": "Available", "status": "True", "reason": "MinimumReplicasAvailable",
             "message": "Deployment has minimum availability.",
             "lastUpdateTime": "2021-10-04T15:10:00Z", "lastTransitionTime": "2021-10-04T15:10:00Z"},
            {"type": "Progressing", "status": "True", "reason": "NewReplicaSetAvailable",
             "message": "ReplicaSet \"example-5d59d67564\" has successfully progressed.",
             "lastUpdateTime": "2021-10-04T15:10:00Z", "lastTransitionTime": "2021-10-04T15:09:37Z"},
        ],
    },
}


def J(o) -> bytes:
    return json.dumps(o, separators=(",", ":")).encode()


def mod(fn, base=BASE):
    o = copy.deepcopy(base)
    fn(o)
    return o


def _set(path, value):
    def f(o):
        cur = o
        for k in path[:-1]:
            cur = cur[k]
        cur[path[-1]] = value
    return f


def _del(path):
    def f(o):
        cur = o
        for k in path[:-1]:
            cur = cur[k]
        del cur[path[-1]]
    return f


def cases():
    B = BASE
    out = []
    add = lambda name, a, b, se, st: out.append((name, a if isinstance(a, bytes) else J(a),
                                                 b if isinstance(b, bytes) else J(b), se, st))
    # 1
    add("01_identical", B, B, True, True)

    # 2 ignored metadata
    def meta_noise(o):
        m = o["metadata"]
        m["uid"] = "99999999-0000-4000-8000-000000000002"
        m["resourceVersion"] = "2002"
        m["generation"] = 7
        m["creationTimestamp"] = "2021-10-05T00:00:00Z"
        m["clusterName"] = "phys-1"
        m["managedFields"] = [{"manager": "syncer", "operation": "Update"}]
        m["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "Deployment", "name": "x", "uid": "u"}]
    add("02_ignored_metadata", B, mod(meta_noise), True, True)

    # 3 labels absent / {} / null
    nolab = mod(_del(["metadata", "labels"]))
    add("03a_labels_absent_vs_empty", nolab, mod(_set(["metadata", "labels"], {})), True, True)
    add("03b_labels_absent_vs_null", nolab, mod(_set(["metadata", "labels"], None)), True, True)
    add("03c_labels_empty_vs_null", mod(_set(["metadata", "labels"], {})),
        mod(_set(["metadata", "labels"], None)), True, True)
    # 4
    add("04_label_str_vs_int", mod(_set(["metadata", "labels"], {"a": "1"})),
        mod(_set(["metadata", "labels"], {"a": 1})), False, True)
    # 5
    add("05_label_int_vs_absent", mod(_set(["metadata", "labels"], {"a": 1})), nolab, True, True)
    # 6
    add("06_annotation_changed", B,
        mod(_set(["metadata", "annotations"], {"deployment.kubernetes.io/revision": "2"})), False, True)
    # 7
    add("07_int_vs_float", J(B), J(B).replace(b'"replicas":3,"selector"', b'"replicas":3.0,"selector"'),
        False, True)
    # 8
    a8 = mod(_set(["spec", "x"], 1.5))
    add("08a_1.5_vs_1.50", J(a8), J(a8).replace(b'"x":1.5', b'"x":1.50'), True, True)
    a8b = mod(_set(["spec", "x"], 100.0))
    add("08b_100.0_vs_1e2", J(a8b), J(a8b).replace(b'"x":100.0', b'"x":1e2'), True, True)
    add("08c_neg0.0_vs_0.0", J(a8b).replace(b'"x":100.0', b'"x":-0.0'),
        J(a8b).replace(b'"x":100.0', b'"x":0.0'), True, True)
    # 9
    add("09_0_vs_neg0", J(a8b).replace(b'"x":100.0', b'"x":0'),
        J(a8b).replace(b'"x":100.0', b'"x":-0'), True, True)
    # 10
    a10 = mod(_set(["spec", "s"], "A"))
    add("10_escape_A", J(a10), J(a10).replace(b'"s":"A"', b'"s":"\\u0041"'), True, True)
    # 11
    add("11_toplevel_spec_null_vs_absent", mod(_set(["spec"], None)), mod(_del(["spec"])), True, True)
    # 12
    add("12_nested_null_vs_absent", mod(_set(["spec", "x"], None)), B, False, True)
    # 13
    add("13a_empty_obj_vs_absent", mod(_set(["spec", "x"], {})), B, False, True)
    add("13b_empty_arr_vs_null", mod(_set(["spec", "x"], [])), mod(_set(["spec", "x"], None)), False, True)
    add("13c_empty_obj_vs_empty_arr", mod(_set(["spec", "x"], {})), mod(_set(["spec", "x"], [])), False, True)
    # 14
    add("14_list_reorder", mod(_set(["spec", "x"], ["a", "b"])), mod(_set(["spec", "x"], ["b", "a"])), False, True)
    # 15 key order / whitespace
    pretty = json.dumps(B, indent=3, sort_keys=True).encode()
    add("15_key_order_whitespace", B, pretty, True, True)
    # 16
    def cpu(v):
        def f(o):
            o["spec"]["template"]["spec"]["containers"][0]["resources"] = {"limits": {"cpu": v}}
        return f
    add("16_quantity_strings", mod(cpu("1000m")), mod(cpu("1")), False, True)
    # 17
    add("17_extra_toplevel_key", B, mod(_set(["data"], {"k": "v"})), False, True)
    # 18
    add("18_only_status_differs", B, mod(_set(["status", "readyReplicas"], 2)), True, False)
    # 19
    add("19a_kind_differs", B, mod(_set(["kind"], "ReplicaSet")), False, True)
    add("19b_apiversion_differs", B, mod(_set(["apiVersion"], "apps/v1beta1")), False, True)
    # 20
    nostat = mod(_del(["status"]))
    add("20_new_has_no_status", B, nostat, True, False)
    # 21
    add("21_old_no_status_new_null", nostat, mod(_set(["status"], None)), True, True)
    # 22
    add("22_old_empty_new_null", mod(_set(["status"], {})), mod(_set(["status"], None)), True, False)
    # 23
    add("23_old_no_status_new_empty", nostat, mod(_set(["status"], {})), True, False)
    # 24
    def reorder(o):
        o["status"]["conditions"].reverse()
    add("24_conditions_reordered", B, mod(reorder), True, False)
    # 25
    a25 = mod(_set(["spec", "x"], 1))
    add("25_int64max_vs_overflow", J(a25).replace(b'"x":1', b'"x":9223372036854775807'),
        J(a25).replace(b'"x":1', b'"x":9223372036854775808'), False, True)
    # 26
    add("26_float_equal_forms", J(a25).replace(b'"x":1', b'"x":9223372036854775808'),
        J(a25).replace(b'"x":1', b'"x":9.223372036854775808e18'), True, True)
    # 27
    add("27_duplicate_key_last_wins", J(a25).replace(b'"x":1', b'"x":{"a":1,"a":2}'),
        J(a25).replace(b'"x":1', b'"x":{"a":2}'), True, True)
    # 28
    add("28_asymmetry_of_23", mod(_set(["status"], {})), nostat, True, False)
    # 29
    add("29_list_length_change", mod(_set(["spec", "x"], [1, 2])), mod(_set(["spec", "x"], [1, 2, 3])), False, True)
    # 30
    add("30_key0_vs_index0", mod(_set(["spec", "x"], {"0": 1})), mod(_set(["spec", "x"], [1])), False, True)

    # ---- extra edge cases (not in A.4; oracle-pinned) ----
    add("x01_labels_metadata_not_map", mod(_set(["metadata"], "oops")), mod(_set(["metadata"], 5)), True, True)
    add("x02_labels_equal_diff_order", mod(_set(["metadata", "labels"], {"a": "1", "b": "2"})),
        mod(_set(["metadata", "labels"], {"b": "2", "a": "1"})), True, True)
    add("x03_label_value_long_change", mod(_set(["metadata", "labels"], {"a": "x" * 40})),
        mod(_set(["metadata", "labels"], {"a": "x" * 39 + "y"})), False, True)
    add("x04_nested_dup_keys_subtree", J(a25).replace(b'"x":1', b'"x":{"a":{"p":1},"a":{"q":2}}'),
        J(a25).replace(b'"x":1', b'"x":{"a":{"q":2}}'), True, True)
    add("x05_invalid_utf8_vs_fffd", J(a10).replace(b'"s":"A"', b'"s":"\xff"'),
        J(a10).replace(b'"s":"A"', b'"s":"\\ufffd"'), True, True)
    add("x06_lone_surrogate", J(a10).replace(b'"s":"A"', b'"s":"\\ud800x"'),
        J(a10).replace(b'"s":"A"', b'"s":"\xef\xbf\xbdx"'), True, True)
    add("x07_surrogate_pair", J(a10).replace(b'"s":"A"', b'"s":"\\ud83d\\ude00"'),
        J(a10).replace(b'"s":"A"', b'"s":"\xf0\x9f\x98\x80"'), True, True)
    add("x08_truncated_utf8_3fffd", J(a10).replace(b'"s":"A"', b'"s":"\xf0\x9f\x98a"'),
        J(a10).replace(b'"s":"A"', b'"s":"\\ufffd\\ufffd\\ufffda"'), True, True)
    add("x09_string_len8_vs_9", J(a10).replace(b'"s":"A"', b'"s":"12345678"'),
        J(a10).replace(b'"s":"A"', b'"s":"123456789"'), False, True)
    add("x10_string_nul_padding", J(a10).replace(b'"s":"A"', b'"s":"ab"'),
        J(a10).replace(b'"s":"A"', b'"s":"ab\\u0000"'), False, True)
    add("x11_decode_error", B, b'{"apiVersion": "v1", ', False, False)
    add("x12_float_underflow_zero", J(a25).replace(b'"x":1', b'"x":1e-400'),
        J(a25).replace(b'"x":1', b'"x":0.0'), True, True)
    add("x13_neg_int64_min", J(a25).replace(b'"x":1', b'"x":-9223372036854775808'),
        J(a25).replace(b'"x":1', b'"x":-9223372036854775809'), False, True)
    add("x14_bool_vs_int", mod(_set(["spec", "x"], True)), mod(_set(["spec", "x"], 1)), False, True)
    add("x15_status_scalar", mod(_set(["status"], "ok")), mod(_set(["status"], "ok")), True, True)
    add("x16_empty_objects", b'{}', b'{}', True, False)
    add("x17_annotation_nonstring_collapses", mod(_set(["metadata", "annotations"], {"a": "1", "b": True})),
        mod(_del(["metadata", "annotations"])), True, True)
    add("x18_long_string_same_hash_prefix", J(a10).replace(b'"s":"A"', b'"s":"' + b'z' * 100 + b'"'),
        J(a10).replace(b'"s":"A"', b'"s":"' + b'z' * 99 + b'y"'), False, True)
    add("x19_deep_nesting", mod(_set(["spec", "x"], {"a": [[[{"b": [1, {"c": None}]}]]]})),
        mod(_set(["spec", "x"], {"a": [[[{"b": [1, {"c": False}]}]]]})), False, True)
    add("x20_trailing_garbage", B, J(B) + b" x", False, False)

    # ---- the informer decoder's list probe (apimachinery unstructuredJSONScheme.decode, reached from
    # pkg/syncer/syncer.go:105-108): a top-level key equal to "Items" under encoding/json's case folding
    # (any value, null included) decodes as an UnstructuredList, which fails the type assertions of
    # specsyncer.go:18-22 / statussyncer.go:16-20 -> both predicates false, even for identical objects
    items = mod(_set(["items"], []))
    add("x21_list_probe_items", items, items, False, False)
    add("x22_list_probe_items_null_in_new", B, mod(_set(["items"], None)), False, False)
    add("x23_list_probe_case_folded", J(B), J(B)[:-1] + b',"iTEMs":{"a":1}}', False, False)
    add("x24_list_probe_long_s", J(B)[:-1] + b',"item\xc5\xbf":1}', J(B), False, False)
    add("x25_list_probe_escaped_key", J(B)[:-1] + b',"\\u0069tems":1}', J(B)[:-1] + b',"\\u0069tems":1}',
        False, False)
    add("x26_not_list_nested_items", mod(_set(["spec", "items"], [1])), mod(_set(["spec", "items"], [1])), True, True)
    add("x27_not_list_near_misses", J(B)[:-1] + b',"itemz":1,"item":2,"itemss":3,"\xc4\xb1tems":4}',
        J(B)[:-1] + b',"itemz":1,"item":2,"itemss":3,"\xc4\xb1tems":4}', True, True)
    # ---- encoding/json's maxNestingDepth (10000): a document nested 10000 containers deep decodes,
    # 10001 is a decode error (the pair is dirty); spec.x sits at depth 2, so n arrays reach depth n + 2
    deep = lambda n: J(a25).replace(b'"x":1', b'"x":' + b'[' * n + b']' * n)
    add("x28_depth_10000", deep(9998), deep(9998), True, True)
    add("x29_depth_10001", deep(9998), deep(9999), False, False)
    add("x30_depth_10000_changed", deep(9998), deep(9997) + b'', False, True)
    # ---- the write-path no-op hints (GPUDIFF_SPEC_NOOP / GPUDIFF_STATUS_NOOP): dirty under
    # DeepEqual (int64 != float64), identical on the wire
    add("x31_noop_int_vs_integral_float", J(B), J(B).replace(b'"replicas":3,"selector"', b'"replicas":3.0,"selector"'),
        False, True)
    add("x32_not_noop_beyond_2p53", J(a25).replace(b'"x":1', b'"x":9007199254740993'),
        J(a25).replace(b'"x":1', b'"x":9007199254740992.0'), False, True)
    add("x33_noop_status_int_vs_float", J(B), J(B).replace(b'"readyReplicas":3', b'"readyReplicas":3e0'), True, False)
    add("x34_not_noop_mixed", J(B), J(B).replace(b'"replicas":3,"selector"', b'"replicas":3.0,"selector"')
        .replace(b'"revisionHistoryLimit":10', b'"revisionHistoryLimit":11'), False, True)
    add("x35_noop_neg_zero", J(a25).replace(b'"x":1', b'"x":0'), J(a25).replace(b'"x":1', b'"x":-0.0'), False, True)
    return out


# write-path no-op hints the oracle must produce for these rows: name -> (spec_noop, status_noop)
NOOP_KAT = {
    "x31_noop_int_vs_integral_float": (True, False),
    "x32_not_noop_beyond_2p53": (False, False),
    "x33_noop_status_int_vs_float": (False, True),
    "x34_not_noop_mixed": (False, False),
    "x35_noop_neg_zero": (True, False),
    "x16_empty_objects": (False, True),           # neither side has a status key: UpdateStatus writes nothing
    "20_new_has_no_status": (False, False),       # A has a status B would clear
    "18_only_status_differs": (False, False),
    "07_int_vs_float": (True, False),
    "25_int64max_vs_overflow": (False, False),     # 2^63 - 1 vs 2^63 (float): beyond 2^53
}

"""Known answers for the API-negotiation update classifier
(pkg/reconciler/apiresource/controller.go:238-295).  Each case states the
action Go 1.16 + the pinned apimachinery produce for (old, new); the outcomes
were derived by hand from the reference code and the encoding/json, time and
Semantic.DeepEqual rules quoted in oracle/negotiate_oracle.py."""
import json

IGNORE, SPEC, STATUS, META, CREATED, DECODE = 0, 1, 2, 3, 4, -1


def obj(rv="1", gen=1, labels=None, ann=None, conds=None, kind="APIResourceImport", extra_meta=None,
        status_extra=None):
    meta = {"name": "deployments.v1.apps", "clusterName": "admin", "resourceVersion": rv, "generation": gen}
    if labels is not None:
        meta["labels"] = labels
    if ann is not None:
        meta["annotations"] = ann
    if extra_meta:
        meta.update(extra_meta)
    st = {}
    if conds is not None:
        st["conditions"] = conds
    if status_extra:
        st.update(status_extra)
    return json.dumps({"apiVersion": "apiresource.kcp.dev/v1alpha1", "kind": kind, "metadata": meta,
                       "spec": {"groupVersion": {"group": "apps", "version": "v1"}, "plural": "deployments",
                                "location": "us-east1", "schemaUpdateStrategy": "UpdateUnpublished"},
                       "status": st}).encode()


def cond(t="Compatible", s="True", ltt="2021-10-04T15:09:37Z", reason="", msg=""):
    c = {"type": t, "status": s, "lastTransitionTime": ltt}
    if reason:
        c["reason"] = reason
    if msg:
        c["message"] = msg
    return c


L = {"kcp.dev/cluster": "c1"}
A = {"note": "x"}
C = [cond()]


def cases():
    """(name, old bytes or None, new bytes, expected action)"""
    out = [
        ("created", None, obj(), CREATED),
        ("same-rv", obj(rv="5", labels=L), obj(rv="5", gen=9, labels={"x": "y"}), IGNORE),
        ("gen-changed", obj(rv="1", gen=1), obj(rv="2", gen=2), SPEC),
        ("gen-changed-beats-status", obj(rv="1", conds=C), obj(rv="2", gen=3, conds=[]), SPEC),
        ("status-cond-added", obj(rv="1", conds=[]), obj(rv="2", conds=C), STATUS),
        ("status-nil-vs-empty", obj(rv="1"), obj(rv="2", conds=[]), META),
        ("status-null-vs-empty", obj(rv="1", conds=None),
         obj(rv="2").replace(b'"status": {}', b'"status": {"conditions": null}'), META),
        ("status-reason", obj(rv="1", conds=C), obj(rv="2", conds=[cond(reason="R")]), STATUS),
        ("status-message", obj(rv="1", conds=[cond(msg="a")]), obj(rv="2", conds=[cond(msg="b")]), STATUS),
        ("status-type", obj(rv="1", conds=C), obj(rv="2", conds=[cond(t="Available")]), STATUS),
        ("status-order", obj(rv="1", conds=[cond(), cond(t="B")]), obj(rv="2", conds=[cond(t="B"), cond()]), STATUS),
        # metav1.Time semantic equality: the same instant in another zone / with zero fraction
        ("time-same-instant-offset", obj(rv="1", conds=[cond(ltt="2021-10-04T15:09:37Z")]),
         obj(rv="2", conds=[cond(ltt="2021-10-04T17:09:37+02:00")]), META),
        ("time-zero-fraction", obj(rv="1", conds=[cond(ltt="2021-10-04T15:09:37Z")]),
         obj(rv="2", conds=[cond(ltt="2021-10-04T15:09:37.000Z")]), META),
        ("time-ns-differs", obj(rv="1", conds=[cond(ltt="2021-10-04T15:09:37.1Z")]),
         obj(rv="2", conds=[cond(ltt="2021-10-04T15:09:37.100000001Z")]), STATUS),
        ("time-one-digit-hour", obj(rv="1", conds=[cond(ltt="2021-10-04T05:09:37Z")]),
         obj(rv="2", conds=[cond(ltt="2021-10-04T5:09:37Z")]), META),
        ("time-null-vs-zero", obj(rv="1", conds=[cond(ltt=None)]),
         obj(rv="2", conds=[cond(ltt="0001-01-01T00:00:00Z")]), META),
        ("time-absent-vs-null", obj(rv="1", conds=[{"type": "T", "status": "True"}]),
         obj(rv="2", conds=[{"type": "T", "status": "True", "lastTransitionTime": None}]), META),
        ("time-negative-zone", obj(rv="1", conds=[cond(ltt="2021-10-04T00:30:00-01:00")]),
         obj(rv="2", conds=[cond(ltt="2021-10-04T01:30:00Z")]), META),
        ("time-leap-day", obj(rv="1", conds=[cond(ltt="2020-02-29T00:00:00Z")]),
         obj(rv="2", conds=[cond(ltt="2020-02-28T24:00:00Z")]), DECODE),  # hour 24: range error
        ("time-bad-day", obj(rv="1"), obj(rv="2", conds=[cond(ltt="2021-02-29T00:00:00Z")]), DECODE),
        ("time-not-rfc3339", obj(rv="1"), obj(rv="2", conds=[cond(ltt="2021-10-04 15:09:37Z")]), DECODE),
        ("time-empty", obj(rv="1"), obj(rv="2", conds=[cond(ltt="")]), DECODE),
        ("time-number", obj(rv="1"), obj(rv="2", conds=[cond(ltt=5)]), DECODE),
        ("time-10-frac-digits", obj(rv="1", conds=[cond(ltt="2021-10-04T15:09:37.000000001Z")]),
         obj(rv="2", conds=[cond(ltt="2021-10-04T15:09:37.0000000001Z")]), META),  # parseNanoseconds quirk
        ("time-second-60", obj(rv="1"), obj(rv="2", conds=[cond(ltt="2021-10-04T15:09:60Z")]), DECODE),
        # the missing `!` at controller.go:278
        ("meta-nothing-changed", obj(rv="1", labels=L, ann=A), obj(rv="2", labels=L, ann=A), META),
        ("meta-labels-changed-only", obj(rv="1", labels=L, ann=A), obj(rv="2", labels={"a": "b"}, ann=A), IGNORE),
        ("meta-annotations-changed", obj(rv="1", labels=L, ann=A), obj(rv="2", labels={"a": "b"}, ann={}), META),
        ("meta-ann-nil-vs-empty", obj(rv="1", labels=L), obj(rv="2", labels={"z": "1"}, ann={}), IGNORE),
        ("meta-labels-nil-vs-empty", obj(rv="1", ann=A), obj(rv="2", labels={}, ann=A), META),
        ("meta-label-null-elem", obj(rv="1", labels={"a": ""}, ann=A), obj(rv="2", labels={"a": None}, ann=A), META),
        # typed decode rules
        ("fold-Metadata", obj(rv="1", gen=1),
         obj(rv="2", gen=1).replace(b'"metadata"', b'"Metadata"'), META),
        ("fold-generation", obj(rv="1", gen=1), obj(rv="2", gen=1).replace(b'"generation": 1', b'"GENERATION": 7'), SPEC),
        ("gen-null-noop", obj(rv="1", gen=0), obj(rv="2").replace(b'"generation": 1', b'"generation": null'), META),
        ("gen-float", obj(rv="1"), obj(rv="2").replace(b'"generation": 1', b'"generation": 1.0'), DECODE),
        ("gen-string", obj(rv="1"), obj(rv="2").replace(b'"generation": 1', b'"generation": "1"'), DECODE),
        ("rv-number", obj(rv="1"), obj(rv="2").replace(b'"resourceVersion": "2"', b'"resourceVersion": 2'), DECODE),
        ("rv-escaped-equal", obj(rv="12"), obj(rv="12").replace(b'"resourceVersion": "12"', b'"resourceVersion": "\\u00312"'), IGNORE),
        ("status-unknown-field", obj(rv="1", conds=C), obj(rv="2", conds=C, status_extra={"phase": "X"}), META),
        ("cond-unknown-field", obj(rv="1", conds=C), obj(rv="2", conds=[dict(cond(), extra=1)]), META),
        ("cond-null-elem", obj(rv="1", conds=[{}]), obj(rv="2", conds=[None]), META),
        ("cond-null-elem-vs-none", obj(rv="1", conds=[]), obj(rv="2", conds=[None]), STATUS),
        ("cond-not-object", obj(rv="1"), obj(rv="2", conds=[5]), DECODE),
        ("label-number", obj(rv="1"), obj(rv="2", labels={"a": 1}), DECODE),
        ("status-string", obj(rv="1"), obj(rv="2").replace(b'"status": {}', b'"status": "x"'), DECODE),
        ("bad-json", obj(rv="1"), b'{"metadata": {', DECODE),
        # outside the reference's domain (Go's typed Unmarshal would reject the object, so the informer never
        # delivers it): the build's documented answers -- classified by the fields read; a root null is DECODE
        ("outside-domain-spec-type-error", obj(rv="1", gen=1),
         obj(rv="2", gen=2).replace(b'"plural": "deployments"', b'"plural": 5'), SPEC),
        ("outside-domain-root-null", obj(rv="1"), b'null', DECODE),
        ("negotiated-kind", obj(rv="1", kind="NegotiatedAPIResource", conds=C),
         obj(rv="2", kind="NegotiatedAPIResource", conds=[cond(s="False")]), STATUS),
    ]
    # repeated keys: Go decodes again into the same field
    rep_old = obj(rv="1", conds=[cond(reason="R")])
    rep_new = (b'{"metadata": {"resourceVersion": "2", "generation": 1}, "status": {"conditions": ['
               b'{"type": "Compatible", "status": "True", "lastTransitionTime": "2021-10-04T15:09:37Z"}],'
               b' "conditions": [{"reason": "R"}]}}')
    out.append(("repeated-conditions-merge", rep_old, rep_new, META))
    rep_new2 = (b'{"metadata": {"resourceVersion": "2", "generation": 1}, "status": {"conditions": ['
                b'{"type": "A"}, {"type": "B"}], "conditions": [{"status": "X"}],'
                b' "conditions": [{}, {}]}}')
    rep_old2 = b'{"metadata": {"resourceVersion": "1", "generation": 1}, "status": {"conditions": [{"type": "A", "status": "X"}, {"type": "B"}]}}'
    out.append(("repeated-conditions-stale-capacity", rep_old2, rep_new2, META))
    out.append(("repeated-labels-merge", obj(rv="1", labels={"a": "1", "b": "2"}, ann=A),
                b'{"metadata": {"resourceVersion": "2", "generation": 1, "labels": {"a": "1"}, "labels": {"b": "2"},'
                b' "annotations": {"note": "x"}}, "status": {}}', META))
    out.append(("repeated-labels-null-resets", obj(rv="1", labels={"b": "2"}, ann=A),
                b'{"metadata": {"resourceVersion": "2", "generation": 1, "labels": {"a": "1"}, "labels": null,'
                b' "labels": {"b": "2"}, "annotations": {"note": "x"}}, "status": {}}', META))
    out.append(("repeated-rv-last-wins", obj(rv="3"),
                b'{"metadata": {"resourceVersion": "1", "resourceVersion": "3", "generation": 9}}', IGNORE))
    return out


# ---------------------------------------------------------------- CustomResourceDefinition events (controller.go:186-199)
NAMES = {"plural": "widgets", "singular": "widget", "kind": "Widget", "listKind": "WidgetList"}
EST = [cond(t="NamesAccepted", reason="NoConflicts", msg="no conflicts found"),
       cond(t="Established", reason="InitialNamesAccepted", msg="the initial names have been accepted")]
_ABSENT = object()


def crd(rv="1", gen=1, labels=None, ann=None, conds=EST, names=_ABSENT, stored=_ABSENT, status_extra=None):
    """An apiextensions/v1 CustomResourceDefinition as the API server writes it
    (names / stored default to NAMES / ["v1"]; pass None for a JSON null,
    _ABSENT -- the default sentinel -- via absent=... below)."""
    meta = {"name": "widgets.example.dev", "clusterName": "admin", "resourceVersion": rv, "generation": gen}
    if labels is not None:
        meta["labels"] = labels
    if ann is not None:
        meta["annotations"] = ann
    st = {}
    if conds is not None:
        st["conditions"] = conds
    st["acceptedNames"] = dict(NAMES) if names is _ABSENT else names
    st["storedVersions"] = ["v1"] if stored is _ABSENT else stored
    if status_extra:
        st.update(status_extra)
    return json.dumps({"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition", "metadata": meta,
                       "spec": {"group": "example.dev", "names": dict(NAMES), "scope": "Namespaced",
                                "versions": [{"name": "v1", "served": True, "storage": True,
                                              "schema": {"openAPIV3Schema": {"type": "object"}}}]},
                       "status": st}).encode()


def _drop(doc, key):
    """remove `"key": <value>, ` / `, "key": <value>` from a compact status (value: a JSON list/object/string)"""
    d = json.loads(doc)
    d["status"].pop(key)
    return json.dumps(d).encode()


def crd_cases():
    """(name, old, new, expected) for kind CustomResourceDefinition; the typed
    status is {conditions, acceptedNames {plural, singular, shortNames, kind,
    listKind, categories}, storedVersions}."""
    n2 = dict(NAMES, shortNames=["wd"], categories=["all"])
    out = [
        ("crd-created", None, crd(), CREATED),
        ("crd-same-rv", crd(rv="4"), crd(rv="4", gen=2, names=dict(NAMES, plural="x")), IGNORE),
        ("crd-gen-changed", crd(rv="1"), crd(rv="2", gen=2, stored=["v1", "v2"]), SPEC),
        ("crd-established", crd(rv="1", conds=[]), crd(rv="2"), STATUS),
        ("crd-plural-changed", crd(rv="1"), crd(rv="2", names=dict(NAMES, plural="widgetz")), STATUS),
        ("crd-listkind-changed", crd(rv="1"), crd(rv="2", names=dict(NAMES, listKind="Widgets")), STATUS),
        ("crd-names-absent-vs-null", _drop(crd(rv="1"), "acceptedNames"), crd(rv="2", names=None), META),
        ("crd-names-absent-vs-empty", _drop(crd(rv="1"), "acceptedNames"), crd(rv="2", names={}), META),
        ("crd-names-null-vs-set", crd(rv="1", names=None), crd(rv="2"), STATUS),
        ("crd-shortnames-nil-vs-empty", crd(rv="1"), crd(rv="2", names=dict(NAMES, shortNames=[])), META),
        ("crd-shortnames-null-vs-empty", crd(rv="1", names=dict(NAMES, shortNames=None)),
         crd(rv="2", names=dict(NAMES, shortNames=[])), META),
        ("crd-shortnames-added", crd(rv="1", names=dict(NAMES, shortNames=[])), crd(rv="2", names=n2), STATUS),
        ("crd-shortnames-order", crd(rv="1", names=dict(NAMES, shortNames=["a", "b"])),
         crd(rv="2", names=dict(NAMES, shortNames=["b", "a"])), STATUS),
        ("crd-categories-changed", crd(rv="1", names=n2), crd(rv="2", names=dict(n2, categories=["all", "x"])), STATUS),
        ("crd-categories-equal", crd(rv="1", names=n2), crd(rv="2", names=dict(n2)), META),
        ("crd-stored-appended", crd(rv="1"), crd(rv="2", stored=["v1", "v2"]), STATUS),
        ("crd-stored-null-vs-empty", crd(rv="1", stored=None), crd(rv="2", stored=[]), META),
        ("crd-stored-absent-vs-null", _drop(crd(rv="1"), "storedVersions"), crd(rv="2", stored=None), META),
        ("crd-stored-null-elem", crd(rv="1", stored=["", "v1"]), crd(rv="2", stored=[None, "v1"]), META),
        ("crd-stored-empty-string-vs-none", crd(rv="1", stored=[]), crd(rv="2", stored=[""]), STATUS),
        ("crd-stored-number", crd(rv="1"), crd(rv="2", stored=[1]), DECODE),
        ("crd-stored-object", crd(rv="1"), crd(rv="2", stored={"v1": True}), DECODE),
        ("crd-names-not-object", crd(rv="1"), crd(rv="2", names="widgets"), DECODE),
        ("crd-names-array", crd(rv="1"), crd(rv="2", names=[]), DECODE),
        ("crd-listkind-number", crd(rv="1"), crd(rv="2", names=dict(NAMES, listKind=3)), DECODE),
        ("crd-shortname-object", crd(rv="1"), crd(rv="2", names=dict(NAMES, shortNames=[{}])), DECODE),
        ("crd-plural-null-noop", crd(rv="1", names=dict(NAMES, plural="")), crd(rv="2", names=dict(NAMES, plural=None)),
         META),
        ("crd-names-fold-key", crd(rv="1"),
         crd(rv="2").replace(b'"plural": "widgets", "singular": "widget", "kind": "Widget", "listKind": "WidgetList"}, '
                             b'"storedVersions"',
                             b'"PLURAL": "widgets", "singular": "widget", "kind": "Widget", "listKind": "WidgetList"}, '
                             b'"storedVersions"'), META),
        ("crd-status-fold-key", crd(rv="1"), crd(rv="2").replace(b'"storedVersions"', b'"StoredVersions"'), META),
        ("crd-names-unknown-field", crd(rv="1"), crd(rv="2", names=dict(NAMES, extra="x")), META),
        ("crd-status-unknown-field", crd(rv="1"), crd(rv="2", status_extra={"phase": "x"}), META),
        ("crd-cond-time-same-instant", crd(rv="1", conds=[cond(t="Established", ltt="2021-10-04T15:09:37Z")]),
         crd(rv="2", conds=[cond(t="Established", ltt="2021-10-04T16:09:37+01:00")]), META),
        ("crd-meta-labels-changed-only", crd(rv="1", labels=L, ann=A), crd(rv="2", labels={"a": "b"}, ann=A), IGNORE),
    ]
    # repeated keys: Go decodes again into the same field
    base = b'{"metadata": {"resourceVersion": "2", "generation": 1}, "status": {%s}}'
    out.append(("crd-repeated-names-merge", crd(rv="1", conds=None, stored=None),
                base % (b'"acceptedNames": {"plural": "widgets", "kind": "Nope"}, "acceptedNames": {"singular": '
                        b'"widget", "kind": "Widget", "listKind": "WidgetList"}'), META))
    out.append(("crd-repeated-names-null-keeps", crd(rv="1", conds=None, stored=None),
                base % (b'"acceptedNames": {"plural": "widgets", "singular": "widget", "kind": "Widget", '
                        b'"listKind": "WidgetList"}, "acceptedNames": null'), META))
    out.append(("crd-repeated-stored-stale-capacity", crd(rv="1", conds=None, names=None, stored=["x", "b"]),
                base % b'"storedVersions": ["a", "b"], "storedVersions": ["x"], "storedVersions": [null, null]', META))
    out.append(("crd-repeated-shortnames-stale-capacity", crd(rv="1", conds=None, stored=None,
                                                           names=dict(NAMES, shortNames=["p", "q", "r"])),
                base % (b'"acceptedNames": {"plural": "widgets", "singular": "widget", "kind": "Widget", "listKind": '
                        b'"WidgetList", "shortNames": ["a", "q", "r"]}, "acceptedNames": {"shortNames": ["p"]}, '
                        b'"acceptedNames": {"shortNames": [null, null, null]}'), META))
    return out


def kcp_kind_ignores_crd_status():
    """The same CRD documents classified as an APIResourceImport (kind 0): only
    status.conditions is read, so acceptedNames / storedVersions changes are
    invisible (metadata then decides)."""
    return [
        ("kcp-kind-plural-changed", crd(rv="1"), crd(rv="2", names=dict(NAMES, plural="widgetz")), META),
        ("kcp-kind-stored-number", crd(rv="1"), crd(rv="2", stored=[1]), META),
        ("kcp-kind-established", crd(rv="1", conds=[]), crd(rv="2"), STATUS),
    ]

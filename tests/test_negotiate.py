"""API-negotiation update classifier (second half;
pkg/reconciler/apiresource/controller.go:238-295) on the CPU: the oracle and the
product's host path (gpudiff_negotiate_pair_host) against the hand-written
known answers, each other on seeded fuzzed populations, and the generator's
designed outcomes."""
import random

import pytest

from kcp_amd import gpudiff as G
from kcp_amd import synth as S
from oracle import negotiate_oracle as N
from tests import negotiate_cases as C

EDITS = [
    (b'"metadata":{', b'"Metadata":{'), (b'"generation":', b'"Generation":'), (b'"labels":{', b'"LABELS":{'),
    (b'"resourceVersion":"', b'"resourceVersion":"\\u0031'), (b'"conditions":[', b'"conditions":null,"conditions":['),
    (b'"conditions":[', b'"conditions":[null,'), (b'"conditions":[', b'"conditions":[{"type":"A"}],"conditions":['),
    (b'"reason":"', b'"REASON":"x","reason":"'), (b'"lastTransitionTime":"2021-', b'"lastTransitionTime":"2021-1'),
    (b'T0', b'T'), (b'Z"', b'.5Z"'), (b'Z"', b'.123456789012Z"'), (b'Z"', b'+00:00"'), (b'Z"', b'-23:59"'),
    (b'"generation":', b'"generation":1.0,"g":'), (b'"generation":', b'"generation":null,"generation":'),
    (b'"annotations":{', b'"annotations":{"x":null,'), (b'"annotations":{', b'"annotations":{"n":5,'),
    (b'"labels":{', b'"labels":{"app":"dup",'), (b'"status":{', b'"status":null,"status":{'),
    (b'"status":{', b'"statu\xc5\xbf":{"conditions":[]},"status":{'), (b'"message":"', b'"message":"\\n'),
    (b'"kind"', b'"kind":1,"k"'), (b'}}', b'}} '), (b'"spec":{', b'"spec":{"q":tru,'),
    (b'"lastTransitionTime":"', b'"lastTransitionTime":null,"x":"'), (b'"type":"', b'"type":7,"t":"'),
]


def fuzz_pairs(n, seed):
    pairs, _ = S.negotiate_population(n, seed=seed)
    rng = random.Random(seed)
    out = []
    for a, b in pairs:
        r = rng.random()
        if r < 0.25:
            x, y = rng.choice(EDITS)
            b = b.replace(x, y, 1)
        elif r < 0.4:
            x, y = rng.choice(EDITS)
            a = a.replace(x, y, 1)
        elif r < 0.45:
            a = None
        out.append((a, b))
    return out


@pytest.mark.parametrize("case", C.cases(), ids=lambda c: c[0])
def test_oracle_kat(case):
    name, a, b, want = case
    assert N.classify(a, b) == want


@pytest.mark.parametrize("case", C.cases(), ids=lambda c: c[0])
def test_host_kat(case):
    name, a, b, want = case
    assert G.negotiate_pair_host(a, b) == want


@pytest.mark.parametrize("s,want", [
    ("1970-01-01T00:00:00Z", (0, 0)), ("0001-01-01T00:00:00Z", N.ZERO_TIME),
    ("2021-10-04T15:09:37.5+02:00", (1633352977, 500000000)), ("2000-02-29T1:02:03Z", (951786123, 0)),
    ("2021-10-04T15:09:37.0000000001Z", (1633360177, 1)), ("9999-12-31T23:59:59.999999999Z", (253402300799, 999999999)),
    ("2021-10-04T15:09:37+-1:00", (1633360177 + 3600, 0)),
])
def test_time_parse(s, want):
    assert N.parse_rfc3339(s) == want


@pytest.mark.parametrize("s", ["2021-13-01T00:00:00Z", "2021-04-31T00:00:00Z", "2021-10-04T24:00:00Z",
                               "2021-10-04T15:60:00Z", "2021-10-04t15:09:37Z", "2021-10-04T15:09:37z",
                               "2021-10-04T15:09:37", "2021-10-04T15:09:37+0100", "21-10-04T15:09:37Z",
                               "2021-10-04T15:09:37.Z", "2021-10-04T15:09:37.1234567890Z", "", " 2021-10-04T15:09:37Z"])
def test_time_parse_rejects(s):
    with pytest.raises(N.DecodeError):
        N.parse_rfc3339(s)


def test_population_matches_design():
    pairs, want = S.negotiate_population(3000, seed=11)
    got = [N.classify(a, b) for a, b in pairs]
    assert got == want.tolist()


def test_host_matches_oracle_fuzz():
    pairs = fuzz_pairs(3000, 20211004 + 71)
    bad = [i for i, (a, b) in enumerate(pairs) if G.negotiate_pair_host(a, b) != N.classify(a, b)]
    assert not bad, (len(bad), pairs[bad[0]], G.negotiate_pair_host(*pairs[bad[0]]), N.classify(*pairs[bad[0]]))


def random_times(n, seed):
    """RFC3339 strings across the whole range: valid ones in every zone/fraction shape, plus near misses."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        y, mo, d = rng.randint(1, 9999), rng.randint(1, 12), rng.randint(1, 28)
        h, mi, s = rng.randint(0, 23), rng.randint(0, 59), rng.randint(0, 59)
        t = "%04d-%02d-%02dT%02d:%02d:%02d" % (y, mo, d, h, mi, s)
        r = rng.random()
        if r < 0.3:
            t += "." + "".join(rng.choice("0123456789") for _ in range(rng.randint(1, 9)))
        z = rng.random()
        if z < 0.5:
            t += "Z"
        else:
            t += "%s%02d:%02d" % (rng.choice("+-"), rng.randint(0, 23), rng.randint(0, 59))
        m = rng.random()
        if m < 0.05:
            t = t.replace("T%02d" % h, "T%d" % h, 1)  # 1-digit hour (Go accepts)
        elif m < 0.08:
            t = t[:8] + "31" + t[10:]                  # day 31: out of range in short months
        elif m < 0.10:
            t = t[:5] + "02-29" + t[10:]                # leap days
        elif m < 0.12:
            t = t.replace(":", "", 1)                   # malformed
        out.append(t)
    return out


def test_time_parse_vs_datetime():
    import datetime as D
    for t in random_times(4000, 3):
        try:
            got = N.parse_rfc3339(t)
        except N.DecodeError:
            got = None
        want = None
        try:
            core, frac = t[:19], 0
            rest = t[19:]
            if len(t) >= 11 and t[10] == "T" and len(t[11:].split(":")[0]) == 1:
                core = t[:11] + "0" + t[11:18]
                rest = t[18:]
            dt = D.datetime.strptime(core, "%Y-%m-%dT%H:%M:%S")
            if rest.startswith("."):
                k = 1
                while k < len(rest) and rest[k].isdigit():
                    k += 1
                frac = int(rest[1:k].ljust(9, "0"))
                rest = rest[k:]
            if rest == "Z":
                off = 0
            elif len(rest) == 6 and rest[0] in "+-" and rest[3] == ":":
                off = (int(rest[1:3]) * 60 + int(rest[4:6])) * 60 * (1 if rest[0] == "+" else -1)
            else:
                raise ValueError(rest)
            secs = (dt - D.datetime(1970, 1, 1)) // D.timedelta(seconds=1) - off
            want = (secs, frac)
        except ValueError:
            want = None
        assert got == want, (t, got, want)


def test_host_batch_entry_point_matches_oracle():
    """gpudiff_classify_updates_host (the host path over a batch, on several
    threads; the negotiation bench's CPU baseline) equals the oracle."""
    from kcp_amd import gpudiff as G
    cs = C.cases()
    pairs = [(a, b) for _, a, b, _ in cs] * 7
    hp = G.HostPairs(pairs)
    got = hp.classify(threads=4).tolist()
    assert got == [N.classify(a, b) for a, b in pairs]


# ---------------------------------------------------------------- CustomResourceDefinition events (controller.go:186-199)
CRD_EDITS = [
    (b'"acceptedNames":{', b'"AcceptedNames":{'), (b'"acceptedNames":{', b'"acceptedNames":null,"acceptedNames":{'),
    (b'"acceptedNames":{', b'"acceptedNames":{"plural":"zz"},"acceptedNames":{'),
    (b'"acceptedNames":{"plural"', b'"acceptedNames":{"PLURAL"'), (b'"storedVersions":[', b'"storedVersions":[null,'),
    (b'"storedVersions":[', b'"storedVersions":["a","b","c"],"storedVersions":['),
    (b'"storedVersions":[', b'"storedVersions":[1,'), (b'"storedVersions":[', b'"storedVersions":["\\u0076",'),
    (b'"storedVersions":["v1"]', b'"storedVersions":null'), (b'"storedVersions":["v1"]', b'"storedVersions":[]'),
    (b'"storedVersions":[', b'"storedversions":["x"],"storedVersions":['),
    (b',"kind":"W', b',"kind":null,"x":"W'), (b',"kind":"W', b',"kind":5,"x":"W'),
    (b'"listKind":"', b'"listKind":"\\n'), (b'"shortNames":[', b'"shortNames":[null,'),
    (b'"shortNames":[', b'"shortNames":{},"x":['), (b'"categories":[', b'"categories":["a","b","c","d","e","f","g","h",'),
    (b'"conditions":[', b'"conditions":[null,'), (b'"status":{"conditions"', b'"status":{"acceptedNames":"x","conditions"'),
    (b'"status":{"conditions"', b'"status":{"acceptedNames":[],"conditions"'),
    (b'"status":{"conditions"', b'"status":{"extra":{"a":[1,2]},"conditions"'),
    (b'"singular":"', b'"singular":"x","singular":"'), (b'"metadata":{', b'"Metadata":{'),
]


def crd_fuzz_pairs(n, seed):
    pairs, _ = S.crd_population(n, seed=seed, n_props=3)
    rng = random.Random(seed)
    out = []
    for a, b in pairs:
        r = rng.random()
        if r < 0.3:
            x, y = rng.choice(CRD_EDITS)
            b = b.replace(x, y, 1)
        elif r < 0.45:
            x, y = rng.choice(CRD_EDITS)
            a = a.replace(x, y, 1)
        elif r < 0.5:
            a = None
        out.append((a, b))
    return out


@pytest.mark.parametrize("case", C.crd_cases(), ids=lambda c: c[0])
def test_crd_oracle_kat(case):
    name, a, b, want = case
    assert N.classify(a, b, N.KIND_CRD) == want


@pytest.mark.parametrize("case", C.crd_cases(), ids=lambda c: c[0])
def test_crd_host_kat(case):
    name, a, b, want = case
    assert G.negotiate_pair_host(a, b, G.NEG_KIND_CRD) == want


@pytest.mark.parametrize("case", C.kcp_kind_ignores_crd_status(), ids=lambda c: c[0])
def test_kind_selects_typed_status(case):
    """The same CRD documents typed as an APIResourceImport read only status.conditions."""
    name, a, b, want = case
    assert N.classify(a, b, N.KIND_KCP) == want
    assert G.negotiate_pair_host(a, b) == want
    assert G.negotiate_pair_host(a, b, G.NEG_KIND_API) == want


def test_crd_population_matches_design():
    pairs, want = S.crd_population(1500, seed=12)
    assert [N.classify(a, b, N.KIND_CRD) for a, b in pairs] == want.tolist()


def test_crd_host_matches_oracle_fuzz():
    pairs = crd_fuzz_pairs(2500, 20211004 + 73)
    got = G.HostPairs(pairs, G.NEG_KIND_CRD).classify(threads=4).tolist()
    want = [N.classify(a, b, N.KIND_CRD) for a, b in pairs]
    bad = [i for i in range(len(pairs)) if got[i] != want[i]]
    assert not bad, (len(bad), pairs[bad[0]], got[bad[0]], want[bad[0]])
    assert len(set(want)) >= 5  # the edits reach every outcome, DECODE included


def test_mixed_kinds_host_batch():
    """One batch holding both kinds: each pair decoded with its own kind's typed status."""
    api = [(a, b) for _, a, b, _ in C.cases()]
    crd = [(a, b) for _, a, b, _ in C.crd_cases()]
    pairs = [p for ab in zip(api, crd) for p in ab]
    kinds = [k for _ in zip(api, crd) for k in (G.NEG_KIND_API, G.NEG_KIND_CRD)]
    got = G.HostPairs(pairs, kinds).classify(threads=2).tolist()
    assert got == [N.classify(a, b, k) for (a, b), k in zip(pairs, kinds)]
    with pytest.raises(G.GpuDiffError):
        G.HostPairs(pairs[:2], [0, 7]).classify()

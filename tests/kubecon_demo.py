"""The kubecon demo's Deployments, as data (TEST INFRASTRUCTURE): the one
reference-held outcome that pins the splitter roll-up.

The reference's demo applies ``contrib/demo/deployment.yaml`` (a root
``my-deployment`` with ``replicas: 10``) with two clusters registered
(``us-east1``, ``us-west1``); the splitter's ``createLeafs``
(``pkg/reconciler/deployment/deployment.go:127-160``) creates one leaf per
cluster -- ``<root>--<cluster>``, labels ``kcp.dev/cluster=<cluster>`` and
``kcp.dev/owned-by=<root>``, ``replicas = 10 / 2`` (+ the remainder on the
first), an owner reference to the root, resourceVersion cleared -- and each
leaf's status is rolled up into the root (``:41-91``).  The golden transcript
``contrib/demo/kubecon.result:196-208`` shows ``kubectl get deployments`` twice:

    my-deployment             0/10    10           0      (leaves 0/5  5  0)
    my-deployment             10/10   10           10     (leaves 5/5  5  5)

READY is ``status.readyReplicas / spec.replicas``, UP-TO-DATE
``status.updatedReplicas``, AVAILABLE ``status.availableReplicas``.  The rows
below are those lines' values (data); the root and leaf objects are the demo
YAML and createLeafs' output written as API-server JSON (server defaults
omitted: the roll-up reads only labels and the five status counters).  Nothing
here reads /root/reference at run time.
"""
from __future__ import annotations

import copy
import json
from typing import Dict, List, Tuple

ROOT_NAME = "my-deployment"
CLUSTERS = ("us-east1", "us-west1")       # the demo's two kind clusters
NAMESPACE = "demo"                         # kubectl apply ... -n demo (kubecon.result:193)

# contrib/demo/deployment.yaml, as the API server stores it
ROOT = {
    "apiVersion": "apps/v1",
    "kind": "Deployment",
    "metadata": {"name": ROOT_NAME, "namespace": NAMESPACE, "uid": "8d6a3c2e-0000-4000-8000-00000000d3m0",
                 "resourceVersion": "501", "generation": 1, "clusterName": "admin"},
    "spec": {
        "replicas": 10,
        "strategy": {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": 0}},
        "selector": {"matchLabels": {"app.kubernetes.io/name": "app"}},
        "template": {"metadata": {"labels": {"app.kubernetes.io/name": "app"}},
                     "spec": {"containers": [{"name": "nginx", "image": "nginx"}]}},
    },
}

# kubecon.result:196-208, columns READY, UP-TO-DATE, AVAILABLE
TRANSCRIPT = {
    "created": {ROOT_NAME: ("0/10", "10", "0"), ROOT_NAME + "--us-east1": ("0/5", "5", "0"),
                ROOT_NAME + "--us-west1": ("0/5", "5", "0")},
    "available": {ROOT_NAME: ("10/10", "10", "10"), ROOT_NAME + "--us-east1": ("5/5", "5", "5"),
                  ROOT_NAME + "--us-west1": ("5/5", "5", "5")},
}


def create_leafs(root: Dict, clusters=CLUSTERS) -> List[Dict]:
    """deployment.go:127-160: one leaf per cluster."""
    each, rest = divmod(root["spec"]["replicas"], len(clusters))
    out = []
    for index, cl in enumerate(clusters):
        vd = copy.deepcopy(root)
        md = vd["metadata"]
        md["name"] = "%s--%s" % (root["metadata"]["name"], cl)
        md.setdefault("labels", {})
        md["labels"]["kcp.dev/cluster"] = cl
        md["labels"]["kcp.dev/owned-by"] = root["metadata"]["name"]
        vd["spec"]["replicas"] = each + (rest if index == 0 else 0)
        md["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "Deployment", "name": root["metadata"]["name"],
                                  "uid": root["metadata"]["uid"]}]
        md.pop("resourceVersion", None)
        md["uid"] = "leaf-%d" % index
        out.append(vd)
    return out


def leaf_status(replicas: int, phase: str) -> Dict:
    """A leaf's status as the physical cluster reports it (int32 counters, omitempty when 0)."""
    st = {"observedGeneration": 1, "replicas": replicas, "updatedReplicas": replicas}
    if phase == "created":
        st["unavailableReplicas"] = replicas
        st["conditions"] = [{"type": "Progressing", "status": "True", "reason": "ReplicaSetUpdated"},
                            {"type": "Available", "status": "False", "reason": "MinimumReplicasUnavailable"}]
    else:
        st["readyReplicas"] = replicas
        st["availableReplicas"] = replicas
        st["conditions"] = [{"type": "Available", "status": "True", "reason": "MinimumReplicasAvailable"},
                            {"type": "Progressing", "status": "True", "reason": "NewReplicaSetAvailable"}]
    return st


def cache(phase: str) -> Tuple[List[bytes], Dict, List[Dict]]:
    """The splitter's cache at a transcript point: [root, leaf us-east1, leaf us-west1] as JSON."""
    root = copy.deepcopy(ROOT)
    leaves = create_leafs(root)
    for lf in leaves:
        lf["status"] = leaf_status(lf["spec"]["replicas"], phase)
    docs = [json.dumps(d, separators=(",", ":")).encode() for d in [root] + leaves]
    return docs, root, leaves


def kubectl_row(spec_replicas: int, status: Dict) -> Tuple[str, str, str]:
    """kubectl get deployments: READY, UP-TO-DATE, AVAILABLE."""
    return ("%d/%d" % (status.get("readyReplicas", 0), spec_replicas), str(status.get("updatedReplicas", 0)),
            str(status.get("availableReplicas", 0)))


def root_status_from_sums(sums) -> Dict:
    """deployment.go:74-85: the root's five counters = the group's int32 sums."""
    keys = ("replicas", "updatedReplicas", "readyReplicas", "availableReplicas", "unavailableReplicas")
    return dict(zip(keys, [int(x) for x in sums]))

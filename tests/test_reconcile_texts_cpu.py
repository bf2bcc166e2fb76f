"""BatchReconciler.reconcile_texts' host logic on the CPU: the device steps replaced by their checkers.

The reconciler's context (trigger hashing, snapshot, schedule) is a stand-in that hashes with the C restatement
(``oracle/kad_trigger_ref.c``) and schedules with the C oracle (``oracle/ref.py``) on the same packed blobs, so the
CPU suite covers what the text reconcile does around the device — the native trigger prefixes and policy lookup,
the skip decisions, the per-profile unit builds and the annotated write-back — against the dict reconcile on
``objects.py`` (the same stand-in under it). The GPU test (tests/test_gpu_reconcile.py) runs both on the device.
"""

import copy
import json

import numpy as np

from kubeadmiral_amd import objects as O
from kubeadmiral_amd import synth
from kubeadmiral_amd.controller import BatchReconciler
from oracle import ref


class OracleContext:
    """The Context calls BatchReconciler makes, served by the checkers (no device)."""

    def __init__(self):
        self.snap = None
        self.suffix = b""
        self.prefixes = []

    def upload_snapshot(self, snap):
        self.snap = snap

    def update_snapshot(self, delta):  # the host snapshot is committed by the caller; the oracle reads it
        pass

    def run(self, fwk, batch):
        return ref.schedule(self.snap, batch, fwk)

    def trigger_suffix_upload(self, suffix):
        self.suffix = bytes(suffix)

    def trigger_prefixes_upload(self, prefixes):
        self.prefixes = [bytes(p) for p in prefixes]

    def trigger_run(self):
        pass

    def trigger_download(self):
        return np.asarray(ref.trigger_hashes(self.prefixes, self.suffix), np.uint32)


def _workload(seed, n=300):
    ftc, clusters, objs, pols = synth.gen_trigger_workload(np.random.default_rng(seed), n, 16, n_policies=8)
    by_key = {}
    for p in pols:
        if p.spec.auto_migration is not None:
            p.spec.auto_migration.when.pod_unschedulable_for = "2m"
        by_key[(p.namespace, p.name)] = p
    uniq = list(by_key.values())
    uniq[0].spec.scheduling_profile = "p1"
    uniq[1].spec.scheduling_profile = "gone"
    am = [p for p in uniq[2:] if p.spec.auto_migration is not None]
    if am:
        am[0].spec.auto_migration.when.pod_unschedulable_for = None  # reconcile :302 dereferences it
    for o in objs[:4]:
        del o["metadata"]["labels"][O.PROPAGATION_POLICY_NAME_LABEL]
    objs[4]["metadata"]["labels"][O.PROPAGATION_POLICY_NAME_LABEL] = "missing"
    for o in objs[5:12]:
        o["metadata"].setdefault("annotations", {})[O.NO_SCHEDULING_ANNOTATION] = "yes"
    objs[12]["spec"]["template"]["spec"]["replicas"] = "5"
    objs[13]["metadata"]["annotations"] = {"x": 1}
    objs[14]["metadata"].pop("annotations", None)
    return ftc, clusters, objs, by_key, uniq, {"p1": None}


def test_text_reconcile_matches_dict_reconcile_on_the_checkers():
    ftc, clusters, objs, by_key, uniq, profiles = _workload(3)
    texts = [json.dumps(o) for o in objs]
    ptexts = [json.dumps(O.policy_to_json(p)) for p in uniq]
    want_objs = copy.deepcopy(objs)
    want = BatchReconciler(ftc, OracleContext(), native_objects=False).reconcile(want_objs, by_key, clusters, profiles)
    rec = BatchReconciler(ftc, OracleContext())
    got, new = rec.reconcile_texts(texts, ptexts, clusters, profiles)
    stages = set()
    for i, (g, w) in enumerate(zip(got, want)):
        assert (g.stage, g.status) == (w.stage, w.status), (i, g.error, w.error)
        stages.add(g.stage)
        if g.stage == "scheduled":
            assert g.result == w.result and g.modified == w.modified, i
        if g.stage in ("scheduled", "no-scheduling"):
            assert json.loads(new[i]) == want_objs[i], i
        else:
            assert new[i] is None, i
    assert {"scheduled", "no-scheduling", "policy-not-found", "trigger-error", "profile-not-found"} <= stages

    # the new texts reconcile as unchanged; bad texts and a policy that does not decode are reported per object
    texts2 = [n if n is not None else t for n, t in zip(new, texts)] + ["{", "[1]"]
    again, new2 = rec.reconcile_texts(texts2, ptexts, clusters, profiles)
    for i, g in enumerate(again[:len(objs)]):
        if got[i].stage in ("scheduled", "no-scheduling"):
            assert g.stage == "unchanged" and new2[i] is None, i
    assert [g.stage for g in again[len(objs):]] == ["bad-json", "bad-json"]


def test_text_reconcile_policy_that_does_not_decode():
    ftc, clusters, objs, by_key, uniq, profiles = _workload(4, n=60)
    bad = json.loads(json.dumps(O.policy_to_json(uniq[2])))
    bad["spec"]["maxClusters"] = "3"  # a string where the spec holds an int: the informer could not decode it
    ptexts = [json.dumps(O.policy_to_json(p)) for p in uniq]
    ptexts[2] = json.dumps(bad)
    got, new = BatchReconciler(ftc, OracleContext()).reconcile_texts([json.dumps(o) for o in objs], ptexts,
                                                                    clusters, profiles)
    name = uniq[2].name
    hit = 0
    for o, g, t in zip(objs, got, new):
        if (o["metadata"].get("labels") or {}).get(O.PROPAGATION_POLICY_NAME_LABEL) == name:
            assert g.stage == "policy-error" and t is None
            hit += 1
    assert hit

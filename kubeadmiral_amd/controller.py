"""Batched reconcile: the scheduler controller's per-object loop, one GPU pass per batch.

``Scheduler.reconcile`` (pkg/controllers/scheduler/scheduler.go:240-309) runs
per federated object on ``--worker-count`` goroutines: look up the policy and
profile (``prepareToSchedule``, :311-443), compute the scheduling-trigger hash
and skip the object if it is unchanged (:394-421), build the SchedulingUnit and
call ``ScheduleAlgorithm.Schedule`` (``schedule``, :445-521), then write the
result back (``applySchedulingResult``, :632-695). :class:`BatchReconciler`
takes a whole batch of objects through the same steps with the two hot
stages batched on the GPU — every object's trigger hash in one
``kad_trigger_run`` and every SchedulingUnit of one framework in one
``kad_schedule`` — and returns, per object, what the reference's reconcile
would have done (worker status, whether it scheduled, whether the object
changed). Objects are mutated in place exactly as the reference mutates its
deep copy before ``Update``.

Out of scope (no API server here): pending-controller bookkeeping
(``pendingcontrollers``), events, the ``Update`` call itself, webhook plugins
(rejected by :class:`~kubeadmiral_amd.framework.Framework`), deletion
timestamps. Policies and profiles are looked up in the dicts the caller passes
(the informer caches of the reference).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from . import framework as F
from . import objects as O
from . import types as T
from .runtime import BatchScheduler, Context, TriggerHasher

STATUS_ALL_OK = "AllOK"   # worker.StatusAllOK
STATUS_ERROR = "Error"    # worker.StatusError


@dataclass
class ReconcileOutcome:
    status: str                                  # STATUS_ALL_OK / STATUS_ERROR
    stage: str = ""                              # where the reconcile ended (see BatchReconciler.reconcile)
    scheduled: bool = False                      # a result was computed and applied
    modified: bool = False                       # applySchedulingResult changed the object
    result: Optional[T.ScheduleResult] = None
    error: str = ""


class BatchReconciler:
    """Scheduler.reconcile for a batch of federated objects of one FederatedTypeConfig."""

    def __init__(self, type_config: O.FederatedTypeConfig, ctx: Optional[Context] = None, device: int = 0,
                 native_objects: bool = True):
        """``native_objects``: SchedulingUnits built and results applied by the library (kad_units_from_objects /
        kad_apply_results, include/kad_objects.h) over the objects' JSON, instead of objects.py per object."""
        self.type_config = type_config
        self.native_objects = native_objects
        self.ctx = ctx if ctx is not None else Context(device)
        self.hasher = TriggerHasher(self.ctx)
        self.scheduler = BatchScheduler(self.ctx)
        self._clusters_key = None

    def _framework(self, profile: Optional[dict]) -> F.Framework:
        """createFramework (scheduler.go:492, profile.go:52-82): default plugins + the profile's changes."""
        return F.Framework(F.apply_profile(F.default_enabled_plugins(), profile))

    def reconcile(self, objs: Sequence[dict], policies: Dict[Tuple[str, str], O.PropagationPolicy],
                  clusters: List[T.FederatedCluster], profiles: Optional[Dict[str, Optional[dict]]] = None
                  ) -> List[ReconcileOutcome]:
        """Reconcile every object against the joined ``clusters``.

        ``policies`` maps (namespace, name) → policy ("" namespace for
        ClusterPropagationPolicies); ``profiles`` maps SchedulingProfile name →
        its ``spec.plugins`` dict (None = no changes). Stages recorded in
        ``ReconcileOutcome.stage``: ``policy-not-found``, ``profile-not-found``,
        ``trigger-error``, ``unchanged`` (trigger hash equal), ``no-scheduling``,
        ``unit-error``, ``framework-error``, ``schedule-error``, ``apply-error``,
        ``scheduled``.
        """
        profiles = profiles or {}
        out: List[Optional[ReconcileOutcome]] = [None] * len(objs)
        ctx_pol: List[Optional[O.PropagationPolicy]] = [None] * len(objs)
        ctx_prof: List[Optional[str]] = [None] * len(objs)

        # prepareToSchedule :349-392 — policy and profile lookup
        live = []
        for i, obj in enumerate(objs):
            key = O.matched_policy_key(obj, self.type_config.namespaced)
            if key is not None:
                pol = policies.get(key)
                if pol is None:
                    out[i] = ReconcileOutcome(STATUS_ALL_OK, "policy-not-found")
                    continue
                ctx_pol[i] = pol
                name = pol.spec.scheduling_profile
                if name:
                    if name not in profiles:
                        out[i] = ReconcileOutcome(STATUS_ALL_OK, "profile-not-found")
                        continue
                    ctx_prof[i] = name
            live.append(i)

        # :394-421 — trigger hashes for the whole batch in one GPU pass
        key = T.clusters_fingerprint(clusters)  # content (labels, taints, API resources), not the list object
        if key != self._clusters_key:
            self.hasher.set_clusters(clusters)
            self._clusters_key = key
        hashed, prefixes = [], []
        for i in live:
            try:
                prefixes.append(O.trigger_prefix(self.type_config, objs[i], ctx_pol[i]))
                hashed.append(i)
            except O.ObjectError as e:
                out[i] = ReconcileOutcome(STATUS_ERROR, "trigger-error", error=str(e))
        self.ctx.trigger_prefixes_upload(prefixes)
        self.ctx.trigger_run()
        hashes = self.ctx.trigger_download()
        to_schedule = []
        for i, h in zip(hashed, hashes.tolist()):
            changed = O.add_annotation(objs[i], O.SCHEDULING_TRIGGER_HASH_ANNOTATION, O.format_trigger_hash(h))
            if not changed:
                out[i] = ReconcileOutcome(STATUS_ALL_OK, "unchanged")
            elif (O.get_annotations(objs[i]) or {}).get(O.NO_SCHEDULING_ANNOTATION, ""):
                out[i] = ReconcileOutcome(STATUS_ALL_OK, "no-scheduling")
            else:
                to_schedule.append(i)

        if self.native_objects:
            self._schedule_and_apply_native(objs, to_schedule, ctx_pol, ctx_prof, profiles, clusters, out)
            return out  # type: ignore[return-value]

        # schedule :445-521 — units grouped by framework, one GPU batch per framework
        results: Dict[int, T.ScheduleResult] = {}
        groups: Dict[Optional[str], List[Tuple[int, T.SchedulingUnit]]] = {}
        for i in to_schedule:
            if ctx_pol[i] is None:
                results[i] = T.ScheduleResult({})  # :454-467 no policy: schedule to no clusters
                continue
            try:
                su = O.scheduling_unit_for_fed_object(self.type_config, objs[i], ctx_pol[i])
            except (O.ObjectError, O.GoPanic) as e:
                out[i] = ReconcileOutcome(STATUS_ERROR, "unit-error", error=str(e))
                continue
            groups.setdefault(ctx_prof[i], []).append((i, su))
        for prof_name, members in groups.items():
            try:
                fwk = self._framework(profiles.get(prof_name) if prof_name else None)
            except F.FrameworkError as e:
                for i, _ in members:
                    out[i] = ReconcileOutcome(STATUS_ERROR, "framework-error", error=str(e))
                continue
            res = self.scheduler.schedule(fwk, [su for _, su in members], clusters)
            for (i, _), r in zip(members, res):
                if isinstance(r, T.ScheduleError):
                    out[i] = ReconcileOutcome(STATUS_ERROR, "schedule-error", error=str(r))
                else:
                    results[i] = r

        # reconcile :291-308 + persistSchedulingResult → applySchedulingResult
        for i, r in results.items():
            pol = ctx_pol[i]
            follower = False
            threshold = None
            try:
                if pol is not None:
                    follower = not pol.spec.disable_follower_scheduling
                    am = pol.spec.auto_migration
                    if am is not None:
                        if am.when.pod_unschedulable_for is None:
                            raise O.GoPanic("invalid memory address or nil pointer dereference")  # :302
                        threshold = O.parse_duration(am.when.pod_unschedulable_for)
                modified = O.apply_scheduling_result(self.type_config, objs[i], r, follower, threshold)
            except (O.ObjectError, O.GoPanic) as e:
                out[i] = ReconcileOutcome(STATUS_ERROR, "apply-error", result=r, error=str(e))
                continue
            out[i] = ReconcileOutcome(STATUS_ALL_OK, "scheduled", True, modified, r)
        return out  # type: ignore[return-value]

    # ------------------------------------------------------------------ the native object path
    @staticmethod
    def _apply_params(pol):
        """(follower, threshold ns) of reconcile :291-308; raises like the reference."""
        if pol is None:
            return False, None
        threshold = None
        am = pol.spec.auto_migration
        if am is not None:
            if am.when.pod_unschedulable_for is None:
                raise O.GoPanic("invalid memory address or nil pointer dereference")  # :302
            threshold = O.parse_duration(am.when.pod_unschedulable_for)
        return not pol.spec.disable_follower_scheduling, threshold

    def _schedule_and_apply_native(self, objs, to_schedule, ctx_pol, ctx_prof, profiles, clusters, out):
        """The schedule and apply stages over the objects' JSON: per framework one kad_units_from_objects, one
        packed GPU batch, then one kad_apply_results for every object with a result."""
        import json

        from . import columns as K
        from .results import to_schedule_result_cols

        results: Dict[int, T.ScheduleResult] = {}
        groups: Dict[Optional[str], List[int]] = {}
        for i in to_schedule:
            if ctx_pol[i] is None:
                results[i] = T.ScheduleResult({})  # :454-467 no policy: schedule to no clusters
                continue
            groups.setdefault(ctx_prof[i], []).append(i)
        pol_index: Dict[int, int] = {}
        pol_json: List[dict] = []
        for i in to_schedule:
            if ctx_pol[i] is not None and id(ctx_pol[i]) not in pol_index:
                pol_index[id(ctx_pol[i])] = len(pol_json)
                pol_json.append(O.policy_to_json(ctx_pol[i]))
        pol_text = [json.dumps(p) for p in pol_json]
        names: List[str] = []
        for prof_name, members in groups.items():
            try:
                fwk = self._framework(profiles.get(prof_name) if prof_name else None)
            except F.FrameworkError as e:
                for i in members:
                    out[i] = ReconcileOutcome(STATUS_ERROR, "framework-error", error=str(e))
                continue
            built = K.units_from_objects(self.type_config, [json.dumps(objs[i]) for i in members], pol_text,
                                         [pol_index[id(ctx_pol[i])] for i in members])
            ok = []
            for k, i in enumerate(members):
                if built.status[k] == K.OBJ_OK:
                    ok.append((i, int(built.unit_index[k])))
                else:
                    out[i] = ReconcileOutcome(STATUS_ERROR, "unit-error", error=built.messages[k])
            if not ok:
                continue
            res, snap = self.scheduler.schedule_columns(fwk, built.cols, clusters)
            names = snap.names
            for i, w in ok:
                r = to_schedule_result_cols(res, w, built.cols, names)
                if isinstance(r, T.ScheduleError):
                    out[i] = ReconcileOutcome(STATUS_ERROR, "schedule-error", error=str(r))
                else:
                    results[i] = r

        # reconcile :291-308 + persistSchedulingResult → applySchedulingResult, one native pass
        todo, follower, threshold = [], [], []
        for i, r in sorted(results.items()):
            try:
                f, t = self._apply_params(ctx_pol[i])
            except (O.ObjectError, O.GoPanic) as e:
                out[i] = ReconcileOutcome(STATUS_ERROR, "apply-error", result=r, error=str(e))
                continue
            todo.append(i)
            follower.append(f)
            threshold.append(t)
        if not todo:
            return
        table = list(names)
        at = {n: k for k, n in enumerate(table)}
        off, cl, rep = [0], [], []
        for i in todo:
            for n, v in (results[i].suggested_clusters or {}).items():
                if n not in at:  # a sticky result's cluster that left the snapshot
                    at[n] = len(table)
                    table.append(n)
                cl.append(at[n])
                rep.append(-1 if v is None else v)
            off.append(len(cl))
        st, modified, texts, msgs, fields = K.apply_results(self.type_config, [json.dumps(objs[i]) for i in todo],
                                                            table, off, cl, rep, follower, threshold, with_fields=True)
        for k, i in enumerate(todo):
            r = results[i]
            if st[k] != K.APPLY_OK:
                out[i] = ReconcileOutcome(STATUS_ERROR, "apply-error", result=r, error=msgs[k])
                continue
            if modified[k]:  # the written fields are set in place, as the reference mutates its deep copy
                for (a, b), v in zip(K.APPLY_FIELDS, fields[k]):
                    if v is not None:
                        objs[i].setdefault(a, {})[b] = json.loads(v)
            out[i] = ReconcileOutcome(STATUS_ALL_OK, "scheduled", True, bool(modified[k]), r)

    # ------------------------------------------------------------------ the reconcile over JSON texts
    def reconcile_texts(self, texts: Sequence, policies: Sequence, clusters: List[T.FederatedCluster],
                        profiles: Optional[Dict[str, Optional[dict]]] = None
                        ) -> Tuple[List[ReconcileOutcome], List[Optional[bytes]]]:
        """:meth:`reconcile` over the federated objects' JSON texts (what an informer or a watch hands over),
        with every per-object step native: the trigger JSON's object part (kad_trigger_prefixes), the trigger
        hashes (kad_trigger_run), the SchedulingUnits (kad_units_from_objects), the schedule (kad_schedule) and
        the write-back with the trigger annotation (kad_apply_results). ``policies``: the
        (Cluster)PropagationPolicies' JSON; each object's policy is found through its labels as
        MatchedPolicyKey does. Returns the outcomes (stages as :meth:`reconcile`, plus ``bad-json`` and
        ``policy-error`` for texts that do not decode) and per object its new text — the deep copy the
        reference goes on to Update (``scheduled``) or holds when it skips scheduling (``no-scheduling``) —
        or None where the reconcile left the object as it was or dropped its copy on an error."""
        import json

        from . import columns as K
        from .results import to_schedule_result_cols

        profiles = profiles or {}
        ot, pt = K._texts(texts), K._texts(policies)
        n = len(ot)
        out: List[Optional[ReconcileOutcome]] = [None] * n
        new_text: List[Optional[bytes]] = [None] * n
        pols: List[Optional[O.PropagationPolicy]] = []
        for t in pt:  # a handful: decoded once for the profile name and the apply parameters
            try:
                pols.append(O.PropagationPolicy.from_json(json.loads(t)))
            except Exception:  # noqa: BLE001 — the native lookup reports it as KAD_OBJ_POLICY_ERROR
                pols.append(None)
        tr = K.trigger_prefixes(self.type_config, ot, pt)

        # prepareToSchedule :349-392 — policy and profile lookup, then the trigger JSON (:394-399)
        hashed: List[int] = []
        pol_of = tr.policy_index
        for i in range(n):
            st = int(tr.status[i])
            if st == K.OBJ_POLICY_NOT_FOUND:
                out[i] = ReconcileOutcome(STATUS_ALL_OK, "policy-not-found")
                continue
            if st == K.OBJ_BAD_JSON:
                out[i] = ReconcileOutcome(STATUS_ERROR, "bad-json", error=tr.messages[i])
                continue
            if st == K.OBJ_POLICY_ERROR:
                out[i] = ReconcileOutcome(STATUS_ERROR, "policy-error", error=tr.messages[i])
                continue
            p = pols[pol_of[i]] if pol_of[i] >= 0 else None
            if p is None and pol_of[i] >= 0:  # the library decoded it but objects.py did not: not scheduled on
                out[i] = ReconcileOutcome(STATUS_ERROR, "policy-error", error="policy does not decode")
                continue
            if p is not None and p.spec.scheduling_profile and p.spec.scheduling_profile not in profiles:
                out[i] = ReconcileOutcome(STATUS_ALL_OK, "profile-not-found")
                continue
            if st != K.OBJ_OK:
                out[i] = ReconcileOutcome(STATUS_ERROR, "trigger-error", error=tr.messages[i])
                continue
            hashed.append(i)

        # :394-421 — the hashes in one GPU pass; AddAnnotation's "changed" against the current annotation
        key = T.clusters_fingerprint(clusters)
        if key != self._clusters_key:
            self.hasher.set_clusters(clusters)
            self._clusters_key = key
        self.ctx.trigger_prefixes_upload([tr.prefixes[i] for i in hashed])
        self.ctx.trigger_run()
        hashes = self.ctx.trigger_download()
        trig: List[Optional[str]] = [None] * n
        ann_only = [False] * n
        to_schedule: List[int] = []
        for i, h in zip(hashed, hashes.tolist()):
            hv = O.format_trigger_hash(h)
            if tr.flags[i] & K.TRIG_HAS_HASH and tr.current_hash[i] == hv:
                out[i] = ReconcileOutcome(STATUS_ALL_OK, "unchanged")
                continue
            trig[i] = hv
            if tr.flags[i] & K.TRIG_NO_SCHEDULING:
                out[i] = ReconcileOutcome(STATUS_ALL_OK, "no-scheduling")
                ann_only[i] = True
            else:
                to_schedule.append(i)

        # schedule :445-521 — per framework one native unit build and one GPU batch
        results: Dict[int, T.ScheduleResult] = {}
        groups: Dict[Optional[str], List[int]] = {}
        for i in to_schedule:
            p = pols[pol_of[i]] if pol_of[i] >= 0 else None
            if p is None:
                results[i] = T.ScheduleResult({})  # :454-467 no policy: schedule to no clusters
                continue
            groups.setdefault(p.spec.scheduling_profile or None, []).append(i)
        # the unit is built from the object after AddAnnotation (:407); that only differs where the annotation
        # replaced annotations that were not a string map (the typed view would reject the old ones)
        unit_text = {}
        fix = [i for i in to_schedule if tr.flags[i] & K.TRIG_ANN_NOT_MAP]
        if fix:
            a = K.apply_results_ex(self.type_config, [ot[i] for i in fix], [], [0] * (len(fix) + 1), [], [],
                                   trigger=[trig[i] for i in fix], ann_only=[True] * len(fix))
            unit_text = {i: a.texts[k] for k, i in enumerate(fix) if a.status[k] == K.APPLY_OK}
        names: List[str] = []
        for prof_name, members in groups.items():
            try:
                fwk = self._framework(profiles.get(prof_name) if prof_name else None)
            except F.FrameworkError as e:
                for i in members:
                    out[i] = ReconcileOutcome(STATUS_ERROR, "framework-error", error=str(e))
                continue
            built = K.units_from_objects(self.type_config, [unit_text.get(i, ot[i]) for i in members], pt,
                                         [int(pol_of[i]) for i in members])
            ok = []
            for k, i in enumerate(members):
                if built.status[k] == K.OBJ_OK:
                    ok.append((i, int(built.unit_index[k])))
                else:
                    out[i] = ReconcileOutcome(STATUS_ERROR, "unit-error", error=built.messages[k])
            if not ok:
                continue
            res, snap = self.scheduler.schedule_columns(fwk, built.cols, clusters)
            names = snap.names
            for i, w in ok:
                r = to_schedule_result_cols(res, w, built.cols, names)
                if isinstance(r, T.ScheduleError):
                    out[i] = ReconcileOutcome(STATUS_ERROR, "schedule-error", error=str(r))
                else:
                    results[i] = r

        # reconcile :291-308 + applySchedulingResult, and the no-scheduling objects' annotation, in one pass
        todo, follower, threshold = [], [], []
        params: Dict[int, object] = {}  # per policy: (follower, threshold) or the error
        for i in range(n):
            if ann_only[i]:
                todo.append(i)
                follower.append(False)
                threshold.append(None)
            elif i in results:
                pi = int(pol_of[i])
                if pi not in params:
                    try:
                        params[pi] = self._apply_params(pols[pi] if pi >= 0 else None)
                    except (O.ObjectError, O.GoPanic) as e:
                        params[pi] = e
                ft = params[pi]
                if isinstance(ft, Exception):
                    out[i] = ReconcileOutcome(STATUS_ERROR, "apply-error", result=results[i], error=str(ft))
                    continue
                f, t = ft
                todo.append(i)
                follower.append(f)
                threshold.append(t)
        if not todo:
            return out, new_text  # type: ignore[return-value]
        table = list(names)
        at = {c: k for k, c in enumerate(table)}
        off, cl, rep = [0], [], []
        for i in todo:
            if not ann_only[i]:
                for c, v in (results[i].suggested_clusters or {}).items():
                    if c not in at:  # a sticky result's cluster that left the snapshot
                        at[c] = len(table)
                        table.append(c)
                    cl.append(at[c])
                    rep.append(-1 if v is None else v)
            off.append(len(cl))
        a = K.apply_results_ex(self.type_config, [ot[i] for i in todo], table, off, cl, rep, follower, threshold,
                               trigger=[trig[i] for i in todo], ann_only=[ann_only[i] for i in todo],
                               with_fields=False)
        for k, i in enumerate(todo):
            if a.status[k] != K.APPLY_OK:
                out[i] = ReconcileOutcome(STATUS_ERROR, "apply-error", result=results.get(i), error=a.messages[k])
                continue
            if a.changed[k]:
                new_text[i] = a.texts[k]
            if not ann_only[i]:
                out[i] = ReconcileOutcome(STATUS_ALL_OK, "scheduled", True, bool(a.modified[k]), results[i])
        return out, new_text  # type: ignore[return-value]

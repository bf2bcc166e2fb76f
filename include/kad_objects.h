/*
 * kad_objects.h — the host side of the batch scheduler's object formats in
 * libkad.so, for a batch of federated objects as
 * JSON text:
 *   f2  kad_units_from_objects — objects + the (Cluster)PropagationPolicies they
 *       name → the kad_su_columns that kad_pack_batch packs;
 *   f3  kad_apply_results — kad_schedule's results written back into the
 *       objects (placements, replica overrides, annotations).
 *
 * Replaces, per object, what the reference's scheduler controller does before
 * Schedule (pkg/controllers/scheduler/scheduler.go:349-392, 445-467):
 *   * MatchedPolicyKey (scheduler/util.go:37-49) and the policy lookup;
 *   * schedulingUnitForFedObject (schedulingunit.go:38-163) with every
 *     annotation override (:224-668): scheduling mode, sticky cluster, cluster
 *     selector, affinity, tolerations, max clusters, placements (cluster names,
 *     min / max replicas, weights), auto-migration info, and the current
 *     clusters from spec.placements + the global scheduler's replica overrides
 *     (getCurrentReplicasFromObject :181-222, util/overrides.go:68-112).
 * Decoding follows Go 1.19 encoding/json where it changes the outcome
 * (exact-then-case-folded field names, null, integer ranges, the sorted key
 * order of runtime.DefaultUnstructuredConverter) — the same rules as
 * kubeadmiral_amd/gojson.py, whose restatement (kubeadmiral_amd/objects.py)
 * the parity tests compare against field by field
 * (tests/test_native_objects.py) together with the reference's own
 * schedulingunit table (tests/golden/schedulingunit.json).
 *
 * Objects are independent: they are parsed and decoded on the library's
 * worker threads; the string table is interned in object order, so the
 * columns are the same for any thread count.
 */
#ifndef KAD_OBJECTS_H
#define KAD_OBJECTS_H

#include <stddef.h>
#include <stdint.h>

#include "kad_pack.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The FederatedTypeConfig fields the scheduler reads (types_federatedtypeconfig.go). */
typedef struct kad_type_config {
  const char* group;
  const char* version;
  const char* kind;
  const char* plural_name;
  int32_t namespaced;          /* Spec.Scope == Namespaced                                  */
  const char* replicas_spec;   /* Spec.PathDefinition.ReplicasSpec: dot path under spec.template, "" none */
} kad_type_config;

/* per-object outcome */
#define KAD_OBJ_OK 0               /* a SchedulingUnit was built (columns row unit_index[i])          */
#define KAD_OBJ_NO_POLICY 1        /* no policy label: the reference schedules to no clusters (:454-467) */
#define KAD_OBJ_POLICY_NOT_FOUND 2 /* the labelled policy is not in `policies` (:359-372)              */
#define KAD_OBJ_UNIT_ERROR 3       /* schedulingUnitForFedObject returns an error                     */
#define KAD_OBJ_UNIT_PANIC 4       /* the reference panics (a non-float64 replicas override value)    */
#define KAD_OBJ_BAD_JSON 5         /* the object's text is not a JSON object                          */
#define KAD_OBJ_POLICY_ERROR 6     /* the matched policy's spec does not decode (json.Unmarshal error) */

typedef struct kad_units kad_units;

/* Build the SchedulingUnits of `objects` (JSON texts of federated objects).
 * `policies`: JSON texts of PropagationPolicies (metadata.namespace set) and
 * ClusterPropagationPolicies (no namespace), keyed by (namespace, name) as the
 * informer caches are. `policy_of` NULL: each object's policy is found through
 * its labels (MatchedPolicyKey); else policy_of[i] is object i's policy index
 * (-1: none — a caller that did the lookup itself; any other value outside
 * [0, policies->n) is KAD_EINVAL). Every kad_strs must have offsets starting
 * at 0 and never decreasing (else KAD_EINVAL). `threads` <= 0: every
 * worker of the library's pool.
 * Returns KAD_OK with *out set (free with kad_units_free) — per-object failures
 * are statuses, not errors — or KAD_EINVAL / KAD_ENOMEM. */
int kad_units_from_objects(const kad_type_config* tc, const kad_strs* objects, const kad_strs* policies,
                           const int32_t* policy_of, int threads, kad_units** out);
/* Views into *u (valid until kad_units_free): the columns of the OK objects in object order, per object
 * its status and its row in the columns (-1 unless OK), and the matched policy's index (-1 none). */
int kad_units_view(const kad_units* u, kad_su_columns* cols, const int32_t** status, const int32_t** unit_index,
                   const int32_t** policy_index);
/* The message of object i's failure ("" when it has none); valid until kad_units_free. */
const char* kad_units_message(const kad_units* u, int32_t i);
void kad_units_free(kad_units* u);

/* ------------------------------------------------------------ row f3
 * applySchedulingResult (scheduler.go:632-695) for a batch: each object's
 * placement for the global scheduler (util.SetPlacementClusterNames,
 * util/placement.go:44-59), its replica overrides (UpdateReplicasOverride /
 * OverrideUpdateNeeded / updateOverridesMap, scheduler/util.go:71-185;
 * util.SetOverrides, util/overrides.go:114-169) and the follower-scheduling /
 * pod-unschedulable-threshold annotations. Results in kad_results_download's
 * form: object i's clusters are res_cluster[res_off[i] .. res_off[i+1]) (ids
 * into `cluster_names`, the snapshot order) with res_replicas (-1: nil,
 * Duplicate mode); follower[i]: !DisableFollowerScheduling; threshold_ns[i]:
 * the policy's AutoMigration.When.PodUnschedulableFor (INT64_MIN: no
 * auto-migration; NULL: none for every object). A modified object comes back
 * as json.Marshal of its unstructured map (keys sorted, Go string escaping
 * and float64 formatting); an unchanged or failed one as its input text. */
#define KAD_APPLY_OK 0       /* applied; modified[i] says whether the object changed                  */
#define KAD_APPLY_ERROR 1    /* applySchedulingResult returns an error (the object is returned as it was) */
#define KAD_APPLY_PANIC 2    /* the reference panics (SetOverrides on an object whose spec is nil)     */
#define KAD_APPLY_BAD_JSON 3 /* the object's text is not a JSON object                                 */

typedef struct kad_applied kad_applied;

int kad_apply_results(const kad_type_config* tc, const kad_strs* objects, const kad_strs* cluster_names,
                      const int32_t* res_off, const int32_t* res_cluster, const int64_t* res_replicas,
                      const uint8_t* follower, const int64_t* threshold_ns, const kad_strs* trigger,
                      const uint8_t* ann_only, int threads, kad_applied** out);
/* `trigger` (may be NULL): per object the scheduling-trigger-hash annotation value the reconcile adds first
 * (annotation.AddAnnotation, scheduler.go:407-417; "" none); `ann_only` (may be NULL): per object 1 = only that
 * annotation, no result to apply (the reconcile's no-scheduling / error stages).
 * Views into *a (valid until kad_applied_free): per object its status, applySchedulingResult's "modified",
 * whether the text changed at all (modified, or the trigger annotation), and its text. */
int kad_applied_view(const kad_applied* a, const int32_t** status, const uint8_t** modified, const uint8_t** changed,
                     kad_strs* texts);
/* The written fields alone, 3 strings per object (3i: spec.placements, 3i+1: spec.overrides, 3i+2:
 * metadata.annotations): the field's new JSON value, "" where it was not written — what a caller holding the
 * object decoded (or sending a patch) needs instead of re-reading the whole text. */
int kad_applied_fields(const kad_applied* a, kad_strs* fields);
const char* kad_applied_message(const kad_applied* a, int32_t i);
void kad_applied_free(kad_applied* a);

/* ------------------------------------------------------------ row f4 (host side)
 * The object part of computeSchedulingTriggerHash (schedulingtriggers.go:106-134) for a batch of object texts —
 * the bytes kad_trigger_prefixes_upload (kad_sched.h) takes — with MatchedPolicyKey + the policy lookup (or
 * `policy_of`, as in kad_units_from_objects), per object its status (KAD_OBJ_OK, _POLICY_NOT_FOUND,
 * _POLICY_ERROR, _BAD_JSON, _UNIT_ERROR = getReplicaCount's error), the matched policy (-1 none), the current
 * value of the kubeadmiral.io/scheduling-trigger-hash annotation and the flags below. */
#define KAD_TRIG_HAS_HASH 1u      /* the annotations (a string map) hold a trigger hash     */
#define KAD_TRIG_NO_SCHEDULING 2u /* kubeadmiral.io/no-scheduling is set (non-empty)         */
#define KAD_TRIG_ANN_NOT_MAP 4u   /* metadata.annotations is set but not a string map: the trigger annotation
                                   * replaces it, so the SchedulingUnit is built from the annotated text */

typedef struct kad_trigger_objs kad_trigger_objs;

int kad_trigger_prefixes(const kad_type_config* tc, const kad_strs* objects, const kad_strs* policies,
                         const int32_t* policy_of, int threads, kad_trigger_objs** out);
int kad_trigger_objs_view(const kad_trigger_objs* t, const int32_t** status, const int32_t** policy_index,
                          const uint8_t** flags, kad_strs* prefixes, kad_strs* current_hash);
const char* kad_trigger_objs_message(const kad_trigger_objs* t, int32_t i);
void kad_trigger_objs_free(kad_trigger_objs* t);

#ifdef __cplusplus
}
#endif
#endif /* KAD_OBJECTS_H */

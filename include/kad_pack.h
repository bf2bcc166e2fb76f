/*
 * kad_pack.h — native batch packer of libkad.so: a batch of SchedulingUnits in
 * columnar form → the batch blob of kad_sched.h (kad_batch_upload /
 * kad_schedule_batch).
 *
 * The reference builds one framework.SchedulingUnit per object
 * (pkg/controllers/scheduler/schedulingunit.go:38-163) and hands it to
 * Schedule by value (core/generic_scheduler.go:92). A cgo shim fills
 * kad_su_columns from a []SchedulingUnit (one pass of slice appends, strings
 * by reference into one string table) and this packer does everything the
 * reference re-derives per (unit, cluster) pair once per batch: interning
 * against the snapshot vocabulary, labels.NewRequirement validation
 * (apimachinery v0.26.6), ClusterSelector / affinity programs
 * (util/clusterselector/util.go:31-132), toleration sets resolved into
 * tolerated-taint masks (corev1 Toleration.ToleratesTaint, framework/util.go:
 * 406-450), placement / current / preference lists, su.Key() bytes
 * (framework/types.go:123-128) and the output slot bounds.
 *
 * The blob is byte-identical to kubeadmiral_amd/pack.py Batch for the same
 * units (tests/test_native_pack.py), which the oracle tests pin.
 */
#ifndef KAD_PACK_H
#define KAD_PACK_H

#include <stddef.h>
#include <stdint.h>

#include "kad_sched.h"

#ifdef __cplusplus
extern "C" {
#endif

/* n strings; string i = bytes[off[i] .. off[i+1]) (off has n+1 entries) */
typedef struct kad_strs {
  int32_t n;
  const int64_t* off;
  const uint8_t* bytes;
} kad_strs;

/* ---------------------------------------------------- snapshot vocabulary
 * What the batch packer interns against: the ids the snapshot blob was
 * packed with (kubeadmiral_amd/pack.py Snapshot).                          */
typedef struct kad_pack_vocab {
  kad_strs cluster_names;   /* snapshot order                                  */
  kad_strs scalar_names;    /* by scalar id                                    */
  kad_strs gvk_group, gvk_version, gvk_kind; /* by GVK id (same n)             */
  kad_strs label_keys;      /* by label key id                                 */
  const int32_t* label_val_off; /* [n_keys + 1]: values of key k are label_vals[label_val_off[k] ..) by value id */
  kad_strs label_vals;
  kad_strs taint_key, taint_value, taint_effect; /* taint definitions by taint id (one per occurrence) */
  int32_t n_taint_words;    /* TW of the snapshot                              */
  uint64_t fingerprint;     /* kad_snapshot_header.fingerprint                 */
} kad_pack_vocab;

/* ------------------------------------------------------ columnar units
 * All strings are ids into `str`. CSR arrays: *_off has n_units + 1 entries
 * (terms: n_terms + 1, ...). Maps keep their iteration order (the order the
 * reference's map iteration would have; only output byte order depends on it,
 * never a result). */
#define KAD_SU_DUPLICATE (1u << 0)          /* SchedulingMode == Duplicate                      */
#define KAD_SU_STICKY (1u << 1)             /* StickyCluster                                    */
#define KAD_SU_AVOID_DISRUPTION (1u << 2)   /* AvoidDisruption                                  */
#define KAD_SU_HAS_DESIRED (1u << 3)        /* DesiredReplicas != nil                           */
#define KAD_SU_HAS_MAX_CLUSTERS (1u << 4)   /* MaxClusters != nil                               */
#define KAD_SU_HAS_AUTO_MIGRATION (1u << 5) /* AutoMigration != nil                             */
#define KAD_SU_KEEP_UNSCHED (1u << 6)       /* AutoMigration.KeepUnschedulableReplicas          */
#define KAD_SU_HAS_CLUSTER_AFFINITY (1u << 7) /* Affinity != nil && Affinity.ClusterAffinity != nil */
#define KAD_SU_HAS_REQUIRED (1u << 8)       /* ...ClusterAffinity.RequiredDuringScheduling... != nil */

typedef struct kad_su_columns {
  int32_t n_units;
  kad_strs str;
  /* per unit */
  const int32_t* group;
  const int32_t* version;
  const int32_t* kind;
  const int32_t* namespace_;     /* su.Key() = namespace + "/" + name, or name when namespace == "" */
  const int32_t* name;
  const uint32_t* flags;         /* KAD_SU_* */
  const int64_t* desired;        /* *DesiredReplicas   (KAD_SU_HAS_DESIRED)      */
  const int64_t* max_clusters;   /* *MaxClusters       (KAD_SU_HAS_MAX_CLUSTERS) */
  const int64_t* req_cpu;        /* ResourceRequest.MilliCPU */
  const int64_t* req_mem;        /* .Memory */
  const int64_t* req_eph;        /* .EphemeralStorage */
  /* ResourceRequest.ScalarResources */
  const int32_t* scalar_off; const int32_t* scalar_name; const int64_t* scalar_val;
  /* Tolerations: key, operator, value, effect */
  const int32_t* tol_off; const int32_t* tol_key; const int32_t* tol_op; const int32_t* tol_value; const int32_t* tol_effect;
  /* ClusterSelector map */
  const int32_t* sel_off; const int32_t* sel_key; const int32_t* sel_value;
  /* requirement table (ClusterSelectorRequirement): key, operator, values (CSR) */
  int32_t n_reqs;
  const int32_t* rq_key; const int32_t* rq_op; const int32_t* rq_val_off; const int32_t* rq_val;
  /* required terms (ClusterSelector.ClusterSelectorTerms): unit w owns terms [rterm_off[w], rterm_off[w+1]);
     term t: MatchExpressions = requirements rt_req[t] .. rt_req[t] + rt_n_expr[t], then
     MatchFields = the next rt_n_field[t] requirements */
  const int32_t* rterm_off; const int32_t* rt_req; const int32_t* rt_n_expr; const int32_t* rt_n_field;
  /* preferred terms: unit w owns [pterm_off[w], pterm_off[w+1]); term t: Weight, and
     Preference.MatchExpressions = requirements pt_req[t] .. pt_req[t] + pt_n_expr[t] */
  const int32_t* pterm_off; const int32_t* pt_weight; const int32_t* pt_req; const int32_t* pt_n_expr;
  /* ClusterNames set */
  const int32_t* place_off; const int32_t* place_name;
  /* CurrentClusters map: name → replicas (cur_has_rep 0 = nil pointer) */
  const int32_t* cur_off; const int32_t* cur_name; const int64_t* cur_rep; const uint8_t* cur_has_rep;
  /* Weights, MinReplicas, MaxReplicas maps; AutoMigration.Info.EstimatedCapacity */
  const int32_t* wt_off; const int32_t* wt_name; const int64_t* wt_val;
  const int32_t* min_off; const int32_t* min_name; const int64_t* min_val;
  const int32_t* max_off; const int32_t* max_name; const int64_t* max_val;
  const int32_t* cap_off; const int32_t* cap_name; const int64_t* cap_val;
} kad_su_columns;

/* Per-unit statistics of a packed batch (optional output, may be NULL):
 * label/field requirements evaluated per cluster (SURVEY §8(d) R_w) and
 * toleration count. */
typedef struct kad_pack_stats {
  int32_t* n_reqs;   /* [n_units] */
  int32_t* n_tols;   /* [n_units] */
  int32_t n_distinct_reqs;
  int32_t n_tolsets;
} kad_pack_stats;

typedef struct kad_packer kad_packer;

/* Build a packer for one snapshot vocabulary (copied; the caller's buffers are free on return). */
int kad_packer_create(const kad_pack_vocab* vocab, kad_packer** out);
int kad_packer_destroy(kad_packer* p);
const char* kad_packer_error(kad_packer* p);
/* Pack a batch for `profile` (output slot bounds depend on its filter / select plugins). The blob
 * stays inside the packer (page-locked host memory, reused by the next pack) until kad_packer_take
 * copies it out; *nbytes = its size. `threads` <= 0: one per hardware thread (every pass runs in
 * parallel; the interning's chunk merge is sharded by hash, its ids equal one serial pass's). */
int kad_pack_batch(kad_packer* p, const kad_profile* profile, const kad_su_columns* su, int threads,
                   size_t* nbytes, kad_pack_stats* stats);
int kad_packer_take(kad_packer* p, void* dst, size_t cap);
/* The packed blob in place (no copy): valid until the next kad_pack_batch / kad_packer_take /
 * kad_packer_destroy; hand it to kad_batch_upload directly (a DMA from page-locked memory). */
int kad_packer_blob(kad_packer* p, const void** data, size_t* nbytes);

#ifdef __cplusplus
}
#endif
#endif /* KAD_PACK_H */

/*
 * kad_sched.h — C ABI of the MI355X-native batch scheduler for KubeAdmiral's
 * scheduling framework (libkad.so).
 *
 * Drop-in boundary. The reference runs, per SchedulingUnit and on one Go
 * goroutine,
 *
 *   core.ScheduleAlgorithm.Schedule(ctx, framework.Framework,
 *       framework.SchedulingUnit, []*FederatedCluster) (ScheduleResult, error)
 *   (pkg/controllers/scheduler/core/generic_scheduler.go:37-44, installed at
 *    pkg/controllers/scheduler/scheduler.go:208, called at scheduler.go:507).
 *
 * This library evaluates the same Filter → Score → Select → Replicas pipeline
 * for a whole batch of SchedulingUnits against one cluster snapshot on the GPU.
 * A cgo shim implements ScheduleAlgorithm on top of it:
 *
 *   kad_snapshot_upload   ← the []*FederatedCluster argument, packed once per
 *                           snapshot version (clusters are read-only informer
 *                           cache objects, generic_scheduler.go:96)
 *   kad_batch_upload      ← a batch of framework.SchedulingUnit values
 *                           (framework/types.go:33-69), packed
 *   kad_schedule          ← genericScheduler.Schedule for every unit
 *                           (generic_scheduler.go:92-150) under the plugin set
 *                           of the framework (kad_profile ← EnabledPlugins,
 *                           pkg/apis/core/types.go:21-43, built by
 *                           scheduler/profile.go:84-113)
 *   kad_results_download  ← ScheduleResult.SuggestedClusters per unit
 *                           (generic_scheduler.go:48-53) + error class
 *
 * Conventions: every function returns 0 on success or a negative KAD_E* code;
 * kad_last_error() gives the message. Inputs are caller-owned host buffers,
 * read only during the call; the library owns all device memory and never
 * keeps caller pointers. A kad_ctx is bound to one HIP device and one HIP
 * stream and is internally serialised (a mutex), so concurrent worker
 * goroutines (worker.go:132-134) may share it.
 *
 * Packed layouts: a snapshot blob and a batch blob are single contiguous byte
 * buffers — a header followed by 256-byte aligned arrays located by byte
 * offsets in the header — so one H2D copy (or one RCCL broadcast) moves them.
 * The host-side packer is kubeadmiral_amd/pack.py; the layout below is the
 * contract a Go packer would reproduce.
 */
#ifndef KAD_SCHED_H
#define KAD_SCHED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KAD_ABI_VERSION 2

/* ---------------------------------------------------------------- errors */
#define KAD_OK 0
#define KAD_EINVAL -1       /* malformed blob / profile / argument          */
#define KAD_EHIP -2         /* HIP runtime error (caller falls back)        */
#define KAD_ENOMEM -3       /* device allocation failed                     */
#define KAD_ESTATE -4       /* e.g. schedule before snapshot/batch upload   */
#define KAD_EUNSUPPORTED -5 /* plugin not in the in-tree set (webhook)      */
#define KAD_EHOST -6        /* other host-side failure (e.g. a pool thread could not start) */

/* ------------------------------------------------------------- plugins
 * In-tree plugin ids = bit positions in kad_profile masks.
 * Names: pkg/controllers/scheduler/framework/plugins/names/names.go:19-30;
 * registry: pkg/controllers/scheduler/profile.go:39-50.                    */
enum kad_plugin {
  KAD_PL_API_RESOURCES = 0,          /* APIResources                       */
  KAD_PL_TAINT_TOLERATION = 1,       /* TaintToleration (filter + score)   */
  KAD_PL_CLUSTER_RESOURCES_FIT = 2,  /* ClusterResourcesFit                */
  KAD_PL_PLACEMENT_FILTER = 3,       /* PlacementFilter                    */
  KAD_PL_CLUSTER_AFFINITY = 4,       /* ClusterAffinity (filter + score)   */
  KAD_PL_BALANCED_ALLOCATION = 5,    /* ClusterResourcesBalancedAllocation */
  KAD_PL_LEAST_ALLOCATED = 6,        /* ClusterResourcesLeastAllocated     */
  KAD_PL_MOST_ALLOCATED = 7,         /* ClusterResourcesMostAllocated      */
  KAD_PL_MAX_CLUSTER = 8,            /* MaxCluster (select)                */
  KAD_PL_CLUSTER_CAPACITY_WEIGHT = 9 /* ClusterCapacityWeight (replicas)   */
};

/* kad_profile.flags */
#define KAD_PROFILE_XORSHIFT_GO121 (1u << 0) /* pdqsort breakPatterns with the
                                                 13/7/17 xorshift triple instead of go1.19's 13/17/5 */

/* The framework: which in-tree plugin runs at which extension point.
 * Filters are an AND (runtime/framework.go:114-126) and score sums are
 * order-independent (core/generic_scheduler.go:182-190), so masks suffice;
 * only the FIRST select / replicas plugin runs (framework.go:194-207,
 * 234-247). Framework construction errors (unknown / duplicate / wrong-type
 * plugin, framework.go:70-95) are raised by the host before this call.      */
typedef struct kad_profile {
  uint32_t filter_mask;    /* bits of KAD_PL_* filter plugins                  */
  uint32_t score_mask;     /* bits of KAD_PL_* score plugins                   */
  int32_t select_plugin;   /* -1 = none (all feasible selected), KAD_PL_MAX_CLUSTER */
  int32_t replicas_plugin; /* -1 = none, KAD_PL_CLUSTER_CAPACITY_WEIGHT        */
  uint32_t flags;          /* KAD_PROFILE_*                                    */
  uint32_t reserved[3];
} kad_profile;

/* ------------------------------------------------------ snapshot blob
 * C clusters in snapshot order (the order of the []*FederatedCluster slice;
 * MaxCluster's tie behaviour is defined relative to it).
 * Array element [i][c] is stored at i*C + c ("row-major by attribute"), so a
 * wavefront reading 64 consecutive clusters is one coalesced access.        */
#define KAD_SNAPSHOT_MAGIC 0x5344414Bu /* "KADS" */
enum kad_snapshot_array {
  KAD_S_ALLOC_CPU = 0, /* i64[C]  Allocatable cpu MilliValue (framework/util.go:106)      */
  KAD_S_ALLOC_MEM,     /* i64[C]  Allocatable memory Value()                            */
  KAD_S_USED_CPU,      /* i64[C]  (Allocatable − Available) cpu via Resource.Sub
                                  (clusterresources/fit.go:140-147)                      */
  KAD_S_USED_MEM,      /* i64[C]                                                         */
  KAD_S_ALLOC_SCALAR,  /* i64[S][C] scalar resources (IsScalarResourceName) allocatable  */
  KAD_S_USED_SCALAR,   /* i64[S][C] scalar resources used                                */
  KAD_S_ALLOC_CORES,   /* i64[C]  Value() of (0 + Allocatable cpu) (rsp.go:305-325)      */
  KAD_S_AVAIL_CORES,   /* i64[C]  Value() of (0 + Available cpu)   (rsp.go:286-304)      */
  KAD_S_GVK,           /* u64[GW][C] bit g set ⇔ cluster lists APIResource g             */
  KAD_S_TAINT_NSNE,    /* u64[TW][C] taints with effect NoSchedule|NoExecute             */
  KAD_S_TAINT_NE,      /* u64[TW][C] taints with effect NoExecute                        */
  KAD_S_TAINT_PNS,     /* u64[TW][C] PreferNoSchedule taints (one id per occurrence)     */
  KAD_S_LABEL_VAL,     /* i32[K][C] value id of label key k (-1 = absent)                */
  KAD_S_LABEL_INT,     /* i64[K][C] strconv.ParseInt(value,10,64)                        */
  KAD_S_LABEL_INT_OK,  /* u8[K][C]  1 if the parse succeeded                             */
  KAD_S_NAME_FNV,      /* u32[C]  FNV-1 32 state after the cluster name bytes
                                  (util/planner/planner.go:185-195)                      */
  KAD_S_CFLAGS,        /* u32[C]  bit0: Resource.Sub error (map-order dependent input)   */
  KAD_S_NARRAYS
};

typedef struct kad_snapshot_header {
  uint32_t magic;
  uint32_t abi_version;
  int32_t n_clusters;    /* C  */
  int32_t n_gvk_words;   /* GW */
  int32_t n_taint_words; /* TW */
  int32_t n_label_keys;  /* K  */
  int32_t n_scalar;      /* S  */
  int32_t reserved0;
  uint64_t total_bytes;
  uint64_t fingerprint; /* vocabulary fingerprint (cluster names in order and
                           the interned label / taint / API-resource / scalar
                           ids a batch is packed against); batches carry it */
  uint64_t off[KAD_S_NARRAYS];
} kad_snapshot_header;

/* ----------------------------------------------- snapshot delta blob
 * Cluster informer updates (scheduler.go:157-177) that change existing
 * clusters without growing the vocabulary — resources (the common case:
 * status collection), a label to an already-interned value, a known taint —
 * are applied to the resident snapshot in place: the delta carries the
 * changed clusters' columns of every snapshot array, so batches packed
 * against the snapshot stay valid. Anything else (cluster join/leave, a new
 * label value, taint, API resource or scalar name) needs a full upload.
 * Layout: header, i32 idx[n_changed] (snapshot positions, strictly
 * increasing), then for each snapshot array a its rows for the changed
 * clusters, element [r][j] at off[a] + (r*n_changed + j)*elem_size(a), rows
 * and element sizes as in the snapshot (1 / S / GW / TW / K rows).          */
#define KAD_DELTA_MAGIC 0x4441444Bu /* "KADD" */
typedef struct kad_snapshot_delta_header {
  uint32_t magic;
  uint32_t abi_version;
  int32_t n_clusters;   /* must equal the resident snapshot's C            */
  int32_t n_changed;    /* clusters rewritten                              */
  uint64_t total_bytes;
  uint64_t fingerprint; /* must equal the resident snapshot's fingerprint  */
  uint64_t idx_off;     /* i32[n_changed]                                  */
  uint64_t off[KAD_S_NARRAYS];
} kad_snapshot_delta_header;

/* --------------------------------------------------------- batch blob
 * W scheduling units; CSR arrays are indexed by *_OFF[w] .. *_OFF[w+1].    */
#define KAD_BATCH_MAGIC 0x4241444Bu /* "KADB" */

/* per-unit flags (KAD_B_FLAGS) */
#define KAD_W_DUPLICATE (1u << 0)         /* SchedulingMode == Duplicate (generic_scheduler.go:130)  */
#define KAD_W_STICKY (1u << 1)            /* StickyCluster && len(CurrentClusters)>0 (:101-104)      */
#define KAD_W_AVOID_DISRUPTION (1u << 2)  /* AvoidDisruption (planner.go:116-176)                   */
#define KAD_W_KEEP_UNSCHED (1u << 3)      /* AutoMigration.KeepUnschedulableReplicas (rsp.go:128-139)*/
#define KAD_W_HAS_DESIRED (1u << 4)       /* DesiredReplicas != nil                                  */
#define KAD_W_HAS_MAX_CLUSTERS (1u << 5)  /* MaxClusters != nil (max_cluster.go:48-58)               */
#define KAD_W_FIT_NONZERO (1u << 6)       /* fit.go:82-87 early return NOT taken                     */
#define KAD_W_HAS_PLACEMENT (1u << 7)     /* len(ClusterNames) > 0 (placement/filter.go:47)          */
#define KAD_W_SCORE_ERROR (1u << 8)       /* ClusterAffinity.Score errors (cluster_affinity.go:121)  */
#define KAD_W_DYNAMIC_WEIGHTS (1u << 9)   /* len(Weights) == 0 (rsp.go:69)                           */
#define KAD_W_HAS_CURRENT (1u << 10)      /* len(CurrentClusters) > 0                                */
#define KAD_W_WIDE_SCORES (1u << 11)      /* affinity weights may exceed the narrow i32 path         */

enum kad_batch_array {
  KAD_B_FLAGS = 0,     /* u32[W]                                                          */
  KAD_B_GVK,           /* i32[W]  snapshot GVK id of (GroupVersion, Kind); -1 = none has it */
  KAD_B_REQ_CPU,       /* i64[W]  ResourceRequest.MilliCPU                                */
  KAD_B_REQ_MEM,       /* i64[W]  ResourceRequest.Memory                                  */
  KAD_B_DESIRED,       /* i64[W]  *DesiredReplicas (0 when nil)                           */
  KAD_B_MAX_CLUSTERS,  /* i64[W]  *MaxClusters                                            */
  KAD_B_TOLSET,        /* i32[W]  toleration-set id                                       */
  KAD_B_TOL_ALL,       /* u64[NT][TW] taints tolerated by some toleration                 */
  KAD_B_TOL_PNS,       /* u64[NT][TW] ... by a toleration with effect "" or PreferNoSchedule */
  KAD_B_SREQ_OFF,      /* i32[W+1] scalar requests (ScalarResources map)                  */
  KAD_B_SREQ_ID,       /* i32[]    snapshot scalar id (-1: no cluster has it)             */
  KAD_B_SREQ_VAL,      /* i64[]    requested value                                        */
  KAD_B_FPROG_OFF,     /* i32[W+1] ClusterAffinity filter program (see KAD_OP_*)          */
  KAD_B_FPROG,         /* i32[]                                                           */
  KAD_B_SPROG_OFF,     /* i32[W+1] ClusterAffinity score program                          */
  KAD_B_SPROG,         /* i32[]                                                           */
  KAD_B_PLACE_OFF,     /* i32[W+1] ClusterNames as snapshot cluster ids (sorted, unique)  */
  KAD_B_PLACE,         /* i32[]                                                           */
  KAD_B_CUR_OFF,       /* i32[W+1] CurrentClusters as snapshot ids (sorted)               */
  KAD_B_CUR_ID,        /* i32[]                                                           */
  KAD_B_CUR_REP,       /* i64[]    replicas (nil resolved to DesiredReplicas, rsp.go:119-126) */
  KAD_B_PREF_OFF,      /* i32[W+1] per-cluster Weights/MinReplicas/MaxReplicas/EstimatedCapacity */
  KAD_B_PREF_ID,       /* i32[]    snapshot cluster id (sorted)                           */
  KAD_B_PREF_W,        /* i64[]    Weights[cluster]           (i32[]: KAD_BATCH_NARROW_PREFS) */
  KAD_B_PREF_MIN,      /* i64[]    MinReplicas[cluster]       (i32[]: KAD_BATCH_NARROW_PREFS) */
  KAD_B_PREF_MAX,      /* i64[]    MaxReplicas[cluster]       (i32[]: KAD_BATCH_NARROW_PREFS) */
  KAD_B_PREF_CAP,      /* i64[]    EstimatedCapacity[cluster] (only entries >= 0; i32[] narrow) */
  KAD_B_PREF_FLAGS,    /* u32[]    bit0 has weight, bit1 has max, bit2 has cap            */
  KAD_B_KEY_OFF,       /* i32[W+1] su.Key() bytes (types.go:123-128)                      */
  KAD_B_KEY,           /* u8[]                                                            */
  KAD_B_OUT_OFF,       /* i64[W+1] output slot ranges (host-computed upper bounds)        */
  KAD_B_REQ_OFF,       /* i32[NR+1] batch-wide table of distinct label/field requirements */
  KAD_B_REQ,           /* i32[]     requirement words (see KAD_OP_*)                       */
  KAD_B_NARRAYS
};

#define KAD_PREF_HAS_WEIGHT 1u
#define KAD_PREF_HAS_MAX 2u
#define KAD_PREF_HAS_CAP 4u

/* kad_batch_header.flags */
#define KAD_BATCH_NARROW_PREFS 1u /* every value of every unit's Weights, MinReplicas, MaxReplicas and
                                     (AutoMigration units) EstimatedCapacity map fits int32: the four
                                     KAD_B_PREF_{W,MIN,MAX,CAP} columns are i32[] (the packers decide it
                                     from the input maps, so both produce the same bytes)             */

typedef struct kad_batch_header {
  uint32_t magic;
  uint32_t abi_version;
  int32_t n_units;       /* W                                        */
  int32_t n_clusters;    /* must equal the snapshot's C              */
  int32_t n_taint_words; /* must equal the snapshot's TW             */
  int32_t n_tolsets;     /* NT                                       */
  int64_t n_out_slots;   /* = OUT_OFF[W]                             */
  int32_t max_row_slots; /* max_w OUT_OFF[w+1]-OUT_OFF[w]            */
  uint32_t packed_filter_mask;  /* profile the output bounds were sized for:  */
  int32_t packed_select_plugin; /* kad_schedule rejects any other profile     */
  int32_t n_reqs;       /* NR: distinct requirements in KAD_B_REQ                         */
  uint32_t flags;       /* KAD_BATCH_*                                                    */
  uint32_t reserved;    /* 0                                                              */
  uint64_t total_bytes;
  uint64_t snapshot_fingerprint;
  uint64_t off[KAD_B_NARRAYS];
} kad_batch_header;

/* ------------------------------------------------ predicate programs
 * Requirements are interned batch-wide: KAD_B_REQ holds each distinct one
 * once as  [op | n_payload<<8, key, payload...]  (i32 words):
 *   KAD_OP_IN / NOTIN / EQ : payload = value ids of that key (labels.Requirement
 *                            In / NotIn / SelectorFromSet's Equals)
 *   KAD_OP_EXISTS / DNE    : no payload
 *   KAD_OP_GT / LT         : payload = int64 threshold as (lo, hi) words
 *   KAD_OP_NAME_EQ / NE    : key = snapshot cluster id (-1: no such cluster);
 *                            field selector on metadata.name
 *                            (util/clusterselector/util.go:65-93)
 *   KAD_OP_TRUE / FALSE    : folded on the host (key or value absent from
 *                            every cluster, field keys other than metadata.name)
 * The device evaluates every distinct requirement once per cluster into a
 * bitmask row (NR × ⌈C/64⌉ u64); a unit's programs then combine rows with
 * word-wide AND/OR instead of re-evaluating selectors per (unit, cluster) pair
 * as the reference does (clusterselector/util.go:35-58 per call).
 * Filter program (cluster_affinity.go:50-94, clusterselector/util.go:97-132):
 *   n_sel, <n_sel requirement ids: ClusterSelector map>,
 *   req_present, [n_terms, { tflags, n_expr, n_field, <expr ids>, <field ids> } ...]
 *   tflags: bit0 has_expr, bit1 expr_valid, bit2 has_field, bit3 field_valid
 *   (invalid parts carry no requirements; reaching one makes the whole
 *    MatchClusterSelectorTerms return false, as the reference's error does).
 * Score program (cluster_affinity.go:96-135): n_terms, { weight, n_expr, <expr ids> } ...
 *   (only valid, non-empty terms with weight != 0)                           */
enum kad_op {
  KAD_OP_IN = 1, KAD_OP_NOTIN = 2, KAD_OP_EXISTS = 3, KAD_OP_DNE = 4,
  KAD_OP_GT = 5, KAD_OP_LT = 6, KAD_OP_EQ = 7, KAD_OP_TRUE = 8, KAD_OP_FALSE = 9,
  KAD_OP_NAME_EQ = 10, KAD_OP_NAME_NE = 11
};
#define KAD_TERM_HAS_EXPR 1
#define KAD_TERM_EXPR_VALID 2
#define KAD_TERM_HAS_FIELD 4
#define KAD_TERM_FIELD_VALID 8

/* ------------------------------------------------------------ results
 * Per unit: status, count and flags; pairs in the unit's output slot range
 * [OUT_OFF[w], OUT_OFF[w] + count) in ascending cluster id.
 *   Duplicate mode: replicas = -1 (the Go nil pointer).
 *   Divide mode   : replicas > 0 (zero entries are dropped, rsp.go:170-179).
 *   KAD_ST_STICKY : SuggestedClusters = CurrentClusters (host copies it).
 *   KAD_ST_NO_FEASIBLE: SuggestedClusters = nil (generic_scheduler.go:112-114). */
enum kad_status {
  KAD_ST_OK = 0,
  KAD_ST_STICKY = 1,
  KAD_ST_NO_FEASIBLE = 2,
  KAD_ST_ERR_SCORE = 3,    /* "failed to scoreClusters"      */
  KAD_ST_ERR_SELECT = 4,   /* "failed to selectClusters"     */
  KAD_ST_ERR_REPLICAS = 5  /* "failed to do replicaScheduling" */
};
/* result flags */
#define KAD_RF_TIE_STRADDLE 1u  /* MaxCluster cut fell inside a run of equal scores: pdqsort emulated */
#define KAD_RF_REMAINDER_TIE 2u /* AvailableToPercentage remainder had tied recipients (rsp.go:257-270) */
#define KAD_RF_HASH_TIE 4u      /* planner (weight, FNV) tie: reference order is map-order dependent */

typedef struct kad_result_view {
  int32_t* status;      /* [W]           */
  int32_t* count;       /* [W]           */
  uint32_t* flags;      /* [W]           */
  int32_t* cluster;     /* [n_out_slots] */
  int64_t* replicas;    /* [n_out_slots] */
} kad_result_view;

/* ------------------------------------------------------------ context */
typedef struct kad_ctx kad_ctx;

int kad_ctx_create(int hip_device, kad_ctx** out);
int kad_ctx_destroy(kad_ctx* ctx);
const char* kad_last_error(kad_ctx* ctx);
int kad_abi_version(void);

/* snapshot / batch residency (H2D, or D2D from a device buffer e.g. after an
 * RCCL broadcast of the snapshot blob). Allocation happens here, never in
 * kad_schedule.                                                              */
int kad_snapshot_upload(kad_ctx* ctx, const void* blob, size_t nbytes);
int kad_snapshot_upload_device(kad_ctx* ctx, const void* dev_blob, size_t nbytes);
/* Apply a kad_snapshot_delta blob to the resident snapshot (one H2D of the
 * delta + one scatter kernel, ordered on the ctx stream after any schedule
 * already issued). The resident batch stays valid.  ← cluster update events
 * (scheduler.go:157-177) that re-enqueue objects against changed clusters. */
int kad_snapshot_update(kad_ctx* ctx, const void* delta, size_t nbytes);
int kad_batch_upload(kad_ctx* ctx, const void* blob, size_t nbytes);

/* Run the pipeline for the resident batch; asynchronous on the ctx stream. */
int kad_schedule(kad_ctx* ctx, const kad_profile* profile);
int kad_sync(kad_ctx* ctx);
/* Device time of the last kad_schedule, from HIP events on the ctx stream:
 * ms[0] = whole pipeline, ms[1] = filter/score/select kernel, ms[2] = planner. */
int kad_last_timing(kad_ctx* ctx, float ms[3]);
/* Record those events in later kad_schedule calls (default on). Off, the
 * stream carries only the kernels (no marker packets between passes) and
 * kad_last_timing returns KAD_ESTATE.  No reference counterpart (instrumentation). */
int kad_set_timing(kad_ctx* ctx, int on);
/* Per-stage device times of the last kad_schedule run with timing on (n <= 7 entries):
 * ms[0] req_mask_kernel, [1] prep_kernel, [2] the main schedule kernel (lean / wide / full),
 * [3] the defer pass (schedule_kernel), [4] the replica planner, [5] the whole pipeline,
 * [6] the long-feasible-list pass (schedule_row_kernel). No reference counterpart. */
int kad_stage_timing(kad_ctx* ctx, float* ms, int n);
/* Which kernel took how many units in the last kad_schedule (blocks until it is done): out[0] units,
 * [1] the full kernel (defer list), [2] the long-feasible-list kernel, [3] planner rows (Divide units).
 * Measurement only (bench.py's per-kernel byte models). No reference counterpart. */
int kad_path_counts(kad_ctx* ctx, int32_t* out);
/* How the resident snapshot is scheduled (no device work): out[0] its resource class (2 every cluster
 * has 1 <= allocatable and used <= allocatable; 1 some cluster has allocatable 0 or available < 0 — the
 * clusters federatedcluster/util.go:178-214 reports when cordoned / tainted nodes are left out of
 * allocatable —, all below 2^46; 0 otherwise), [1] 1 if the exact-f64 fast path applies (class 2, or class
 * 1 with the filter folded), [2] 1 if the main kernel is schedule_wide_kernel, [3] taint / API filters
 * folded into the static words, [4] the fit threshold rows folded too. Returns KAD_ESTATE without a
 * snapshot. Measurement / tests only. No reference counterpart. */
int kad_snapshot_paths(kad_ctx* ctx, int32_t* out);
int kad_results_download(kad_ctx* ctx, const kad_result_view* out);
/* Page-locked host memory for the download's (or a batch blob's) buffers, reused across batches: the
 * copies then DMA straight into / out of it (no staging). kad_host_free(NULL) is a no-op. Caller-side
 * plumbing, no reference counterpart. */
int kad_host_alloc(size_t nbytes, void** out);
int kad_host_free(void* p);
/* The same results copied device-to-device into caller DEVICE buffers of the result view's sizes
 * (e.g. the send buffers of an RCCL all-gather of placements across GPUs); blocking. */
int kad_results_copy_device(kad_ctx* ctx, const kad_result_view* dev_out);

/* All in one: upload batch, schedule, download (blocking). */
int kad_schedule_batch(kad_ctx* ctx, const kad_profile* profile, const void* batch_blob, size_t nbytes,
                       const kad_result_view* out);

/* ---------------------------------------------------- multi-GPU group
 * One process driving N GPUs of a node: the reference runs one scheduler process whose --worker-count
 * goroutines call Schedule (worker.go:132-134, scheduler.go:507), and units are independent given the
 * read-only cluster list (scheduler.go:246-309), so a batch splits into N contiguous unit ranges with no
 * exchange while scheduling. A kad_group holds one kad_ctx per listed device (a device may repeat: the
 * members then share it, e.g. tests on one GPU) and one host thread per member, so every member's
 * uploads, launches and copies are issued concurrently.
 *   kad_group_snapshot_upload: H2D to member 0, then device to device to the others (xGMI peer copies);
 *                              each member rebuilds its derived snapshot state on its own device.
 *   kad_group_snapshot_update: the delta applied on every member.
 *   kad_group_batch_upload   : the whole blob validated once; member i takes units
 *                              [unit_lo[i], unit_lo[i+1]) (kad_batch_split) and H2Ds only the blob bytes
 *                              those units read (their per-unit entries, their CSR data, the batch-wide
 *                              tables) into a buffer of the blob's layout.
 *   kad_group_schedule       : every member's pipeline, asynchronous on its stream.
 *   kad_group_results_download: each member writes its units' status / count / flags at unit_lo[i] and
 *                              its slots at slot_lo[i] = OUT_OFF[unit_lo[i]] of the ONE caller view sized
 *                              for the whole batch — the same bytes as one kad_ctx over the whole batch.
 * A kad_group is internally serialised (a mutex), like a kad_ctx. */
typedef struct kad_group kad_group;
int kad_group_create(const int* hip_devices, int n, kad_group** out);
int kad_group_destroy(kad_group* group);
const char* kad_group_last_error(kad_group* group);
int kad_group_size(kad_group* group);
int kad_group_snapshot_upload(kad_group* group, const void* blob, size_t nbytes);
int kad_group_snapshot_update(kad_group* group, const void* delta, size_t nbytes);
int kad_group_batch_upload(kad_group* group, const void* blob, size_t nbytes);
int kad_group_schedule(kad_group* group, const kad_profile* profile);
int kad_group_sync(kad_group* group);
int kad_group_results_download(kad_group* group, const kad_result_view* out);
/* All in one: upload batch, schedule on every member, download (blocking). */
int kad_group_schedule_batch(kad_group* group, const kad_profile* profile, const void* batch_blob, size_t nbytes,
                             const kad_result_view* out);
/* The resident batch's split: unit_lo[n+1], slot_lo[n+1]. */
int kad_group_ranges(kad_group* group, int64_t* unit_lo, int64_t* slot_lo);
/* kad_path_counts summed over the members; kad_set_timing on every member. */
int kad_group_path_counts(kad_group* group, int32_t* out);
int kad_group_set_timing(kad_group* group, int on);
/* Member i's kad_ctx, for per-member instrumentation only (kad_stage_timing, kad_path_counts): it
 * schedules units [unit_lo[i], unit_lo[i+1]) of the group's batch; its own kad_results_download writes
 * them at offset 0. */
int kad_group_member(kad_group* group, int i, kad_ctx** out);
/* Host only (no device): the split kad_group_batch_upload makes of a packed batch blob for n members —
 * unit_lo[i] = W*i/n, slot_lo[i] = OUT_OFF[unit_lo[i]], i = 0..n. */
int kad_batch_split(const void* batch_blob, size_t nbytes, int n, int64_t* unit_lo, int64_t* slot_lo);

/* ---------------------------------------------------- stage entry points
 * The select and planner stages on caller-provided rows, for parity tests of
 * each plugin in isolation (max_cluster_test.go, planner_test.go).          */
/* MaxCluster over rows of scores in input order; out_sel gets, per row, the
 * selected input positions (ascending) in [row_off[r], row_off[r]+out_count[r]). */
int kad_select_rows(kad_ctx* ctx, int n_rows, const int32_t* row_off, const int64_t* scores,
                    const int64_t* max_clusters /* <0: error, INT64_MAX: nil */, uint32_t profile_flags,
                    int32_t* out_count, int32_t* out_sel, int32_t* out_status);

/* planner.Plan over rows: per element name hash (FNV-1 of name‖key), weight,
 * min, max (flags bit1), capacity (flags bit2), current; per row total
 * replicas, avoid_disruption / keep_unschedulable (row_flags bit0 / bit1).
 * Outputs per element plan and overflow.                                    */
int kad_plan_rows(kad_ctx* ctx, int n_rows, const int32_t* row_off, const uint32_t* hash, const int64_t* weight,
                  const int64_t* min_r, const int64_t* max_r, const int64_t* cap, const int64_t* current,
                  const uint32_t* elem_flags, const int64_t* total, const uint32_t* row_flags,
                  int64_t* out_plan, int64_t* out_overflow);

/* Debug: per (unit, cluster) feasibility and total score of the last
 * kad_schedule (feasible: u8[W*C]; total: i64[W*C], meaningful where feasible). */
int kad_debug_scores(kad_ctx* ctx, const kad_profile* profile, uint8_t* feasible, int64_t* total);

/* ------------------------------------------------ result application (§8 f3)
 * applySchedulingResult (pkg/controllers/scheduler/scheduler.go:632-695) writes a unit's result into its
 * federated object: the scheduler controller's placement (util.SetPlacementClusterNames,
 * util/placement.go:48-59 → SetPlacementNames, types/v1alpha1/extensions_placements.go:78-103) and its
 * replicas overrides (UpdateReplicasOverride → OverrideUpdateNeeded, scheduler/util.go:71-94, 154-185).
 * kad_result_diff decides on the device, where the results of the last kad_schedule are, which of the two
 * would change for every unit, so the caller edits and re-serialises only those objects. The caller
 * describes each object's CURRENT state with snapshot cluster positions (-1: a name not in the snapshot):
 *   place_off[W+1] / place_cluster: the clusters of the FIRST placement whose controller is the scheduler
 *     (any order, duplicates allowed); place_has[W] = 1 if that placement exists (DeletePlacement's
 *     hasChange when the result is empty);
 *   ovr_off[W+1] / ovr_cluster / ovr_value / ovr_kind: the scheduler controller's override patches whose
 *     path is the replicas path (util.GetOverrides, one entry per patch); ovr_kind 0: the value decoded as
 *     a JSON number (float64) and ovr_value = int64(value) (Go's truncating conversion); 1: any other type.
 * out_flags[W]: KAD_DIFF_PLACEMENT and / or KAD_DIFF_OVERRIDES as the reference reports them
 * (placementUpdated, overridesUpdated); KAD_DIFF_SKIP for units whose Schedule returned an error (nothing is
 * applied, scheduler.go:505-517); KAD_DIFF_STICKY for sticky units (the result is su.CurrentClusters, which
 * the caller holds and applies itself). The annotation half of applySchedulingResult (follower scheduling,
 * unschedulable threshold) does not depend on the result and stays with the caller. Blocks until done.  */
typedef struct kad_result_state {
  int32_t n_units;              /* = the resident batch's n_units */
  const int32_t* place_off;     /* [n_units + 1] */
  const int32_t* place_cluster; /* [place_off[n_units]] */
  const uint8_t* place_has;     /* [n_units] */
  const int32_t* ovr_off;       /* [n_units + 1] */
  const int32_t* ovr_cluster;   /* [ovr_off[n_units]] */
  const int64_t* ovr_value;     /* [ovr_off[n_units]] */
  const uint8_t* ovr_kind;      /* [ovr_off[n_units]] */
} kad_result_state;
#define KAD_DIFF_PLACEMENT 1u
#define KAD_DIFF_OVERRIDES 2u
#define KAD_DIFF_SKIP 4u
#define KAD_DIFF_STICKY 8u
int kad_result_diff(kad_ctx* ctx, const kad_result_state* state, uint32_t* out_flags);

/* ------------------------------------------- scheduling-trigger hashes
 * Replaces the FNV-1 half of Scheduler.computeSchedulingTriggerHash
 * (pkg/controllers/scheduler/schedulingtriggers.go:106-147, called per object
 * from prepareToSchedule, scheduler.go:394). The caller splits each object's
 * json.Marshal(schedulingTriggers) bytes at the "clusterLabels" value: the
 * object part (prefix: scheduling annotations, replica count, resource
 * request, auto-migration info, policy name + generation, up to and including
 * `"clusterLabels":`) and the cluster part (suffix: clusterLabels value,
 * clusterTaints, clusterAPIResourceTypes, closing brace), which is identical
 * for every object scheduled against the same joined-cluster list. Output:
 * hash.Sum32() per object (the reference formats it with strconv.FormatInt).
 *   suffix: uploaded once per cluster-set change (bytes, any alignment)
 *   prefixes: CSR, prefix_off[0] = 0, non-decreasing, n+1 entries
 *   run: asynchronous on the ctx stream (summarises the suffix into a
 *        256-entry FNV table, then hashes every object); download blocks.  */
int kad_trigger_suffix_upload(kad_ctx* ctx, const uint8_t* suffix, size_t nbytes);
int kad_trigger_prefixes_upload(kad_ctx* ctx, int n, const int64_t* prefix_off, const uint8_t* prefix);
int kad_trigger_run(kad_ctx* ctx);
/* ms[0] = whole trigger run, ms[1] = the cluster-part summary kernels */
int kad_trigger_timing(kad_ctx* ctx, float ms[2]);
int kad_trigger_download(kad_ctx* ctx, uint32_t* out_hash);
/* All in one (blocking): both uploads, run, download. */
int kad_trigger_hashes(kad_ctx* ctx, int n, const int64_t* prefix_off, const uint8_t* prefix, const uint8_t* suffix,
                       size_t suffix_len, uint32_t* out_hash);

/* Profiling builds only (-DKAD_PHASE_PROF): copy 32 per-phase cycle / event
 * counters of the kernels to out (and zero them if reset). Returns 32, or
 * 0 in product builds (no counters compiled in). Not part of the reference. */
int kad_debug_phase_counters(uint64_t* out, int reset);

/* Tests only: fault injection. where = 1: the next rebuild of the snapshot's
 * derived state (kad_snapshot_upload / _upload_device / _update) fails with
 * KAD_ENOMEM, as an allocation failure would. A failed snapshot upload or
 * update leaves no snapshot and no batch resident (kad_schedule then returns
 * KAD_ESTATE). where = 0 clears a pending fault. Not part of the reference. */
int kad_debug_inject_fault(kad_ctx* ctx, int where);

/* Tests only: on = 1 sends every row of kad_plan_rows through the LDS-workspace planner (the path of rows
 * with more than 64 clusters), so the golden planner cases cover both planners; on = 2 runs rows two per
 * wave where both hold at most 32 clusters (plan_pair_kernel's half-wave planner); 0 restores the default
 * choice by row length. Not part of the reference. */
int kad_debug_plan_force_workspace(kad_ctx* ctx, int on);

#ifdef __cplusplus
}
#endif
#endif /* KAD_SCHED_H */

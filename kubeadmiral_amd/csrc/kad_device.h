// Device-side views of the packed snapshot / batch (include/kad_sched.h) and
// the kernel launchers of libkad.so. gfx950 (MI355X) only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/kad_sched.h"

namespace kad {

constexpr int FITFOLD_MAX_C = 16384;
// taint words (64 ids each) prep_kernel folds into the static filter words (SnapDev::fold): up to 256 ids
constexpr int TFOLD_MAX_TW = 4;
// byte cap of the per-id slices + taint table (SnapDev::slices / taint_tab): 2*8*TW*256 words per 64-cluster
// chunk, 41 MB at C5 (10k clusters, TW = 4), 268 MB at 65535 clusters; above the cap (C > ~32k at TW = 4,
// ~128k-cluster-equivalents at TW = 1) the snapshot runs unfolded
constexpr size_t TTAB_MAX_BYTES = (size_t)128 << 20;
// unit work queue of the schedule kernels: WQ_HEADS counters, one 128-B line apart (BatchDev::wq)
constexpr int WQ_HEADS = 64, WQ_STRIDE = 32;
#ifndef KAD_FIT_FENCES
#define KAD_FIT_FENCES 256
#endif
constexpr int FIT_FENCES = KAD_FIT_FENCES;  // prep's LDS copy of every (fit_mp / FIT_FENCES)-th fit value
constexpr int REQ_SEG_G = 8;  // chunks per req_mask_kernel wave (kad_kernels.hip REQ_G)
// SnapDev::vrows: label value ids below VR_SLOTS get a cluster row; requirements naming at most
// VR_MAX_VALS such values are ORs of rows (req_row_kernel)
constexpr int VR_SLOTS = 64, VR_MAX_VALS = 5;
constexpr size_t VR_MAX_BYTES = (size_t)256 << 20;  // prep_kernel's LDS copy of every (fit_mp / 256)-th fit value

struct SnapDev {
  int C, GW, TW, K, S;
  // host: every cluster's cpu/mem score through the exact-f64 path (kad_api.hip res_clean): strict clusters
  // (1 <= allocatable, used <= allocatable), or — with the filter folded (fold, fitfold) — relaxed ones with
  // allocatable 0 or used > allocatable (their score operands: score_res)
  int clean;
  // TW <= TFOLD_MAX_TW: prep_kernel folds TaintToleration's and APIResources' filters into each unit's
  // static filter words from per-id cluster bitmask slices ([128*TW + 64*GW][nch]: rows t < 64*TW the
  // NoSchedule|NoExecute taint id t, rows 64*TW + t the NoExecute taint id t, rows 128*TW + g GVK id g of
  // any GVK word — a discovery list of ~150 API resources per cluster is 3 words, clusterstatus.go:221-266),
  // so the schedule kernels only test resource fit per lane (or nothing, with SnapDev::fitfold)
  int fold;
  uint64_t present_taints[TFOLD_MAX_TW];  // per taint word: OR of every cluster's NoSchedule|NoExecute word
  const uint64_t* slices;
  // [2][8*TW][256][nch]: entry (tbl, g, sub, ch) = OR of the chunk-ch slices of taint ids 8g + b, b in sub,
  // table tbl (0: NoSchedule|NoExecute, 1: NoExecute) — a unit's untolerated taints in <= 8*TW lookups
  const uint64_t* taint_tab;
  // clean snapshots with C <= FITFOLD_MAX_C: ClusterResourcesFit's cpu / memory test as a threshold
  // table per resource r (0 cpu, 1 memory) — fit_vals[r]: the m_r distinct available amounts
  // (allocatable - used) ascending, then INT64_MAX up to fit_mp; fit_rows[r][j][nch]: clusters whose available
  // amount is >= fit_vals[r][j] (row m_r empty). prep_kernel ANDs row lower_bound(request) into the
  // static words, and the schedule kernels skip their own cpu / memory compare (SnapDev::fitfold).
  int fitfold;
  int fit_m[2];
  int fit_mp;  // fit_vals[r] length: a power of two >= FIT_FENCES, > fit_m[r] (INT64_MAX padding)
  const int64_t* fit_vals[2];
  const uint64_t* fit_rows[2];
  const int64_t *alloc_cpu, *alloc_mem, *used_cpu, *used_mem, *alloc_s, *used_s, *alloc_cores, *avail_cores;
  const uint64_t *gvk, *nsne, *ne, *pns;
  // [K][VR_SLOTS + 1][nch]: row (k, s) = clusters whose label k has value id s, row (k, VR_SLOTS) = clusters
  // with label k (rebuilt at upload / update; null when larger than VR_MAX_BYTES)
  const uint64_t* vrows;
  const int32_t* lval;
  const int64_t* lint;
  const uint8_t* lok;
  const uint32_t* name_fnv;
  // clean snapshots: the score operands of the exact clean-f64 path per cluster, rebuilt at upload / update
  // (res_cols_kernel) so that kernels gathering them per feasible position (schedule_row_kernel) do one
  // 32-B + one 8-B load instead of four i64 loads and two f64 divisions: res4[c] = (alloc_cpu - used_cpu,
  // alloc_mem - used_mem, alloc_cpu, alloc_mem) as f64, res_iv[c] = (float)(100 / alloc) per resource
  const double4* res4;
  const float2* res_iv;
  // the PreferNoSchedule words of cluster c, cluster-major (words >= TW zero; TW <= 4, clean snapshots):
  // one 32-B gather per feasible position instead of TW 8-B ones from the [TW][C] array
  const ulonglong4* pns4;
};

// The exact-f64 score operands (cap, available = allocatable - used) of one resource of a clean cluster.
// Least / Most / Balanced read them as x = available - request, exact in f64 (< 2^47): Least
// floor(100 x / cap) when x >= 0 else 0 (least_allocated.go:88-96: requested > capacity => 0), Most
// floor(100 (cap - x) / cap) when x >= 0 else 0, Balanced (cap - x) / cap = requested / capacity
// (balanced_allocation.go:84-88). used > allocatable (available < 0) needs nothing: x < 0 scores 0 in
// Least / Most and the fraction is > 1 (Balanced 0), as in Go. allocatable 0 scores 0 everywhere in Go
// (capacity == 0 => 0, fractionOfCapacity => 1): (cap, available) = (1, -1) gives exactly that (x < 0,
// fraction 2 + request >= 1) without a zero divisor. Fit never reads these (the relaxed clusters run only
// with the fit threshold rows, SnapDev::fitfold), so the substitute amount changes no filter.
__host__ __device__ inline void score_res(int64_t alloc, int64_t used, double& cap, double& avail) {
  cap = alloc == 0 ? 1.0 : (double)alloc;
  avail = alloc == 0 ? -1.0 : (double)(alloc - used);
}

struct BatchDev {
  int W, NT, TW;
  uint32_t flags_or;        // OR of every unit's KAD_W_* flags (host, at upload)
  int may_defer;            // host: some unit may reach the lean kernel's defer list (else that pass is skipped)
  int zero_req;             // host: no unit of the batch has a ResourceRequest (the live controller's batches)
  const uint32_t* flags;
  const int32_t *gvk, *tolset;
  const int64_t *req_cpu, *req_mem, *desired, *maxc;
  const uint64_t *tol_all, *tol_pns;
  const int32_t *sreq_off, *sreq_id;
  const int64_t* sreq_val;
  const int32_t *fprog_off, *fprog, *sprog_off, *sprog, *place_off, *place, *cur_off, *cur_id;
  const int64_t* cur_rep;
  const int32_t *pref_off, *pref_id;
  const int64_t *pref_w, *pref_min, *pref_max, *pref_cap;          // wide batches (null when narrow)
  const int32_t *pref_w32, *pref_min32, *pref_max32, *pref_cap32;  // KAD_BATCH_NARROW_PREFS batches
  int pref_narrow;
  const uint32_t* pref_fl;
  const int32_t* key_off;
  const uint8_t* key;
  const int64_t* out_off;
  int NR;                   // distinct requirements
  const int32_t *req_off, *req;
  // requirements grouped by label key (host, at upload): req_perm lists the requirements key by key as
  // 8-word entries (id, word offset, op | n << 8, key word, payload 0..3); segment i = (key, first entry,
  // count <= 64, 0), key -1 for the label-free ops (TRUE / FALSE / metadata.name); req_mask_kernel
  // evaluates one segment per wave
  int n_seg;
  const int32_t* req_perm;
  const int4* req_seg;
  int n_rowreq;             // requirements evaluated from SnapDev::vrows: 8-word entries (id, op | n << 8,
  const int4* req_rows;     // key, value ids 0..4)
  uint64_t* req_mask;       // device workspace [NR][ceil(C/64)]: requirement × cluster bitmask
  // device workspace written by prep_kernel at every launch
  struct UnitRec* rec;      // [W] per-unit records
  uint64_t* sw;             // [W][ceil(C/64)] static filter words: ClusterAffinity ∧ PlacementFilter
  uint64_t* cw;             // [W][ceil(C/64)] CurrentClusters words (units that have them)
  int32_t* defer;           // [W] units the lean kernel hands to schedule_kernel
  int32_t* defer_n;         // [1] length of defer
  int32_t* work_n;          // [1] lean kernel work queue: next batch of LEAN_BATCH units
  int use_rows;             // host: schedule_row_kernel runs (clean, folded, fit-folded snapshot, C <= ROW_MAX_C)
  int early_rows;           // host: the wide kernel runs on static words that are the whole filter, so prep_kernel
                            // routes units with more than WIDE_P feasible clusters to rows (REC_ROW) and the row
                            // kernel runs beside the wide kernel (a second stream) instead of after it
  int32_t* rows;            // [W] units whose feasible list outgrows the lean / wide kernels' registers
  int32_t* rows_n;          // [1] length of rows (reset by prep_kernel)
  int32_t* rows_head;       // [1] schedule_row_kernel's dequeue counter (reset by prep_kernel)
  char* row_slabs;          // [ROW_MAX_BLOCKS][row_slab_bytes(C)]: long replays' position scratch
  uint32_t* wq;             // [WQ_HEADS * WQ_STRIDE] schedule kernels' work heads (reset by prep_kernel)
};

// Per-unit record, rebuilt by prep_kernel at every kad_schedule: the fixed-size
// fields schedule_lean_kernel reads for one SchedulingUnit, in one 64-B line
// that lanes 0-15 fetch with a single coalesced load one unit ahead of use.
struct UnitRec {
  uint32_t flags;       // KAD_W_* | REC_DESIRED_POS
  int32_t gvk;          // snapshot GVK id (-1: none)
  int32_t tolset;       // toleration-set id
  int32_t sprog_off;    // ClusterAffinity score program offset
  int64_t req_cpu, req_mem;
  int64_t maxc;         // *MaxClusters
  int64_t out_off;      // first output slot
  uint64_t tol0;        // tol_all[tolset][0]
  uint64_t tolp0;       // tol_pns[tolset][0]
};
static_assert(sizeof(UnitRec) == 64, "UnitRec is one 64-B line");
constexpr uint32_t REC_DESIRED_POS = 1u << 31;  // DesiredReplicas != nil && *DesiredReplicas > 0
constexpr uint32_t REC_FULL = 1u << 30;         // scheduled by schedule_kernel (features the lean kernel omits)
constexpr uint32_t REC_ROW = 1u << 29;          // routed to schedule_row_kernel by prep_kernel (BatchDev::early_rows)
constexpr int ROW_MAX_TERMS = 8;                // schedule_row_kernel: preferred terms held as per-chunk words
constexpr int WIDE_Q = 8;                       // schedule_wide_kernel: positions per lane
constexpr int WIDE_P = WIDE_Q * 64;             //   and per wave (longer feasible lists: schedule_row_kernel)

struct OutDev {
  int32_t* status;
  int32_t* count;
  uint32_t* flags;
  int32_t* cluster;
  int64_t* replicas;
  uint8_t* dbg_feas;   // optional [W*C]
  int64_t* dbg_total;  // optional [W*C]
};

struct ProfDev {
  uint32_t filter_mask, score_mask;
  int32_t select_plugin, replicas_plugin;
  uint32_t flags;
};

// Rows for the stand-alone planner entry point (kad_plan_rows).
struct PlanRowsDev {
  int n_rows;
  const int32_t* row_off;
  const uint32_t* hash;
  const int64_t *weight, *min_r, *max_r, *cap, *current;
  const uint32_t* elem_flags;
  const int64_t* total;
  const uint32_t* row_flags;
  int64_t *out_plan, *out_overflow;
};

// Scheduling-trigger hash pipeline (kad_trigger.hip): device buffers of one run.
struct TriggerDev {
  int n;                          // objects
  const uint8_t* prefix;          // per-object bytes (CSR by prefix_off)
  const int64_t* prefix_off;      // [n+1]
  const uint32_t* suffix;         // shared cluster part (4-B aligned)
  int64_t suffix_len;             // bytes
  uint32_t* tables;               // [trigger_table_count][256] segment / composed tables
  uint32_t* powers;               // [trigger_table_count] p^len of each table's bytes
  uint32_t* out;                  // [n]
};
int64_t trigger_segment_len(int64_t suffix_len);
int64_t trigger_table_count(int64_t suffix_len);
hipError_t launch_trigger_summary(const TriggerDev& t, hipStream_t st);
hipError_t launch_trigger_objects(const TriggerDev& t, hipStream_t st);

// bytes of per-wave scratch for the filter/score/select kernel at C clusters
size_t select_wave_bytes(int C);
// true if schedule_row_kernel can take the long feasible lists of this snapshot (C <= ROW_MAX_C)
bool row_kernel_fits(int C);
constexpr int ROW_MAX_BLOCKS = 1024;  // schedule_row_kernel grid cap (its global slabs are sized for it)
__host__ __device__ size_t row_slab_bytes(int C);
size_t plan_wave_bytes(int K);

// phase counters of a -DKAD_PHASE_PROF build (returns 0 in product builds)
int debug_phase_counters(uint64_t* out, int reset);

// Tuning / measurement knobs read from the environment ONLY in profiling builds (-DKAD_PHASE_PROF,
// scripts/phase_prof.py; -DKAD_TUNING, scripts/wide_exp.py): the product library ignores the environment, so no variable set in a
// controller process can switch it off the reference-exact path (KAD_WIDE_EXPERIMENT, for one,
// skips the pdqsort replay). Product builds always return the default.
inline int tuning_env(const char* name, int dflt) {
#if defined(KAD_PHASE_PROF) || defined(KAD_TUNING)
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

// zero_rows: also empty the row list (BatchDev::rows_n, rows_head) before prep_kernel; *zeroed says whether
// a launched kernel did (else the caller clears it)
hipError_t launch_req_masks(const SnapDev& s, const BatchDev& b, hipStream_t st, bool zero_rows, bool* zeroed);
// per-id cluster bitmask slices of the snapshot (SnapDev::slices) and the taint table over them
// (SnapDev::taint_tab), rebuilt at upload / update
hipError_t launch_slices(const SnapDev& s, uint64_t* slices, hipStream_t st);
hipError_t launch_value_rows(const SnapDev& s, uint64_t* vrows, hipStream_t st);
// SnapDev::res4 / res_iv (+ pns4 when TW <= 4) of a clean snapshot (buf: 72 B per cluster: res4, res_iv, pns4)
hipError_t launch_res_cols(const SnapDev& s, void* buf, hipStream_t st);
inline size_t res_cols_pns4_offset(int C) { return ((size_t)40 * C + 255) & ~(size_t)255; }
inline size_t res_cols_bytes(int C) { return res_cols_pns4_offset(C) + (size_t)32 * C; }
// true if the batch runs on schedule_lean_kernel (+ schedule_kernel over its
// defer list); then launch_prep must run between launch_req_masks and launch_schedule.
bool fast_path(int C);
// true if launch_schedule runs schedule_wide_kernel for this snapshot (clean, 5..16 chunks)
bool wide_path(const SnapDev& s);
// prep_kernel lanes per unit (a power of two <= 64 lets it count a unit's feasible clusters in one wave)
int prep_lanes_per_unit(int C);
hipError_t launch_prep(const SnapDev& s, const BatchDev& b, const ProfDev& p, bool force_full, hipStream_t st);
// after_main / after_rows (optional): recorded after the main schedule kernel and after the long-row
// kernel, before the defer pass (stage timing)
hipError_t launch_schedule(const SnapDev& s, const BatchDev& b, const OutDev& o, const ProfDev& p,
                           void* global_scratch, size_t scratch_bytes, hipStream_t st, hipEvent_t after_main = nullptr,
                           hipEvent_t after_rows = nullptr, hipStream_t side = nullptr, hipEvent_t fork = nullptr,
                           hipEvent_t join = nullptr);
// One planner row's unit-level operands, gathered once per batch upload (plan_hdr_kernel) from the batch's
// per-unit arrays so that plan_kernel reads one 64-B line per row (its lanes 0..15 hold the dwords) instead
// of ten scattered per-unit loads one dependent step before everything else.
struct PlanRowHdr {
  int32_t w;          // unit
  uint32_t flags;     // KAD_W_*
  int64_t off;        // OUT_OFF[w]
  int32_t slots;      // OUT_OFF[w + 1] - OUT_OFF[w] (the unit's slot bound)
  int32_t p0, p1;     // PREF_OFF[w], PREF_OFF[w + 1]
  int32_t c0, c1;     // CUR_OFF[w], CUR_OFF[w + 1]
  int32_t k0, k1;     // KEY_OFF[w], KEY_OFF[w + 1]
  int32_t pad;
  int64_t desired;    // *DesiredReplicas
  int64_t pad2;
};
static_assert(sizeof(PlanRowHdr) == 64, "one line per planner row");
hipError_t launch_plan_hdr(const BatchDev& b, const int32_t* rows, int n_rows, PlanRowHdr* out, hipStream_t st);
// big / big_n: device list of planner rows (n_rows + 1 ints) for plan_pair_kernel's rows of 32 < K <= 64 (null:
// one row per wave throughout)
hipError_t launch_plan(const SnapDev& s, const BatchDev& b, const OutDev& o, const ProfDev& p, const PlanRowHdr* rows,
                       int n_rows, int kmax, void* global_scratch, size_t scratch_bytes, hipStream_t st,
                       int32_t* big = nullptr, int32_t* big_n = nullptr);
hipError_t launch_select_rows(int n_rows, const int32_t* row_off, const int64_t* scores, const int64_t* maxc,
                              uint32_t pflags, int kmax, int32_t* out_count, int32_t* out_sel, int32_t* out_status,
                              void* global_scratch, size_t scratch_bytes, hipStream_t st);
hipError_t launch_plan_rows(const PlanRowsDev& r, int kmax, int force_ws, void* global_scratch, size_t scratch_bytes,
                            hipStream_t st);

// kad_snapshot_update: scatter the changed clusters' columns of every snapshot
// array from a resident delta blob into the resident snapshot blob.
struct DeltaDev {
  uint8_t* snap;
  const uint8_t* delta;
  const int32_t* idx;  // [n] snapshot positions of the changed clusters
  int n, C;
  uint64_t s_off[KAD_S_NARRAYS], d_off[KAD_S_NARRAYS];
  int32_t esz[KAD_S_NARRAYS];
  int64_t start[KAD_S_NARRAYS + 1];  // prefix of rows(a) * n: element ranges per array
};
hipError_t launch_snapshot_delta(const DeltaDev& d, hipStream_t st);

// kad_result_diff (§8 f3): the last kad_schedule's outputs + the callers' current object state, canonical
// (placement ids sorted and unique per unit, names outside the snapshot folded into uflag bit 1)
struct ResultDiffDev {
  int W;
  const int32_t* status;
  const int32_t* count;
  const int32_t* cluster;
  const int64_t* replicas;
  const int64_t* out_off;  // [W + 1] (BatchDev::out_off)
  const int32_t* pl_off;   // [W + 1]
  const int32_t* pl_id;
  const uint8_t* uflag;    // bit 0: the scheduler's placement exists, bit 1: it names a cluster outside the snapshot
  const int32_t* ov_off;   // [W + 1]
  const int32_t* ov_id;
  const int64_t* ov_val;
  const uint8_t* ov_kind;
  uint32_t* out;           // [W] KAD_DIFF_*
};
hipError_t launch_result_diff(const ResultDiffDev& d, hipStream_t st);

}  // namespace kad

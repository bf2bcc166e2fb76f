// C ABI of libkad.so (include/kad_sched.h): context, residency, launch, results.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kad_sched.h"
#include "kad_device.h"
#include "kad_pool.h"

using namespace kad;

struct kad_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;                   // schedule_row_kernel beside the wide kernel (BatchDev::early_rows)
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  // stage events: 0 start, 3 after req_mask, 4 after prep, 5 after the main schedule kernel, 1 after the
  // defer pass, 2 after the planner
  hipEvent_t ev[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  std::mutex mu;
  std::string err;
  // snapshot
  void* d_snap = nullptr;
  size_t snap_bytes = 0;
  kad_snapshot_header snap_hdr{};
  SnapDev sd{};
  // batch
  void* d_batch = nullptr;
  size_t batch_cap = 0;
  kad_batch_header batch_hdr{};
  BatchDev bd{};
  std::vector<int32_t> plan_rows;
  int32_t* d_plan_rows = nullptr;
  size_t plan_rows_cap = 0;
  void* d_plan_hdr = nullptr;  // PlanRowHdr per planner row (plan_hdr_kernel at upload)
  void* d_plan_big = nullptr;  // i32[rows + 1]: plan_pair_kernel's list of rows for the 64-lane planner + its length
  size_t plan_big_cap = 0;
  size_t plan_hdr_cap = 0;
  // outputs
  int32_t *d_status = nullptr, *d_count = nullptr, *d_cluster = nullptr;
  uint32_t* d_flags = nullptr;
  int64_t* d_replicas = nullptr;
  size_t out_w_cap = 0, out_slot_cap = 0;
  uint64_t* d_req_mask = nullptr;
  size_t req_mask_cap = 0;
  std::vector<int32_t> h_reqseg;  // BatchDev::req_perm [NR][8] then req_seg [n_seg][4] (host copy until the next upload)
  void* d_reqseg = nullptr;
  size_t reqseg_cap = 0;
  int n_seg_reqs = 0;         // requirements on req_mask_kernel's segment path (the rest: value rows)
  void* d_vrows = nullptr;    // SnapDev::vrows
  size_t vrows_cap = 0;
  void* d_rescols = nullptr;  // SnapDev::res4 / res_iv
  size_t rescols_cap = 0;
  void* d_rowslab = nullptr;  // BatchDev::row_slabs
  size_t rowslab_cap = 0;
  void* d_rec = nullptr;  // UnitRec[W] (prep_kernel)
  size_t rec_cap = 0;
  void* d_sw = nullptr;   // u64[W][nch] static filter words (prep_kernel)
  size_t sw_cap = 0;
  void* d_cw = nullptr;   // u64[W][nch] current-cluster words (prep_kernel)
  size_t cw_cap = 0;
  void* d_defer = nullptr;  // i32[2W + 4]: defer_n, work_n, rows_n, rows_head, the defer list, the row list
  size_t defer_cap = 0;
  void* d_wq = nullptr;     // u32[WQ_HEADS * WQ_STRIDE]: schedule kernels' work heads
  size_t wq_cap = 0;
  // scratch (per-wave slabs for rows that do not fit LDS)
  void* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  bool have_snapshot = false, have_batch = false, ran = false;
  // the resident batch's units this ctx schedules: all of them, or a kad_group member's contiguous shard
  // [unit_lo, unit_lo + unit_n) whose output slots are [slot_lo, slot_lo + slot_n) of the batch's
  int64_t unit_lo = 0, unit_n = 0, slot_lo = 0, slot_n = 0;
  int inject_fault = 0;  // kad_debug_inject_fault: 1 = the next refresh_derived fails (tests)
  int plan_force_ws = 0;  // kad_debug_plan_force_workspace: kad_plan_rows through the workspace planner (tests)
  void* d_diff = nullptr;  // kad_result_diff: canonical object state + flags
  size_t diff_cap = 0;
  // HIP event records around the stages (kad_set_timing); timed = the last
  // kad_schedule recorded them
  bool timing = false, timed = false;
  bool snap_negative = false;  // some allocatable / used cpu or memory < 0 or >= 2^46 (odd score ranges)
  int clean_kind = 0;          // res_clean of the resident snapshot: 2 strict, 1 relaxed, 0 generic
  std::vector<int64_t> h_res;  // host shadow of alloc/used cpu/mem [4][C] (snap_negative after deltas)
  std::vector<uint64_t> h_ns;  // host shadow of the NoSchedule|NoExecute taint words [TW][C] (SnapDev::present_taints)
  void* d_slices = nullptr;    // SnapDev::slices [128*TW + 64*GW][nch], then SnapDev::taint_tab [2][8*TW][256][nch]
  size_t slices_cap = 0;
  std::vector<int64_t> h_fit;  // SnapDev::fit_vals / fit_rows (host copy the upload reads from)
  void* d_fit = nullptr;
  size_t fit_cap = 0;
  void* d_delta = nullptr;     // kad_snapshot_update: resident delta blob
  size_t delta_cap = 0;
  bool batch_defer = false;    // some unit uses a feature the lean kernel defers
  bool batch_zero_req = false;  // no unit has a ResourceRequest (BatchDev::zero_req)
  bool batch_many_terms = false;  // some unit has more than ROW_MAX_TERMS preferred terms (the row path defers it)
  // scheduling-trigger hashes (kad_trigger_*)
  void* t_suffix = nullptr;
  size_t t_suffix_cap = 0;
  int64_t t_suffix_len = -1;   // -1: no suffix uploaded
  void* t_prefix = nullptr;
  size_t t_prefix_cap = 0;
  void* t_work = nullptr;      // prefix_off, out
  size_t t_work_cap = 0;
  void* t_tabs = nullptr;      // segment / composed tables + powers of the suffix
  size_t t_tabs_cap = 0;
  int t_n = -1;                // -1: no prefixes uploaded
  bool t_ran = false;
  TriggerDev td{};
  hipEvent_t tev[4] = {nullptr, nullptr, nullptr, nullptr};
};

static int fail(kad_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPCHK(ctx, x)                                                                             \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return fail(ctx, KAD_EHIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

// Nothing unwinds through the C ABI: a host-side exception (std::bad_alloc from a check's or a planner
// row's vectors, rethrown by the worker pool once all its workers are done) becomes an error code.
template <class F>
static int guarded(kad_ctx* c, F f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return fail(c, KAD_ENOMEM, "host allocation failed");
  } catch (const std::exception& e) {  // e.g. std::system_error from a pool thread's creation
    return fail(c, KAD_EHOST, std::string("host error: ") + e.what());
  } catch (...) {
    return fail(c, KAD_EHOST, "host error: unknown exception");
  }
}

template <class T>
static const T* at(const void* base, const uint64_t* off, int i) {
  return reinterpret_cast<const T*>(static_cast<const char*>(base) + off[i]);
}

static int grow(kad_ctx* c, void** p, size_t* cap, size_t need) {
  if (need <= *cap && *p) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (need == 0) need = 256;
  hipError_t e = hipMalloc(p, need);
  if (e != hipSuccess) return fail(c, KAD_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  *cap = need;
  return 0;
}

template <class T>
static int to_dev(kad_ctx* c, const T* h, size_t n, T** d, std::vector<void*>& owned) {
  HIPCHK(c, hipMalloc((void**)d, (n ? n : 1) * sizeof(T)));
  owned.push_back(*d);
  if (n && h) HIPCHK(c, hipMemcpyAsync(*d, h, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return 0;
}

// ------------------------------------------------------ batch validation
// A batch blob may come from any packer (the Go port INTEGRATION.md proposes),
// so before anything is copied to the device every array is checked to lie in
// the blob, every CSR offset array to be monotone and to end inside its data
// array, every id the kernels index with to be in range, and every predicate
// program to be well formed — the kernels then read only inside the blob.
// [lo, hi) pieces of n on up to 16 host threads
template <class F>
static void host_parallel(int n, F f, int serial_below = 4096) {
  const int T = n < serial_below ? 1 : kadpool::pool().threads();
  if (T <= 1) {
    f(0, n);
    return;
  }
  kadpool::run_checks(T, [&](int t) { f((int)((int64_t)n * t / T), (int)((int64_t)n * (t + 1) / T)); });
}
// the smallest i in [0, n) with bad(i), or -1: pieces checked on up to 16 host threads, each
// stopping at its first failure or once an earlier one is known — the same index, so the same
// error, as one serial pass
template <class F>
static int64_t first_bad(int64_t n, F bad) {
  if (n < 65536) {
    for (int64_t i = 0; i < n; i++)
      if (bad(i)) return i;
    return -1;
  }
  std::atomic<int64_t> best{INT64_MAX};
  const int T = kadpool::pool().threads();
  kadpool::run_checks(T, [&](int t) {
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    for (int64_t i = lo; i < hi; i++) {
      if ((i & 1023) == 0 && i > best.load(std::memory_order_relaxed)) return;
      if (bad(i)) {
        int64_t cur = best.load();
        while (i < cur && !best.compare_exchange_weak(cur, i)) {
        }
        return;
      }
    }
  });
  const int64_t r = best.load();
  return r == INT64_MAX ? -1 : r;
}

namespace {
struct BatchCheck {
  kad_ctx* c;
  const char* base;
  size_t nbytes;
  const kad_batch_header& h;
  // array a holds count elements of esz bytes inside the blob
  bool extent(int a, uint64_t count, int esz, const char* what) {
    const uint64_t o = h.off[a];
    if (o > nbytes || (o % (uint64_t)esz) || count > (nbytes - o) / (uint64_t)esz) {
      fail(c, KAD_EINVAL, std::string("batch array ") + what + " lies outside the blob");
      return false;
    }
    return true;
  }
  template <class T>
  const T* arr(int a) const { return reinterpret_cast<const T*>(base + h.off[a]); }
  // CSR offsets off_a[0..n]: 0-based, non-decreasing; the data array d has off[n] elements of esz bytes
  bool csr(int off_a, int n, int data_a, int esz, const char* what, int64_t* total) {
    if (!extent(off_a, (uint64_t)n + 1, 4, what)) return false;
    const int32_t* o = arr<int32_t>(off_a);
    if (o[0] != 0) return fail(c, KAD_EINVAL, std::string(what) + " offsets must start at 0"), false;
    if (first_bad(n, [o](int64_t i) { return o[i + 1] < o[i]; }) >= 0)
      return fail(c, KAD_EINVAL, std::string(what) + " offsets must be non-decreasing"), false;
    *total = o[n];
    return data_a < 0 || extent(data_a, (uint64_t)o[n], esz, what);
  }
  // each row's ids in [lo, hi), ascending (strictly when unique)
  bool sorted_ids(int off_a, int ids_a, int n, int lo, int hi, bool unique, const char* what) {
    const int32_t* o = arr<int32_t>(off_a);
    const int32_t* v = arr<int32_t>(ids_a);
    // 0 ok, 1 out of range, 2 not ascending: the first failing element of row w
    auto row = [=](int64_t w) {
      for (int j = o[w]; j < o[w + 1]; j++) {
        if (v[j] < lo || v[j] >= hi) return 1;
        if (j > o[w] && (unique ? v[j] <= v[j - 1] : v[j] < v[j - 1])) return 2;
      }
      return 0;
    };
    const int64_t w = first_bad(n, [&](int64_t w) { return row(w) != 0; });
    if (w < 0) return true;
    return fail(c, KAD_EINVAL, std::string(what) + (row(w) == 1 ? " id out of range" : " ids must be ascending")), false;
  }
};
}  // namespace

static int validate_batch(kad_ctx* c, const void* blob, size_t nbytes, const kad_batch_header& h) {
  const kad_snapshot_header& sh = c->snap_hdr;
  const int W = h.n_units, C = sh.n_clusters, TW = h.n_taint_words, NT = h.n_tolsets, NR = h.n_reqs;
  if (W < 0 || NT < 0 || NR < 0 || (W > 0 && NT < 1)) return fail(c, KAD_EINVAL, "bad batch counts");
  for (int i = 0; i < KAD_B_NARRAYS; i++)
    if (h.off[i] > nbytes || (h.off[i] & 7)) return fail(c, KAD_EINVAL, "bad batch array offset");
  BatchCheck k{c, static_cast<const char*>(blob), nbytes, h};
  const uint64_t Wu = (uint64_t)W;
  if (!k.extent(KAD_B_FLAGS, Wu, 4, "flags") || !k.extent(KAD_B_GVK, Wu, 4, "gvk") ||
      !k.extent(KAD_B_REQ_CPU, Wu, 8, "req_cpu") || !k.extent(KAD_B_REQ_MEM, Wu, 8, "req_mem") ||
      !k.extent(KAD_B_DESIRED, Wu, 8, "desired") || !k.extent(KAD_B_MAX_CLUSTERS, Wu, 8, "max_clusters") ||
      !k.extent(KAD_B_TOLSET, Wu, 4, "tolset") || !k.extent(KAD_B_TOL_ALL, (uint64_t)NT * TW, 8, "tol_all") ||
      !k.extent(KAD_B_TOL_PNS, (uint64_t)NT * TW, 8, "tol_pns") || !k.extent(KAD_B_OUT_OFF, Wu + 1, 8, "out_off"))
    return KAD_EINVAL;
  if ((h.flags & ~KAD_BATCH_NARROW_PREFS) != 0 || h.reserved != 0)
    return fail(c, KAD_EINVAL, "batch: unknown header flags");
  const uint32_t pvb = (h.flags & KAD_BATCH_NARROW_PREFS) ? 4u : 8u;  // bytes per preference value
  int64_t n_s, n_f, n_sp, n_pl, n_cur, n_pref, n_key, n_req;
  if (!k.csr(KAD_B_SREQ_OFF, W, KAD_B_SREQ_ID, 4, "sreq", &n_s) || !k.extent(KAD_B_SREQ_VAL, n_s, 8, "sreq_val") ||
      !k.csr(KAD_B_FPROG_OFF, W, KAD_B_FPROG, 4, "fprog", &n_f) ||
      !k.csr(KAD_B_SPROG_OFF, W, KAD_B_SPROG, 4, "sprog", &n_sp) ||
      !k.csr(KAD_B_PLACE_OFF, W, KAD_B_PLACE, 4, "place", &n_pl) ||
      !k.csr(KAD_B_CUR_OFF, W, KAD_B_CUR_ID, 4, "cur", &n_cur) || !k.extent(KAD_B_CUR_REP, n_cur, 8, "cur_rep") ||
      !k.csr(KAD_B_PREF_OFF, W, KAD_B_PREF_ID, 4, "pref", &n_pref) ||
      !k.extent(KAD_B_PREF_W, n_pref, pvb, "pref_w") || !k.extent(KAD_B_PREF_MIN, n_pref, pvb, "pref_min") ||
      !k.extent(KAD_B_PREF_MAX, n_pref, pvb, "pref_max") || !k.extent(KAD_B_PREF_CAP, n_pref, pvb, "pref_cap") ||
      !k.extent(KAD_B_PREF_FLAGS, n_pref, 4, "pref_flags") || !k.csr(KAD_B_KEY_OFF, W, KAD_B_KEY, 1, "key", &n_key) ||
      !k.csr(KAD_B_REQ_OFF, NR, KAD_B_REQ, 4, "req", &n_req))
    return KAD_EINVAL;
  if (!k.sorted_ids(KAD_B_PLACE_OFF, KAD_B_PLACE, W, 0, C, true, "placement") ||
      !k.sorted_ids(KAD_B_CUR_OFF, KAD_B_CUR_ID, W, 0, C, true, "current cluster") ||
      !k.sorted_ids(KAD_B_PREF_OFF, KAD_B_PREF_ID, W, 0, C, true, "preference"))
    return KAD_EINVAL;
  const uint32_t* fl = k.arr<uint32_t>(KAD_B_FLAGS);
  const int32_t* gv = k.arr<int32_t>(KAD_B_GVK);
  const int32_t* ts = k.arr<int32_t>(KAD_B_TOLSET);
  const int64_t* mc = k.arr<int64_t>(KAD_B_MAX_CLUSTERS);
  const int64_t* oo = k.arr<int64_t>(KAD_B_OUT_OFF);
  const int32_t* sid = k.arr<int32_t>(KAD_B_SREQ_ID);
  const int32_t* po = k.arr<int32_t>(KAD_B_PLACE_OFF);
  if (first_bad(n_s, [&](int64_t j) { return sid[j] < -1 || sid[j] >= sh.n_scalar; }) >= 0)
    return fail(c, KAD_EINVAL, "scalar request id out of range");
  // output slot ranges must hold every pair the kernels can write for the packed
  // profile: min(C, MaxClusters, |ClusterNames|) (pack.py Batch), 0 when sticky
  if (oo[0] != 0 || oo[W] != h.n_out_slots) return fail(c, KAD_EINVAL, "out_off must run from 0 to n_out_slots");
  const bool sel_max = h.packed_select_plugin == KAD_PL_MAX_CLUSTER;
  const bool place_on = h.packed_filter_mask & (1u << KAD_PL_PLACEMENT_FILTER);
  auto unit_err = [&](int64_t w) -> const char* {
    if (gv[w] < -1 || gv[w] >= 64 * sh.n_gvk_words) return "gvk id out of range";
    if (ts[w] < 0 || ts[w] >= NT) return "toleration-set id out of range";
    const int64_t len = oo[w + 1] - oo[w];
    if (len < 0 || len > h.max_row_slots) return "output slot range exceeds max_row_slots";
    int64_t bound = C;
    if (sel_max && (fl[w] & KAD_W_HAS_MAX_CLUSTERS) && mc[w] >= 0 && mc[w] < bound) bound = mc[w];
    if (place_on && (fl[w] & KAD_W_HAS_PLACEMENT) && po[w + 1] - po[w] < bound) bound = po[w + 1] - po[w];
    if (fl[w] & KAD_W_STICKY) bound = 0;
    if (len < bound) return "output slot range smaller than the unit's selection bound";
    return nullptr;
  };
  if (const int64_t w = first_bad(W, [&](int64_t w) { return unit_err(w) != nullptr; }); w >= 0)
    return fail(c, KAD_EINVAL, unit_err(w));
  if (h.max_row_slots < 0 || h.max_row_slots > (C > 0 ? C : 1)) return fail(c, KAD_EINVAL, "bad max_row_slots");
  // requirement table: [op | n << 8, key, payload...]
  const int32_t* ro = k.arr<int32_t>(KAD_B_REQ_OFF);
  const int32_t* rq = k.arr<int32_t>(KAD_B_REQ);
  auto req_err = [&](int64_t r) -> const char* {
    const int len = ro[r + 1] - ro[r];
    if (len < 2) return "requirement shorter than two words";
    const int32_t* p = rq + ro[r];
    const int op = p[0] & 0xff, n = (int)((uint32_t)p[0] >> 8), key = p[1];
    if (len != 2 + n) return "requirement payload length mismatch";
    switch (op) {
      case KAD_OP_IN: case KAD_OP_NOTIN: case KAD_OP_EQ:
        if (key < 0 || key >= sh.n_label_keys || n < 1) return "bad label requirement";
        break;
      case KAD_OP_EXISTS: case KAD_OP_DNE:
        if (key < 0 || key >= sh.n_label_keys || n != 0) return "bad label requirement";
        break;
      case KAD_OP_GT: case KAD_OP_LT:
        if (key < 0 || key >= sh.n_label_keys || n != 2) return "bad Gt/Lt requirement";
        break;
      case KAD_OP_NAME_EQ: case KAD_OP_NAME_NE:
        if (key < -1 || key >= C) return "bad field requirement";
        break;
      case KAD_OP_TRUE: case KAD_OP_FALSE:
        break;
      default:
        return "unknown requirement op";
    }
    return nullptr;
  };
  if (const int64_t r = first_bad(NR, [&](int64_t r) { return req_err(r) != nullptr; }); r >= 0)
    return fail(c, KAD_EINVAL, req_err(r));
  // programs: every requirement id in range, structure consumes exactly the unit's words
  const int32_t* fo = k.arr<int32_t>(KAD_B_FPROG_OFF);
  const int32_t* fp = k.arr<int32_t>(KAD_B_FPROG);
  const int32_t* spo = k.arr<int32_t>(KAD_B_SPROG_OFF);
  const int32_t* sp = k.arr<int32_t>(KAD_B_SPROG);
  auto ids_ok = [&](const int32_t* p, int at, int n, int len) {
    if (n < 0 || at + n > len) return false;
    for (int i = 0; i < n; i++)
      if (p[at + i] < 0 || p[at + i] >= NR) return false;
    return true;
  };
  // 0 ok, 1 malformed filter program, 2 malformed score program
  auto prog_err = [&](int64_t w) {
    const int32_t* p = fp + fo[w];
    const int len = fo[w + 1] - fo[w];
    bool ok = len >= 2;
    int pc = 0;
    if (ok) {
      const int n_sel = p[pc++];
      ok = ids_ok(p, pc, n_sel, len);
      pc += ok ? n_sel : 0;
      ok = ok && pc < len;
      if (ok && p[pc++]) {
        ok = pc < len;
        const int n_terms = ok ? p[pc++] : 0;
        ok = ok && n_terms >= 0;
        for (int t = 0; ok && t < n_terms; t++) {
          ok = pc + 3 <= len;
          if (!ok) break;
          const int ne = p[pc + 1], nf = p[pc + 2];
          ok = ne >= 0 && nf >= 0 && ids_ok(p, pc + 3, ne + nf, len);
          pc += 3 + (ok ? ne + nf : 0);
        }
      }
    }
    if (!ok || pc != len) return 1;
    p = sp + spo[w];
    const int sl = spo[w + 1] - spo[w];
    ok = sl >= 1;
    pc = 0;
    if (ok) {
      const int n_terms = p[pc++];
      ok = n_terms >= 0;
      for (int t = 0; ok && t < n_terms; t++) {
        ok = pc + 2 <= sl;
        if (!ok) break;
        const int ne = p[pc + 1];
        ok = ids_ok(p, pc + 2, ne, sl);
        pc += 2 + (ok ? ne : 0);
      }
    }
    if (!ok || pc != sl) return 2;
    return 0;

  };
  if (const int64_t w = first_bad(W, [&](int64_t w) { return prog_err(w) != 0; }); w >= 0)
    return fail(c, KAD_EINVAL, std::string(prog_err(w) == 1 ? "malformed filter program of unit " : "malformed score program of unit ") + std::to_string(w));
  return 0;
}

extern "C" {

int kad_abi_version(void) { return KAD_ABI_VERSION; }

int kad_ctx_create(int hip_device, kad_ctx** out) {
  if (!out) return KAD_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return KAD_EHIP;
  if (hip_device < 0 || hip_device >= n) return KAD_EINVAL;
  auto* c = new kad_ctx();
  c->device = hip_device;
  if (hipSetDevice(hip_device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return KAD_EHIP;
  }
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming) != hipSuccess) {
    kad_ctx_destroy(c);
    return KAD_EHIP;
  }
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) {
      kad_ctx_destroy(c);
      return KAD_EHIP;
    }
  for (auto& e : c->tev)
    if (hipEventCreate(&e) != hipSuccess) {
      kad_ctx_destroy(c);
      return KAD_EHIP;
    }
  *out = c;
  return KAD_OK;
}

int kad_ctx_destroy(kad_ctx* c) {
  if (!c) return KAD_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->side) (void)hipStreamSynchronize(c->side);  // the row kernel may run there: drain it before any free
  for (void* p : {c->d_snap, c->d_batch, (void*)c->d_plan_rows, c->d_plan_hdr, c->d_plan_big, (void*)c->d_req_mask, (void*)c->d_status, (void*)c->d_count,
                  (void*)c->d_cluster, (void*)c->d_flags, (void*)c->d_replicas, c->d_scratch, c->d_rec, c->d_delta, c->d_sw, c->d_cw, c->d_defer, c->d_wq, c->d_slices, c->d_fit, c->d_reqseg, c->d_rowslab, c->d_vrows, c->d_rescols,
                  c->t_suffix, c->t_prefix, c->t_work, c->t_tabs, c->d_diff})
    if (p) (void)hipFree(p);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->tev)
    if (e) (void)hipEventDestroy(e);
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
  }
  for (hipEvent_t e : {c->fork_ev, c->join_ev})
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return KAD_OK;
}

const char* kad_last_error(kad_ctx* c) { return c ? c->err.c_str() : "null context"; }

static int bind_snapshot(kad_ctx* c, const kad_snapshot_header& h) {
  const char* base = static_cast<const char*>(c->d_snap);
  SnapDev& s = c->sd;
  s.C = h.n_clusters;
  s.GW = h.n_gvk_words;
  s.TW = h.n_taint_words;
  s.K = h.n_label_keys;
  s.S = h.n_scalar;
  s.alloc_cpu = at<int64_t>(base, h.off, KAD_S_ALLOC_CPU);
  s.alloc_mem = at<int64_t>(base, h.off, KAD_S_ALLOC_MEM);
  s.used_cpu = at<int64_t>(base, h.off, KAD_S_USED_CPU);
  s.used_mem = at<int64_t>(base, h.off, KAD_S_USED_MEM);
  s.alloc_s = at<int64_t>(base, h.off, KAD_S_ALLOC_SCALAR);
  s.used_s = at<int64_t>(base, h.off, KAD_S_USED_SCALAR);
  s.alloc_cores = at<int64_t>(base, h.off, KAD_S_ALLOC_CORES);
  s.avail_cores = at<int64_t>(base, h.off, KAD_S_AVAIL_CORES);
  s.gvk = at<uint64_t>(base, h.off, KAD_S_GVK);
  s.nsne = at<uint64_t>(base, h.off, KAD_S_TAINT_NSNE);
  s.ne = at<uint64_t>(base, h.off, KAD_S_TAINT_NE);
  s.pns = at<uint64_t>(base, h.off, KAD_S_TAINT_PNS);
  s.lval = at<int32_t>(base, h.off, KAD_S_LABEL_VAL);
  s.lint = at<int64_t>(base, h.off, KAD_S_LABEL_INT);
  s.lok = at<uint8_t>(base, h.off, KAD_S_LABEL_INT_OK);
  s.name_fnv = at<uint32_t>(base, h.off, KAD_S_NAME_FNV);
  if (s.C < 0 || s.C > 65535) return fail(c, KAD_EINVAL, "n_clusters must be in [0, 65535]");
  return 0;
}


static const int kResArrays[4] = {KAD_S_ALLOC_CPU, KAD_S_ALLOC_MEM, KAD_S_USED_CPU, KAD_S_USED_MEM};

static bool res_negative(const std::vector<int64_t>& v) {
  bool neg = false;
  for (int64_t x : v) neg |= x < 0 || x >= (1ll << 46);
  return neg;
}
// The exact-f64 resource path (SnapDev::clean) per cluster and resource r in {cpu, memory}, allocatable a and
// used u = allocatable - available:
//   2 (strict)  every cluster has 1 <= a < 2^46 and 0 <= u <= a;
//   1 (relaxed) every cluster has 0 <= a < 2^46 and 0 <= u < 2^46, some with a = 0 or u > a — what
//     aggregateResources (federatedcluster/util.go:178-214) reports for a cluster whose cordoned / tainted
//     nodes are left out of allocatable while their pods still count (:183-189, :199-210): available < 0,
//     or allocatable 0 when every node is left out;
//   0 otherwise (the generic int64 path: Go's wrap-around, used < 0 from Resource.Sub errors).
// Relaxed clusters score through the same f64 expressions (SnapDev::clean), which are exact for them as
// long as their Fit test does not read the cached operands: the folded filter (fit threshold rows, exact
// int64 compares of available against the request) — refresh_derived enables them only then. Their score
// operands: score_res (kad_device.h).
static int res_clean(const std::vector<int64_t>& v) {
  const size_t C = v.size() / 4;
  int strict = 1;
  for (size_t c = 0; c < C; c++)
    for (int r = 0; r < 2; r++) {
      const int64_t a = v[r * C + c], u = v[(2 + r) * C + c];
      if (a < 0 || a >= (1ll << 46) || u < 0 || u >= (1ll << 46)) return 0;
      strict &= a >= 1 && u <= a;
    }
  return strict ? 2 : 1;
}

// rows and element size of snapshot array a (include/kad_sched.h, enum kad_snapshot_array)
static void snapshot_array_shape(const kad_snapshot_header& h, int a, int64_t* rows, int* esz) {
  *rows = 1;
  *esz = 8;
  switch (a) {
    case KAD_S_ALLOC_SCALAR: case KAD_S_USED_SCALAR: *rows = h.n_scalar; break;
    case KAD_S_GVK: *rows = h.n_gvk_words; break;
    case KAD_S_TAINT_NSNE: case KAD_S_TAINT_NE: case KAD_S_TAINT_PNS: *rows = h.n_taint_words; break;
    case KAD_S_LABEL_VAL: *rows = h.n_label_keys; *esz = 4; break;
    case KAD_S_LABEL_INT: *rows = h.n_label_keys; break;
    case KAD_S_LABEL_INT_OK: *rows = h.n_label_keys; *esz = 1; break;
    case KAD_S_NAME_FNV: case KAD_S_CFLAGS: *esz = 4; break;
    default: break;
  }
}

// every array of the snapshot lies inside the blob: rows(a) * C elements of its size at an aligned offset
static int check_snapshot_header(kad_ctx* c, const kad_snapshot_header& h, size_t nbytes) {
  if (nbytes < sizeof(h) || h.magic != KAD_SNAPSHOT_MAGIC) return fail(c, KAD_EINVAL, "bad snapshot magic");
  if (h.abi_version != KAD_ABI_VERSION) return fail(c, KAD_EINVAL, "snapshot ABI version mismatch");
  if (h.total_bytes != nbytes) return fail(c, KAD_EINVAL, "snapshot size mismatch");
  if (h.n_clusters < 0 || h.n_clusters > 65535) return fail(c, KAD_EINVAL, "n_clusters must be in [0, 65535]");
  // the kernels read GVK and taint word 0 of every cluster
  if (h.n_gvk_words < 1 || h.n_taint_words < 1 || h.n_label_keys < 0 || h.n_scalar < 0)
    return fail(c, KAD_EINVAL, "snapshot needs n_gvk_words >= 1, n_taint_words >= 1, n_label_keys >= 0, n_scalar >= 0");
  for (int i = 0; i < KAD_S_NARRAYS; i++) {
    int64_t rows;
    int esz;
    snapshot_array_shape(h, i, &rows, &esz);
    const uint64_t len = (uint64_t)rows * (uint64_t)h.n_clusters * (uint64_t)esz;
    if (h.off[i] > nbytes || (h.off[i] & 7) || len > nbytes - h.off[i])
      return fail(c, KAD_EINVAL, "snapshot array " + std::to_string(i) + " lies outside the blob");
  }
  return 0;
}

// SnapDev::fit_vals / fit_rows from the host shadow of the resources (clean snapshots, C <= FITFOLD_MAX_C)
static int build_fit_table(kad_ctx* c) {
  const int C = c->sd.C;
  c->sd.fitfold = 0;
  if (!c->sd.clean || C <= 0 || C > FITFOLD_MAX_C) return 0;
  // (available may be negative on relaxed clusters: the rows compare exact int64 amounts, available >= request
  // <=> allocatable >= request + (allocatable - available) of fit.go:89,98 without overflow below 2^46)
  const int nch = (C + 63) / 64;
  std::vector<int64_t> vals[2];
  std::vector<int> order(C);
  size_t words = 0;
  for (int r = 0; r < 2; r++) {
    vals[r].resize(C);
    for (int x = 0; x < C; x++) vals[r][x] = c->h_res[(size_t)r * C + x] - c->h_res[(size_t)(2 + r) * C + x];
    std::vector<int64_t> u = vals[r];
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    c->sd.fit_m[r] = (int)u.size();
  }
  int mp = FIT_FENCES;  // vals padded with INT64_MAX to a power of two >= m + 1 (fence search)
  while (mp < c->sd.fit_m[0] + 1 || mp < c->sd.fit_m[1] + 1) mp *= 2;
  c->sd.fit_mp = mp;
  for (int r = 0; r < 2; r++) words += (size_t)mp + ((size_t)c->sd.fit_m[r] + 1) * nch;
  c->h_fit.assign(words, 0);
  size_t o = 0;
  size_t vo[2], ro[2];
  for (int r = 0; r < 2; r++) {  // vals
    const int m = c->sd.fit_m[r];
    std::vector<int64_t> u = vals[r];
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    vo[r] = o;
    std::copy(u.begin(), u.end(), c->h_fit.begin() + (ptrdiff_t)o);
    std::fill(c->h_fit.begin() + (ptrdiff_t)(o + m), c->h_fit.begin() + (ptrdiff_t)(o + mp), INT64_MAX);
    o += (size_t)mp;
  }
  for (int r = 0; r < 2; r++) {  // rows, from the largest amount down: row j = row j+1 | clusters at vals[j]
    const int m = c->sd.fit_m[r];
    const int64_t* u = c->h_fit.data() + vo[r];
    ro[r] = o;
    for (int x = 0; x < C; x++) order[x] = x;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return vals[r][a] > vals[r][b]; });
    uint64_t* rows = reinterpret_cast<uint64_t*>(c->h_fit.data() + o);
    int q = 0;
    for (int j = m - 1; j >= 0; j--) {
      std::memcpy(rows + (size_t)j * nch, rows + (size_t)(j + 1) * nch, (size_t)nch * 8);
      for (; q < C && vals[r][order[q]] == u[j]; q++) rows[(size_t)j * nch + (order[q] >> 6)] |= 1ull << (order[q] & 63);
    }
    o += ((size_t)m + 1) * nch;
  }
  if (int r = grow(c, &c->d_fit, &c->fit_cap, words * 8)) return r;
  HIPCHK(c, hipMemcpyAsync(c->d_fit, c->h_fit.data(), words * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));  // h_fit may be rebuilt by the next upload / update
  const int64_t* d = static_cast<const int64_t*>(c->d_fit);
  for (int r = 0; r < 2; r++) {
    c->sd.fit_vals[r] = d + vo[r];
    c->sd.fit_rows[r] = reinterpret_cast<const uint64_t*>(d + ro[r]);
  }
  c->sd.fitfold = 1;
  return 0;
}

// state derived from the resident snapshot: clean / negative ranges (host shadows) and, with up to
// TFOLD_MAX_TW taint words, the per-id cluster slices + taint table prep_kernel folds the taint and API
// filters from (SnapDev::fold)
// SnapDev::vrows: per label key, clusters holding value id s < VR_SLOTS, and clusters with the key
static int build_value_rows(kad_ctx* c) {
  const int C = c->sd.C, K = c->sd.K;
  const size_t nch = (size_t)((C + 63) / 64);
  const size_t bytes = (size_t)K * (VR_SLOTS + 1) * nch * 8;
  c->sd.vrows = nullptr;
  if (C <= 0 || K <= 0 || bytes > VR_MAX_BYTES) return 0;
  if (int r = grow(c, &c->d_vrows, &c->vrows_cap, bytes)) return r;
  c->sd.vrows = static_cast<const uint64_t*>(c->d_vrows);
  HIPCHK(c, launch_value_rows(c->sd, static_cast<uint64_t*>(c->d_vrows), c->stream));
  return 0;
}

static int refresh_derived(kad_ctx* c) {
  if (c->inject_fault == 1) {
    c->inject_fault = 0;
    return fail(c, KAD_ENOMEM, "injected refresh_derived failure (kad_debug_inject_fault)");
  }
  if (int r = build_value_rows(c)) return r;
  c->snap_negative = res_negative(c->h_res);
  const int C = c->sd.C, TW = c->sd.TW;
  {
    // relaxed clusters (res_clean 1) take the fast path only with the filter folded: taint / API words
    // (fold, decided below from the same sizes) and the fit threshold rows (build_fit_table: C <= FITFOLD_MAX_C)
    const size_t nc1 = C > 0 ? (size_t)((C + 63) / 64) : 1;
    const size_t fold_words = ((size_t)128 * TW + (size_t)64 * c->sd.GW) * nc1 + (size_t)2 * 8 * TW * 256 * nc1;
    const bool can_fold = TW >= 1 && TW <= TFOLD_MAX_TW && fold_words * 8 <= TTAB_MAX_BYTES;
    const int rc = res_clean(c->h_res);
    c->clean_kind = rc;
    c->sd.clean = rc == 2 || (rc == 1 && can_fold && C > 0 && C <= FITFOLD_MAX_C);
  }
  c->sd.res4 = nullptr;
  c->sd.res_iv = nullptr;
  c->sd.pns4 = nullptr;
  if (c->sd.clean && C > 0) {
    if (int r = grow(c, &c->d_rescols, &c->rescols_cap, res_cols_bytes(C))) return r;
    HIPCHK(c, launch_res_cols(c->sd, c->d_rescols, c->stream));
    c->sd.res4 = static_cast<const double4*>(c->d_rescols);
    c->sd.res_iv = reinterpret_cast<const float2*>(c->sd.res4 + C);
    if (TW <= 4)
      c->sd.pns4 = reinterpret_cast<const ulonglong4*>(static_cast<const char*>(c->d_rescols) + res_cols_pns4_offset(C));
  }
  c->sd.fold = TW >= 1 && TW <= TFOLD_MAX_TW;
  for (int t = 0; t < TFOLD_MAX_TW; t++) {
    uint64_t present = 0;
    if (t < TW)
      for (int x = 0; x < C; x++) present |= c->h_ns[(size_t)t * C + x];
    c->sd.present_taints[t] = present;
  }
  const size_t nch = (size_t)((C + 63) / 64);
  const size_t nc1 = nch ? nch : 1;
  const size_t n_slices = ((size_t)128 * TW + (size_t)64 * c->sd.GW) * nc1, n_tab = (size_t)2 * 8 * TW * 256 * nc1;
  // the table is rebuilt whole on every upload / update: above TTAB_MAX_BYTES (C beyond ~32k clusters at
  // 4 taint words) the kernels test taints per cluster instead (unfolded path)
  if (c->sd.fold && (n_slices + n_tab) * 8 > TTAB_MAX_BYTES) c->sd.fold = 0;
  if (!c->sd.fold) return build_fit_table(c);
  if (int r = grow(c, &c->d_slices, &c->slices_cap, (n_slices + n_tab) * 8)) return r;
  c->sd.slices = static_cast<const uint64_t*>(c->d_slices);
  c->sd.taint_tab = c->sd.slices + n_slices;
  HIPCHK(c, launch_slices(c->sd, static_cast<uint64_t*>(c->d_slices), c->stream));
  return build_fit_table(c);
}

// nothing resident may be scheduled: the snapshot (and so any batch validated against it) is being replaced
static void invalidate_snapshot(kad_ctx* c) {
  c->have_snapshot = false;
  c->have_batch = false;
  c->ran = false;
}

static int snapshot_upload_locked(kad_ctx* c, const void* blob, size_t nbytes);

int kad_snapshot_upload(kad_ctx* c, const void* blob, size_t nbytes) {
  return guarded(c, [&]() -> int {
    if (!c || !blob) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return snapshot_upload_locked(c, blob, nbytes);
  });
}

static int snapshot_upload_locked(kad_ctx* c, const void* blob, size_t nbytes) {
  kad_snapshot_header h;
  std::memcpy(&h, blob, sizeof(h) < nbytes ? sizeof(h) : nbytes);
  if (int r = check_snapshot_header(c, h, nbytes)) return r;
  // the resident snapshot, its derived state and any batch validated against it are about to be
  // overwritten: nothing may run on them until every step below has succeeded
  invalidate_snapshot(c);
  HIPCHK(c, hipSetDevice(c->device));
  if (int r = grow(c, &c->d_snap, &c->snap_bytes, nbytes)) return r;
  HIPCHK(c, hipMemcpyAsync(c->d_snap, blob, nbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->snap_hdr = h;
  if (int r = bind_snapshot(c, h)) return r;
  c->h_res.assign((size_t)4 * h.n_clusters, 0);
  {
    for (int q = 0; q < 4; q++)
      if (h.n_clusters) std::memcpy(c->h_res.data() + (size_t)q * h.n_clusters, at<int64_t>(blob, h.off, kResArrays[q]), (size_t)h.n_clusters * 8);
  }
  c->h_ns.assign(at<uint64_t>(blob, h.off, KAD_S_TAINT_NSNE),
                at<uint64_t>(blob, h.off, KAD_S_TAINT_NSNE) + (size_t)h.n_taint_words * h.n_clusters);
  if (int r = refresh_derived(c)) return r;
  c->have_snapshot = true;
  return KAD_OK;
}

// kad_group: member c takes the snapshot resident on member src (same vocabulary and host shadows) with
// one device-to-device copy (xGMI between two GPUs) and rebuilds its derived state on its own device
static int snapshot_from_peer_locked(kad_ctx* c, kad_ctx* src) {
  if (!src->have_snapshot) return fail(c, KAD_ESTATE, "source member has no snapshot");
  invalidate_snapshot(c);
  const size_t nbytes = src->snap_hdr.total_bytes;
  HIPCHK(c, hipSetDevice(c->device));
  if (int r = grow(c, &c->d_snap, &c->snap_bytes, nbytes)) return r;
  if (c->device == src->device)
    HIPCHK(c, hipMemcpyAsync(c->d_snap, src->d_snap, nbytes, hipMemcpyDeviceToDevice, c->stream));
  else
    HIPCHK(c, hipMemcpyPeerAsync(c->d_snap, c->device, src->d_snap, src->device, nbytes, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->snap_hdr = src->snap_hdr;
  if (int r = bind_snapshot(c, c->snap_hdr)) return r;
  c->h_res = src->h_res;
  c->h_ns = src->h_ns;
  if (int r = refresh_derived(c)) return r;
  c->have_snapshot = true;
  return KAD_OK;
}

int kad_snapshot_upload_device(kad_ctx* c, const void* dev_blob, size_t nbytes) {
  return guarded(c, [&]() -> int {
    if (!c || !dev_blob) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    kad_snapshot_header h;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(&h, dev_blob, sizeof(h), hipMemcpyDeviceToHost));
    if (int r = check_snapshot_header(c, h, nbytes)) return r;
    invalidate_snapshot(c);
    if (int r = grow(c, &c->d_snap, &c->snap_bytes, nbytes)) return r;
    HIPCHK(c, hipMemcpyAsync(c->d_snap, dev_blob, nbytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->snap_hdr = h;
    if (int r = bind_snapshot(c, h)) return r;
    c->h_res.assign((size_t)4 * h.n_clusters, 0);
    c->h_ns.assign((size_t)h.n_taint_words * h.n_clusters, 0);
    if (h.n_clusters) {
      for (int q = 0; q < 4; q++)
        HIPCHK(c, hipMemcpy(c->h_res.data() + (size_t)q * h.n_clusters, static_cast<const char*>(dev_blob) + h.off[kResArrays[q]],
                            (size_t)h.n_clusters * 8, hipMemcpyDeviceToHost));
      HIPCHK(c, hipMemcpy(c->h_ns.data(), static_cast<const char*>(dev_blob) + h.off[KAD_S_TAINT_NSNE],
                          (size_t)h.n_taint_words * h.n_clusters * 8, hipMemcpyDeviceToHost));
    }
    if (int r = refresh_derived(c)) return r;
    c->have_snapshot = true;
    return KAD_OK;
  });
}

static int snapshot_update_locked(kad_ctx* c, const void* delta, size_t nbytes);

int kad_snapshot_update(kad_ctx* c, const void* delta, size_t nbytes) {
  return guarded(c, [&]() -> int {
    if (!c || !delta) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return snapshot_update_locked(c, delta, nbytes);
  });
}

static int snapshot_update_locked(kad_ctx* c, const void* delta, size_t nbytes) {
  if (!c->have_snapshot) return fail(c, KAD_ESTATE, "no snapshot uploaded");
  kad_snapshot_delta_header h;
  if (nbytes < sizeof(h)) return fail(c, KAD_EINVAL, "delta too small");
  std::memcpy(&h, delta, sizeof(h));
  const kad_snapshot_header& sh = c->snap_hdr;
  if (h.magic != KAD_DELTA_MAGIC) return fail(c, KAD_EINVAL, "bad delta magic");
  if (h.abi_version != KAD_ABI_VERSION) return fail(c, KAD_EINVAL, "delta ABI version mismatch");
  if (h.total_bytes != nbytes) return fail(c, KAD_EINVAL, "delta size mismatch");
  if (h.n_clusters != sh.n_clusters || h.fingerprint != sh.fingerprint)
    return fail(c, KAD_EINVAL, "delta was packed against a different snapshot vocabulary");
  const int n = h.n_changed, C = sh.n_clusters;
  if (n < 0 || n > C) return fail(c, KAD_EINVAL, "bad n_changed");
  if (n == 0) return KAD_OK;
  if (h.idx_off > nbytes || (h.idx_off & 3) || h.idx_off + (uint64_t)n * 4 > nbytes)
    return fail(c, KAD_EINVAL, "bad delta index offset");
  const int32_t* idx = reinterpret_cast<const int32_t*>(static_cast<const char*>(delta) + h.idx_off);
  for (int j = 0; j < n; j++)
    if (idx[j] < 0 || idx[j] >= C || (j && idx[j] <= idx[j - 1]))
      return fail(c, KAD_EINVAL, "delta cluster indices must be strictly increasing snapshot positions");
  DeltaDev d{};
  d.n = n;
  d.C = C;
  d.start[0] = 0;
  for (int a = 0; a < KAD_S_NARRAYS; a++) {
    int64_t rows;
    int esz;
    snapshot_array_shape(sh, a, &rows, &esz);
    const uint64_t len = (uint64_t)rows * n * esz;
    if (h.off[a] > nbytes || (h.off[a] % esz) || h.off[a] + len > nbytes)
      return fail(c, KAD_EINVAL, "bad delta array offset");
    d.s_off[a] = sh.off[a];
    d.d_off[a] = h.off[a];
    d.esz[a] = esz;
    d.start[a + 1] = d.start[a] + rows * n;
  }
  HIPCHK(c, hipSetDevice(c->device));
  if (int r = grow(c, &c->d_delta, &c->delta_cap, nbytes)) return r;
  HIPCHK(c, hipMemcpyAsync(c->d_delta, delta, nbytes, hipMemcpyHostToDevice, c->stream));
  d.snap = static_cast<uint8_t*>(c->d_snap);
  d.delta = static_cast<const uint8_t*>(c->d_delta);
  d.idx = reinterpret_cast<const int32_t*>(d.delta + h.idx_off);
  {
    hipError_t e = launch_snapshot_delta(d, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // the caller's delta buffer is free on return
    if (e != hipSuccess) {
      invalidate_snapshot(c);  // the scatter may have run partway
      return fail(c, KAD_EHIP, std::string("snapshot delta scatter: ") + hipGetErrorString(e));
    }
  }
  {
    for (int q = 0; q < 4; q++) {
      const int64_t* v = at<int64_t>(delta, h.off, kResArrays[q]);
      for (int j = 0; j < n; j++) c->h_res[(size_t)q * C + idx[j]] = v[j];
    }
    const uint64_t* ns = at<uint64_t>(delta, h.off, KAD_S_TAINT_NSNE);  // [TW][n_changed]
    for (int t = 0; t < sh.n_taint_words; t++)
      for (int j = 0; j < n; j++) c->h_ns[(size_t)t * C + idx[j]] = ns[(size_t)t * n + j];
  }
  if (int r = refresh_derived(c)) {
    invalidate_snapshot(c);  // the scattered snapshot no longer matches its derived rows / tables
    return r;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KAD_OK;
}

// The host-side batch array extents a shard [lo, hi) of units reads (kad_group members): per-unit arrays
// [lo, hi) (offset arrays [lo, hi]), CSR data between its units' offsets, batch-wide tables whole. Each
// entry: (array, first byte, bytes) relative to the array's offset.
struct BlobRange {
  int a;
  uint64_t first, bytes;
};
static std::vector<BlobRange> shard_ranges(const void* blob, const kad_batch_header& h, int64_t lo, int64_t hi) {
  std::vector<BlobRange> out;
  const uint64_t n = (uint64_t)(hi - lo);
  auto unit = [&](int a, int esz) { out.push_back({a, (uint64_t)lo * esz, n * esz}); };
  auto offs = [&](int a, int esz) { out.push_back({a, (uint64_t)lo * esz, (n + 1) * esz}); };
  auto csr = [&](int off_a, std::initializer_list<std::pair<int, int>> data) {
    offs(off_a, 4);
    const int32_t* o = at<int32_t>(blob, h.off, off_a);
    for (auto [a, esz] : data) out.push_back({a, (uint64_t)o[lo] * esz, (uint64_t)(o[hi] - o[lo]) * esz});
  };
  const int pvb = (h.flags & KAD_BATCH_NARROW_PREFS) ? 4 : 8;
  for (int a : {KAD_B_FLAGS, KAD_B_GVK, KAD_B_TOLSET}) unit(a, 4);
  for (int a : {KAD_B_REQ_CPU, KAD_B_REQ_MEM, KAD_B_DESIRED, KAD_B_MAX_CLUSTERS}) unit(a, 8);
  offs(KAD_B_OUT_OFF, 8);
  csr(KAD_B_SREQ_OFF, {{KAD_B_SREQ_ID, 4}, {KAD_B_SREQ_VAL, 8}});
  csr(KAD_B_FPROG_OFF, {{KAD_B_FPROG, 4}});
  csr(KAD_B_SPROG_OFF, {{KAD_B_SPROG, 4}});
  csr(KAD_B_PLACE_OFF, {{KAD_B_PLACE, 4}});
  csr(KAD_B_CUR_OFF, {{KAD_B_CUR_ID, 4}, {KAD_B_CUR_REP, 8}});
  csr(KAD_B_PREF_OFF, {{KAD_B_PREF_ID, 4}, {KAD_B_PREF_W, pvb}, {KAD_B_PREF_MIN, pvb}, {KAD_B_PREF_MAX, pvb},
                       {KAD_B_PREF_CAP, pvb}, {KAD_B_PREF_FLAGS, 4}});
  csr(KAD_B_KEY_OFF, {{KAD_B_KEY, 1}});
  const uint64_t tol = (uint64_t)h.n_tolsets * (uint64_t)h.n_taint_words * 8;
  out.push_back({KAD_B_TOL_ALL, 0, tol});
  out.push_back({KAD_B_TOL_PNS, 0, tol});
  out.push_back({KAD_B_REQ_OFF, 0, ((uint64_t)h.n_reqs + 1) * 4});
  out.push_back({KAD_B_REQ, 0, (uint64_t)at<int32_t>(blob, h.off, KAD_B_REQ_OFF)[h.n_reqs] * 4});
  return out;
}

// lo, hi: the units this ctx schedules (hi < 0: all); a shard copies only the blob bytes it reads
// (shard_ranges) into a device buffer of the whole blob's layout, so every offset stays valid. validated:
// the caller (kad_group_batch_upload) has run validate_batch on this blob already.
static int batch_upload_locked(kad_ctx* c, const void* blob, size_t nbytes, int64_t lo = 0, int64_t hi = -1,
                               bool validated = false) {
  // any failed upload leaves no batch resident (validation failed, or device buffers half-written)
  c->have_batch = false;
  c->ran = false;
  if (!c->have_snapshot) return fail(c, KAD_ESTATE, "no snapshot uploaded");
  kad_batch_header h;
  if (nbytes < sizeof(h)) return fail(c, KAD_EINVAL, "batch too small");
  std::memcpy(&h, blob, sizeof(h));
  if (h.magic != KAD_BATCH_MAGIC) return fail(c, KAD_EINVAL, "bad batch magic");
  if (h.abi_version != KAD_ABI_VERSION) return fail(c, KAD_EINVAL, "batch ABI version mismatch");
  if (h.total_bytes != nbytes) return fail(c, KAD_EINVAL, "batch size mismatch");
  if (h.snapshot_fingerprint != c->snap_hdr.fingerprint || h.n_clusters != c->snap_hdr.n_clusters ||
      h.n_taint_words != c->snap_hdr.n_taint_words)
    return fail(c, KAD_EINVAL, "batch was packed against a different snapshot");
  // KAD_UPLOAD_TIMING: host-side laps of the upload on stderr (measurement builds only: tuning_env)
  static const bool tm = tuning_env("KAD_UPLOAD_TIMING", 0) != 0;
  auto t_prev = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!tm) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[kad_upload] %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_prev).count());
    t_prev = t;
  };
  if (!validated)
    if (int r = validate_batch(c, blob, nbytes, h)) return r;
  lap("validate");
  if (hi < 0) hi = h.n_units;
  if (lo < 0 || lo > hi || hi > h.n_units) return fail(c, KAD_EINVAL, "bad unit range");
  const bool shard = lo > 0 || hi < h.n_units;
  HIPCHK(c, hipSetDevice(c->device));
  // 256 B of slack past the blob: the schedule kernels read a unit's score program as a 64-word window from
  // its offset (affinity_score_pv), which may run past the last array
  if (int r = grow(c, &c->d_batch, &c->batch_cap, nbytes + 256)) return r;
  if (!shard) {
    HIPCHK(c, hipMemcpyAsync(c->d_batch, blob, nbytes, hipMemcpyHostToDevice, c->stream));
  } else {
    char* d = static_cast<char*>(c->d_batch);
    const char* hb = static_cast<const char*>(blob);
    HIPCHK(c, hipMemcpyAsync(d, hb, sizeof(h), hipMemcpyHostToDevice, c->stream));
    for (const BlobRange& r : shard_ranges(blob, h, lo, hi))
      if (r.bytes)
        HIPCHK(c, hipMemcpyAsync(d + h.off[r.a] + r.first, hb + h.off[r.a] + r.first, r.bytes, hipMemcpyHostToDevice,
                                 c->stream));
  }
  lap("dma-issue");
  const int W = (int)(hi - lo);
  const int64_t* oo_h = at<int64_t>(blob, h.off, KAD_B_OUT_OFF);
  const int64_t slot_lo = oo_h[lo], S = oo_h[hi] - oo_h[lo];
  // rows that need the replica planner: Divide mode, DesiredReplicas > 0, not sticky (unit ids of the shard)
  const uint32_t* fl = at<uint32_t>(blob, h.off, KAD_B_FLAGS) + lo;
  const int64_t* des = at<int64_t>(blob, h.off, KAD_B_DESIRED) + lo;
  uint32_t flags_or = 0;
  // batch_defer: units the lean kernel would defer whatever the profile (prep_kernel's
  // REC_FULL reasons; wide affinity weights or negative requests can give
  // totals spanning >= 2^32)
  {
    const int32_t* gv = at<int32_t>(blob, h.off, KAD_B_GVK) + lo;
    const int32_t* so = at<int32_t>(blob, h.off, KAD_B_SREQ_OFF) + lo;
    const int64_t* rc = at<int64_t>(blob, h.off, KAD_B_REQ_CPU) + lo;
    const int64_t* rm = at<int64_t>(blob, h.off, KAD_B_REQ_MEM) + lo;
    c->batch_defer = first_bad(W, [&](int64_t w) {
      return (gv[w] >= 64 && !c->sd.fold) || so[w] < so[w + 1] || rc[w] < 0 || rm[w] < 0 || rc[w] >= (1ll << 46) ||
             rm[w] >= (1ll << 46) || (fl[w] & KAD_W_WIDE_SCORES);
    }) >= 0;
    c->batch_zero_req = first_bad(W, [&](int64_t w) { return rc[w] != 0 || rm[w] != 0; }) < 0;
    const int32_t* spo = at<int32_t>(blob, h.off, KAD_B_SPROG_OFF) + lo;
    const int32_t* sp = at<int32_t>(blob, h.off, KAD_B_SPROG);
    c->batch_many_terms = first_bad(W, [&](int64_t w) { return sp[spo[w]] > ROW_MAX_TERMS; }) >= 0;
  }
  {
    // plan rows in unit order: per-piece counts, then each piece writes at its prefix. (Grouping them by path
    // class — dynamic weights × avoid disruption — so that plan_pair_kernel's pairs share their passes made the
    // pair kernel 11 % slower: neighbouring rows then lie ~4 units apart and share fewer lines of the per-unit
    // columns; profiles/r06/ab_c4_planner_occupancy_classes.txt)
    constexpr int PIECES = 16;
    int64_t cnt[PIECES + 1] = {};
    uint32_t ors[PIECES] = {};
    auto plan = [&](int w) {
      const uint32_t f = fl[w];
      return !(f & KAD_W_DUPLICATE) && !(f & KAD_W_STICKY) && (f & KAD_W_HAS_DESIRED) && des[w] > 0;
    };
    auto pieces = [&](auto&& body) {
      host_parallel(
          PIECES,
          [&](int a, int b) {
            for (int q = a; q < b; q++) body(q, (int)((int64_t)W * q / PIECES), (int)((int64_t)W * (q + 1) / PIECES));
          },
          W < 65536 ? PIECES + 1 : 0);
    };
    pieces([&](int q, int lo, int hi) {
      uint32_t o = 0;
      int64_t n = 0;
      for (int w = lo; w < hi; w++) {
        o |= fl[w];
        n += plan(w);
      }
      ors[q] = o;
      cnt[q + 1] = n;
    });
    for (int q = 0; q < PIECES; q++) {
      flags_or |= ors[q];
      cnt[q + 1] += cnt[q];
    }
    c->plan_rows.resize((size_t)cnt[PIECES]);
    pieces([&](int q, int lo, int hi) {
      int32_t* o = c->plan_rows.data() + cnt[q];
      for (int w = lo; w < hi; w++)
        if (plan(w)) *o++ = w;
    });
  }
  if (int r = grow(c, (void**)&c->d_plan_rows, &c->plan_rows_cap, c->plan_rows.size() * 4)) return r;
  if (!c->plan_rows.empty())
    HIPCHK(c, hipMemcpyAsync(c->d_plan_rows, c->plan_rows.data(), c->plan_rows.size() * 4, hipMemcpyHostToDevice,
                             c->stream));
  // outputs
  size_t wcap = c->out_w_cap, scap = c->out_slot_cap;
  if ((size_t)W > c->out_w_cap || !c->d_status) {
    if (c->d_status) { (void)hipFree(c->d_status); (void)hipFree(c->d_count); (void)hipFree(c->d_flags); }
    c->d_status = c->d_count = nullptr;
    c->d_flags = nullptr;
    wcap = W > 0 ? W : 1;
    HIPCHK(c, hipMalloc(&c->d_status, wcap * 4));
    HIPCHK(c, hipMalloc(&c->d_count, wcap * 4));
    HIPCHK(c, hipMalloc(&c->d_flags, wcap * 4));
    c->out_w_cap = wcap;
  }
  const size_t slots = S > 0 ? (size_t)S : 1;
  if (slots > scap || !c->d_cluster) {
    if (c->d_cluster) { (void)hipFree(c->d_cluster); (void)hipFree(c->d_replicas); }
    HIPCHK(c, hipMalloc(&c->d_cluster, slots * 4));
    HIPCHK(c, hipMalloc(&c->d_replicas, slots * 8));
    c->out_slot_cap = slots;
  }
  // scratch for rows whose state does not fit LDS
  size_t need = 0;
  const size_t sw = select_wave_bytes(c->sd.C);
  if (sw > 64 * 1024) need = sw * (W < 8192 ? (W > 0 ? W : 1) : 8192);
  const size_t pw = plan_wave_bytes(h.max_row_slots);
  if (pw > 64 * 1024) {
    size_t n2 = pw * (c->plan_rows.size() < 8192 ? (c->plan_rows.empty() ? 1 : c->plan_rows.size()) : 8192);
    need = need > n2 ? need : n2;
  }
  if (need > c->scratch_bytes) {
    if (c->d_scratch) (void)hipFree(c->d_scratch);
    c->d_scratch = nullptr;
    c->scratch_bytes = 0;
    HIPCHK(c, hipMalloc(&c->d_scratch, need));
    c->scratch_bytes = need;
  }
  const size_t nch = (size_t)((c->sd.C + 63) / 64);
  if (int r = grow(c, (void**)&c->d_req_mask, &c->req_mask_cap, (size_t)h.n_reqs * nch * 8)) return r;
  // Label requirements whose value ids are all < VR_SLOTS (at most VR_MAX_VALS of them; Exists / DoesNotExist)
  // read the snapshot's value rows (req_row_kernel: a word is the OR of <= 5 row words); so do the label-free
  // ops (TRUE / FALSE / metadata.name =, !=), whose words are constants or one bit. The rest is grouped
  // by label key (req_mask_kernel: one label-row load per segment and chunk): a counting sort by key, cut
  // into segments of <= seg_len ids; shorter segments when the batch has few requirements, so the grid
  // still fills the chip.
  int n_seg = 0, n_rowreq = 0;
  {
    const int NR = h.n_reqs, K = c->snap_hdr.n_label_keys;
    const int32_t* ro = at<int32_t>(blob, h.off, KAD_B_REQ_OFF);
    const int32_t* rq = at<int32_t>(blob, h.off, KAD_B_REQ);
    const bool vr = c->sd.vrows != nullptr;
    auto by_rows = [&](int r) {
      const int32_t* q = rq + ro[r];
      const int op = q[0] & 0xff, n = (int)((uint32_t)q[0] >> 8);
      // label-free ops: their words need no snapshot data at all
      if (op == KAD_OP_TRUE || op == KAD_OP_FALSE || op == KAD_OP_NAME_EQ || op == KAD_OP_NAME_NE) return true;
      if (!vr) return false;
      if (op == KAD_OP_EXISTS || op == KAD_OP_DNE) return true;
      if (op != KAD_OP_IN && op != KAD_OP_NOTIN && op != KAD_OP_EQ) return false;
      if (n > VR_MAX_VALS) return false;
      for (int t = 0; t < n; t++)
        if (q[2 + t] < 0 || q[2 + t] >= VR_SLOTS) return false;
      return true;
    };
    // the segment path sees label requirements only (by_rows takes every label-free op): group = label key
    auto group = [&](int r) { return rq[ro[r] + 1]; };
    std::vector<uint8_t> rowr((size_t)NR);
    std::vector<int32_t> start((size_t)K + 2, 0);
    host_parallel(NR, [&](int lo, int hi) {
      for (int r = lo; r < hi; r++) rowr[r] = by_rows(r);
    });
    for (int r = 0; r < NR; r++) {
      if (rowr[r])
        n_rowreq++;
      else
        start[(size_t)group(r) + 1]++;
    }
    const int NS = NR - n_rowreq;  // requirements on the segment path
    for (int g = 0; g <= K; g++) start[(size_t)g + 1] += start[g];
    const long ngrp = ((long)nch + REQ_SEG_G - 1) / REQ_SEG_G;
    int seg_len = 64;
    while (seg_len > 8 && (long)NS * ngrp / seg_len < 16384) seg_len /= 2;
    long segs = 0;
    for (int g = 0; g <= K; g++) segs += (start[(size_t)g + 1] - start[g] + seg_len - 1) / seg_len;
    // entry e of req_perm: 8 words (id, word offset, op | n << 8, key word, payload 0..3) so a lane
    // fetches its requirement with two 16-B loads, independent of the segment's label-row loads;
    // value-row entries: (id, op | n << 8, key, value ids 0..4)
    const size_t perm_len = (size_t)NS * 8, seg_len_w = 4 * (size_t)segs;
    c->h_reqseg.assign(perm_len + seg_len_w + (size_t)n_rowreq * 8, 0);
    std::vector<int32_t> fill(start.begin(), start.end() - 1);
    int32_t* rows_e = c->h_reqseg.data() + perm_len + seg_len_w;
    int nr2 = 0;
    for (int r = 0; r < NR; r++) {
      const int32_t* q = rq + ro[r];
      const int n = (int)((uint32_t)q[0] >> 8);
      if (rowr[r]) {
        int32_t* e = rows_e + 8 * (size_t)nr2++;
        e[0] = r;
        e[1] = q[0];
        e[2] = q[1];
        for (int t = 0; t < VR_MAX_VALS && t < n; t++) e[3 + t] = q[2 + t];
        continue;
      }
      int32_t* e = c->h_reqseg.data() + 8 * (size_t)fill[(size_t)group(r)]++;
      e[0] = r;
      e[1] = ro[r];
      e[2] = q[0];
      e[3] = q[1];
      for (int t = 0; t < 4 && t < n; t++) e[4 + t] = q[2 + t];
    }
    int32_t* sg = c->h_reqseg.data() + perm_len;
    for (int g = 0; g <= K; g++)
      for (int f = start[g]; f < start[(size_t)g + 1]; f += seg_len) {
        sg[4 * n_seg] = g;
        sg[4 * n_seg + 1] = f;
        sg[4 * n_seg + 2] = start[(size_t)g + 1] - f < seg_len ? start[(size_t)g + 1] - f : seg_len;
        n_seg++;
      }
    if (int r = grow(c, &c->d_reqseg, &c->reqseg_cap, c->h_reqseg.size() * 4 + 16)) return r;
    if (!c->h_reqseg.empty())
      HIPCHK(c, hipMemcpyAsync(c->d_reqseg, c->h_reqseg.data(), c->h_reqseg.size() * 4, hipMemcpyHostToDevice, c->stream));
    c->n_seg_reqs = NS;
  }

  lap("segments");
  if (int r = grow(c, &c->d_rec, &c->rec_cap, (size_t)W * sizeof(UnitRec))) return r;
  if (int r = grow(c, &c->d_sw, &c->sw_cap, (size_t)W * nch * 8)) return r;
  if (int r = grow(c, &c->d_cw, &c->cw_cap, (size_t)W * nch * 8)) return r;
  if (int r = grow(c, &c->d_defer, &c->defer_cap, (2 * (size_t)W + 4) * 4)) return r;
  if (int r = grow(c, &c->d_wq, &c->wq_cap, (size_t)WQ_HEADS * WQ_STRIDE * 4)) return r;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  lap("sync");
  c->batch_hdr = h;
  c->unit_lo = lo;
  c->unit_n = W;
  c->slot_lo = slot_lo;
  c->slot_n = S;
  const char* base = static_cast<const char*>(c->d_batch);
  BatchDev& b = c->bd;
  b.W = W;
  b.flags_or = flags_or;
  b.zero_req = c->batch_zero_req ? 1 : 0;
  b.NT = h.n_tolsets;
  b.TW = h.n_taint_words;
  b.flags = at<uint32_t>(base, h.off, KAD_B_FLAGS);
  b.gvk = at<int32_t>(base, h.off, KAD_B_GVK);
  b.req_cpu = at<int64_t>(base, h.off, KAD_B_REQ_CPU);
  b.req_mem = at<int64_t>(base, h.off, KAD_B_REQ_MEM);
  b.desired = at<int64_t>(base, h.off, KAD_B_DESIRED);
  b.maxc = at<int64_t>(base, h.off, KAD_B_MAX_CLUSTERS);
  b.tolset = at<int32_t>(base, h.off, KAD_B_TOLSET);
  b.tol_all = at<uint64_t>(base, h.off, KAD_B_TOL_ALL);
  b.tol_pns = at<uint64_t>(base, h.off, KAD_B_TOL_PNS);
  b.sreq_off = at<int32_t>(base, h.off, KAD_B_SREQ_OFF);
  b.sreq_id = at<int32_t>(base, h.off, KAD_B_SREQ_ID);
  b.sreq_val = at<int64_t>(base, h.off, KAD_B_SREQ_VAL);
  b.fprog_off = at<int32_t>(base, h.off, KAD_B_FPROG_OFF);
  b.fprog = at<int32_t>(base, h.off, KAD_B_FPROG);
  b.sprog_off = at<int32_t>(base, h.off, KAD_B_SPROG_OFF);
  b.sprog = at<int32_t>(base, h.off, KAD_B_SPROG);
  b.place_off = at<int32_t>(base, h.off, KAD_B_PLACE_OFF);
  b.place = at<int32_t>(base, h.off, KAD_B_PLACE);
  b.cur_off = at<int32_t>(base, h.off, KAD_B_CUR_OFF);
  b.cur_id = at<int32_t>(base, h.off, KAD_B_CUR_ID);
  b.cur_rep = at<int64_t>(base, h.off, KAD_B_CUR_REP);
  b.pref_off = at<int32_t>(base, h.off, KAD_B_PREF_OFF);
  b.pref_id = at<int32_t>(base, h.off, KAD_B_PREF_ID);
  b.pref_narrow = (h.flags & KAD_BATCH_NARROW_PREFS) ? 1 : 0;
  b.pref_w = b.pref_narrow ? nullptr : at<int64_t>(base, h.off, KAD_B_PREF_W);
  b.pref_min = b.pref_narrow ? nullptr : at<int64_t>(base, h.off, KAD_B_PREF_MIN);
  b.pref_max = b.pref_narrow ? nullptr : at<int64_t>(base, h.off, KAD_B_PREF_MAX);
  b.pref_cap = b.pref_narrow ? nullptr : at<int64_t>(base, h.off, KAD_B_PREF_CAP);
  b.pref_w32 = b.pref_narrow ? at<int32_t>(base, h.off, KAD_B_PREF_W) : nullptr;
  b.pref_min32 = b.pref_narrow ? at<int32_t>(base, h.off, KAD_B_PREF_MIN) : nullptr;
  b.pref_max32 = b.pref_narrow ? at<int32_t>(base, h.off, KAD_B_PREF_MAX) : nullptr;
  b.pref_cap32 = b.pref_narrow ? at<int32_t>(base, h.off, KAD_B_PREF_CAP) : nullptr;
  b.pref_fl = at<uint32_t>(base, h.off, KAD_B_PREF_FLAGS);
  b.key_off = at<int32_t>(base, h.off, KAD_B_KEY_OFF);
  b.key = at<uint8_t>(base, h.off, KAD_B_KEY);
  b.out_off = at<int64_t>(base, h.off, KAD_B_OUT_OFF);
  // a shard: every per-unit array starts at its first unit (CSR offsets and out_off keep their batch-wide
  // values, so the data arrays and the output slots are indexed as in the whole batch; OutDev's slot
  // arrays are shifted by slot_lo instead, out_dev)
  b.flags += lo;
  b.gvk += lo;
  b.req_cpu += lo;
  b.req_mem += lo;
  b.desired += lo;
  b.maxc += lo;
  b.tolset += lo;
  b.sreq_off += lo;
  b.fprog_off += lo;
  b.sprog_off += lo;
  b.place_off += lo;
  b.cur_off += lo;
  b.pref_off += lo;
  b.key_off += lo;
  b.out_off += lo;
  b.NR = h.n_reqs;
  b.req_off = at<int32_t>(base, h.off, KAD_B_REQ_OFF);
  b.req = at<int32_t>(base, h.off, KAD_B_REQ);
  b.req_mask = c->d_req_mask;
  b.n_seg = n_seg;
  b.req_perm = static_cast<const int32_t*>(c->d_reqseg);
  b.req_seg = reinterpret_cast<const int4*>(static_cast<const int32_t*>(c->d_reqseg) + (size_t)c->n_seg_reqs * 8);
  b.n_rowreq = n_rowreq;
  b.req_rows = reinterpret_cast<const int4*>(reinterpret_cast<const int32_t*>(b.req_seg) + 4 * (size_t)n_seg);
  b.rec = static_cast<UnitRec*>(c->d_rec);
  b.sw = static_cast<uint64_t*>(c->d_sw);
  b.cw = static_cast<uint64_t*>(c->d_cw);
  b.defer_n = static_cast<int32_t*>(c->d_defer);
  b.work_n = b.defer_n + 1;
  b.rows_n = b.defer_n + 2;
  b.rows_head = b.defer_n + 3;
  b.defer = b.defer_n + 4;
  b.rows = b.defer + W;
  b.wq = static_cast<uint32_t*>(c->d_wq);
  // the planner rows' unit-level operands in one line per row (plan_kernel), gathered on the device
  if (int r = grow(c, &c->d_plan_hdr, &c->plan_hdr_cap, c->plan_rows.size() * sizeof(PlanRowHdr))) return r;
  if (int r = grow(c, &c->d_plan_big, &c->plan_big_cap, (c->plan_rows.size() + 1) * sizeof(int32_t))) return r;
  HIPCHK(c, launch_plan_hdr(b, c->d_plan_rows, (int)c->plan_rows.size(), static_cast<PlanRowHdr*>(c->d_plan_hdr),
                            c->stream));
  c->have_batch = true;
  c->ran = false;
  return KAD_OK;
}

int kad_batch_upload(kad_ctx* c, const void* blob, size_t nbytes) {
  return guarded(c, [&]() -> int {
    if (!c || !blob) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return batch_upload_locked(c, blob, nbytes);
  });
}

static int validate_profile(kad_ctx* c, const kad_profile* p) {
  if (!p) return fail(c, KAD_EINVAL, "null profile");
  const uint32_t filters = (1u << KAD_PL_API_RESOURCES) | (1u << KAD_PL_TAINT_TOLERATION) |
                           (1u << KAD_PL_CLUSTER_RESOURCES_FIT) | (1u << KAD_PL_PLACEMENT_FILTER) |
                           (1u << KAD_PL_CLUSTER_AFFINITY);
  const uint32_t scores = (1u << KAD_PL_TAINT_TOLERATION) | (1u << KAD_PL_BALANCED_ALLOCATION) |
                          (1u << KAD_PL_LEAST_ALLOCATED) | (1u << KAD_PL_MOST_ALLOCATED) |
                          (1u << KAD_PL_CLUSTER_AFFINITY);
  if (p->filter_mask & ~filters) return fail(c, KAD_EUNSUPPORTED, "filter plugin outside the in-tree set");
  if (p->score_mask & ~scores) return fail(c, KAD_EUNSUPPORTED, "score plugin outside the in-tree set");
  if (p->select_plugin != -1 && p->select_plugin != KAD_PL_MAX_CLUSTER)
    return fail(c, KAD_EUNSUPPORTED, "select plugin outside the in-tree set");
  if (p->replicas_plugin != -1 && p->replicas_plugin != KAD_PL_CLUSTER_CAPACITY_WEIGHT)
    return fail(c, KAD_EUNSUPPORTED, "replicas plugin outside the in-tree set");
  return 0;
}

static OutDev out_dev(kad_ctx* c) {
  OutDev o{};
  o.status = c->d_status;
  o.count = c->d_count;
  o.flags = c->d_flags;
  // the kernels write slot out_off[w] (batch-wide): a shard's buffer holds slots [slot_lo, slot_lo + slot_n)
  o.cluster = reinterpret_cast<int32_t*>(reinterpret_cast<uintptr_t>(c->d_cluster) - 4 * (uintptr_t)c->slot_lo);
  o.replicas = reinterpret_cast<int64_t*>(reinterpret_cast<uintptr_t>(c->d_replicas) - 8 * (uintptr_t)c->slot_lo);
  return o;
}

static int schedule_locked(kad_ctx* c, const kad_profile* p, uint8_t* dbg_feas, int64_t* dbg_total) {
  if (!c->have_snapshot || !c->have_batch) return fail(c, KAD_ESTATE, "snapshot and batch must be uploaded first");
  if (int r = validate_profile(c, p)) return r;
  if (p->filter_mask != c->batch_hdr.packed_filter_mask || p->select_plugin != c->batch_hdr.packed_select_plugin)
    return fail(c, KAD_EINVAL, "profile differs from the one the batch output bounds were packed for");
  HIPCHK(c, hipSetDevice(c->device));
  ProfDev pd{p->filter_mask, p->score_mask, p->select_plugin, p->replicas_plugin, p->flags};
  OutDev o = out_dev(c);
  o.dbg_feas = dbg_feas;
  o.dbg_total = dbg_total;
  const bool tm = c->timing;
  // long feasible lists go to schedule_row_kernel when every filter is in the static words
  const bool no_rows = tuning_env("KAD_NO_ROWS", 0) != 0;  // (read per launch: tuning builds only)
  c->bd.use_rows = !no_rows && c->sd.clean && c->sd.fold && c->sd.fitfold && row_kernel_fits(c->sd.C);
  const bool rows_after = tuning_env("KAD_ROWS_AFTER", 0) != 0;
  const int per = prep_lanes_per_unit(c->sd.C);
  const bool wide = wide_path(c->sd);
  c->bd.early_rows = c->bd.use_rows && !rows_after && wide && (per & (per - 1)) == 0 && per <= 64 &&
                     !dbg_feas && !dbg_total;
  // can any unit reach the defer list (schedule_kernel)? The wide kernel with early routing (every filter in
  // the static words, long lists routed by prep) defers only the units batch_defer names; the row path also
  // those with more preferred terms than it holds. Otherwise as before: the lean kernel's own reasons, and
  // on the wide path without early routing, lists past WIDE_P.
  const bool rows_defer = c->batch_many_terms && (p->score_mask & (1u << KAD_PL_CLUSTER_AFFINITY));
  if (wide)
    c->bd.may_defer = c->batch_defer || dbg_feas || dbg_total || !c->bd.early_rows || rows_defer;
  else
    c->bd.may_defer = c->batch_defer || c->snap_negative || c->sd.TW > 1 || dbg_feas || dbg_total;
  if (c->bd.use_rows) {
    if (int r = grow(c, &c->d_rowslab, &c->rowslab_cap, (size_t)ROW_MAX_BLOCKS * row_slab_bytes(c->sd.C))) return r;
    c->bd.row_slabs = static_cast<char*>(c->d_rowslab);
  }
  // early_rows: prep_kernel appends to the row list from all its blocks, so the list is emptied before it
  // starts (rows_n, rows_head: two adjacent words) — by req_row_kernel when it runs, else a memset
  if (tm) HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  bool zeroed = false;
  HIPCHK(c, launch_req_masks(c->sd, c->bd, c->stream, c->bd.early_rows, &zeroed));
  if (tm) HIPCHK(c, hipEventRecord(c->ev[3], c->stream));
  if (c->bd.early_rows && !zeroed) HIPCHK(c, hipMemsetAsync(c->bd.rows_n, 0, 2 * sizeof(int32_t), c->stream));
  if (fast_path(c->sd.C))
    HIPCHK(c, launch_prep(c->sd, c->bd, pd, dbg_feas || dbg_total, c->stream));
  if (tm) HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
  if (tm) HIPCHK(c, hipEventRecord(c->ev[5], c->stream));  // re-recorded after the main kernel when it runs
  if (tm) HIPCHK(c, hipEventRecord(c->ev[6], c->stream));  // re-recorded after the long-row kernel
  HIPCHK(c, launch_schedule(c->sd, c->bd, o, pd, c->d_scratch, c->scratch_bytes, c->stream, tm ? c->ev[5] : nullptr,
                            tm ? c->ev[6] : nullptr, c->side, c->fork_ev, c->join_ev));
  if (tm) HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  if (p->replicas_plugin == KAD_PL_CLUSTER_CAPACITY_WEIGHT && !c->plan_rows.empty())
    HIPCHK(c, launch_plan(c->sd, c->bd, o, pd, static_cast<const PlanRowHdr*>(c->d_plan_hdr), (int)c->plan_rows.size(),
                          c->batch_hdr.max_row_slots, c->d_scratch, c->scratch_bytes, c->stream,
                          static_cast<int32_t*>(c->d_plan_big),
                          static_cast<int32_t*>(c->d_plan_big) + c->plan_rows.size()));
  if (tm) HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
  c->ran = true;
  c->timed = tm;
  return KAD_OK;
}

int kad_schedule(kad_ctx* c, const kad_profile* p) {
  return guarded(c, [&]() -> int {
    if (!c) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return schedule_locked(c, p, nullptr, nullptr);
  });
}

int kad_sync(kad_ctx* c) {
  if (!c) return KAD_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KAD_OK;
}

int kad_set_timing(kad_ctx* c, int on) {
  if (!c) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->timing = on != 0;
  return KAD_OK;
}

int kad_last_timing(kad_ctx* c, float ms[3]) {
  if (!c || !ms) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->ran) return fail(c, KAD_ESTATE, "nothing ran");
  if (!c->timed) return fail(c, KAD_ESTATE, "the last kad_schedule ran with timing off");
  HIPCHK(c, hipEventSynchronize(c->ev[2]));
  HIPCHK(c, hipEventElapsedTime(&ms[0], c->ev[0], c->ev[2]));
  HIPCHK(c, hipEventElapsedTime(&ms[1], c->ev[0], c->ev[1]));
  HIPCHK(c, hipEventElapsedTime(&ms[2], c->ev[1], c->ev[2]));
  return KAD_OK;
}

// the ctx's units' results into out; at_offsets (kad_group): into the whole batch's view, at the shard's
// unit and slot offsets
static int results_download_locked(kad_ctx* c, const kad_result_view* out, bool at_offsets = false) {
  if (!c->ran) return fail(c, KAD_ESTATE, "nothing ran");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t W = (size_t)c->unit_n, S = (size_t)c->slot_n;
  const size_t uo = at_offsets ? (size_t)c->unit_lo : 0, so = at_offsets ? (size_t)c->slot_lo : 0;
  if (W) {
    HIPCHK(c, hipMemcpyAsync(out->status + uo, c->d_status, W * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out->count + uo, c->d_count, W * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out->flags + uo, c->d_flags, W * 4, hipMemcpyDeviceToHost, c->stream));
  }
  if (S) {
    HIPCHK(c, hipMemcpyAsync(out->cluster + so, c->d_cluster, S * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out->replicas + so, c->d_replicas, S * 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KAD_OK;
}

int kad_stage_timing(kad_ctx* c, float* ms, int n) {
  if (!c || !ms || n < 0) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->ran) return fail(c, KAD_ESTATE, "nothing ran");
  if (!c->timed) return fail(c, KAD_ESTATE, "the last kad_schedule ran with timing off");
  HIPCHK(c, hipEventSynchronize(c->ev[2]));
  // req_mask, prep, main, defer (schedule_kernel over the defer list), planner, total, rows (schedule_row_kernel)
  const int pairs[7][2] = {{0, 3}, {3, 4}, {4, 5}, {6, 1}, {1, 2}, {0, 2}, {5, 6}};
  for (int i = 0; i < n && i < 7; i++) HIPCHK(c, hipEventElapsedTime(&ms[i], c->ev[pairs[i][0]], c->ev[pairs[i][1]]));
  return KAD_OK;
}

// device-to-device copy of the last results into caller device buffers (e.g. the send buffers of an
// RCCL all-gather of placements); ordered on the ctx stream and synchronised before return
int kad_results_copy_device(kad_ctx* c, const kad_result_view* dev_out) {
  if (!c || !dev_out) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->ran) return fail(c, KAD_ESTATE, "nothing ran");
  HIPCHK(c, hipSetDevice(c->device));
  // this ctx's units and slots (a kad_group member holds a shard: unit_n / slot_n of it, its own result
  // buffers from index 0)
  const size_t W = (size_t)c->unit_n;
  const size_t S = (size_t)c->slot_n;
  if (W) {
    HIPCHK(c, hipMemcpyAsync(dev_out->status, c->d_status, W * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(dev_out->count, c->d_count, W * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(dev_out->flags, c->d_flags, W * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  if (S) {
    HIPCHK(c, hipMemcpyAsync(dev_out->cluster, c->d_cluster, S * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(dev_out->replicas, c->d_replicas, S * 8, hipMemcpyDeviceToDevice, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KAD_OK;
}

int kad_host_alloc(size_t nbytes, void** out) {
  if (!out) return KAD_EINVAL;
  *out = nullptr;
  if (hipHostMalloc(out, nbytes ? nbytes : 1, hipHostMallocDefault) != hipSuccess) {
    *out = nullptr;
    return KAD_ENOMEM;
  }
  return KAD_OK;
}

int kad_host_free(void* p) {
  if (p && hipHostFree(p) != hipSuccess) return KAD_EHIP;
  return KAD_OK;
}

int kad_results_download(kad_ctx* c, const kad_result_view* out) {
  return guarded(c, [&]() -> int {
    if (!c || !out) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return results_download_locked(c, out);
  });
}

// One critical section from upload to download: worker goroutines sharing the
// ctx cannot interleave and schedule / download each other's batches.
int kad_schedule_batch(kad_ctx* c, const kad_profile* p, const void* blob, size_t nbytes, const kad_result_view* out) {
  return guarded(c, [&]() -> int {
    if (!c || !blob || !out) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (int r = batch_upload_locked(c, blob, nbytes)) return r;
    if (int r = schedule_locked(c, p, nullptr, nullptr)) return r;
    return results_download_locked(c, out);
  });
}

int kad_debug_phase_counters(uint64_t* out, int reset) { return kad::debug_phase_counters(out, reset); }

// ------------------------------------------------ §8 f3: result application diff

int kad_result_diff(kad_ctx* c, const kad_result_state* st, uint32_t* out) {
  return guarded(c, [&]() -> int {
    if (!c || !st || !out) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->ran || !c->have_batch) return fail(c, KAD_ESTATE, "no scheduled batch resident");
    // this ctx's units (a kad_group member: its shard, whose out_off keeps the batch-wide slot numbers that
    // out_dev's shifted slot arrays are indexed by)
    const int W = (int)c->unit_n, C = c->sd.C;
    if (st->n_units != W) return fail(c, KAD_EINVAL, "state n_units differs from the resident batch");
    if (W == 0) return KAD_OK;
    if (!st->place_off || !st->place_has || !st->ovr_off) return fail(c, KAD_EINVAL, "null state array");
    auto csr_ok = [&](const int32_t* off) {
      if (off[0] != 0) return false;
      for (int w = 0; w < W; w++)
        if (off[w + 1] < off[w]) return false;
      return true;
    };
    if (!csr_ok(st->place_off) || !csr_ok(st->ovr_off)) return fail(c, KAD_EINVAL, "state offsets not monotone from 0");
    const int64_t NP = st->place_off[W], NO = st->ovr_off[W];
    if ((NP && !st->place_cluster) || (NO && (!st->ovr_cluster || !st->ovr_value || !st->ovr_kind)))
      return fail(c, KAD_EINVAL, "null state array");
    for (int64_t i = 0; i < NP; i++)
      if (st->place_cluster[i] < -1 || st->place_cluster[i] >= C) return fail(c, KAD_EINVAL, "placement cluster out of range");
    for (int64_t i = 0; i < NO; i++)
      if (st->ovr_cluster[i] < -1 || st->ovr_cluster[i] >= C) return fail(c, KAD_EINVAL, "override cluster out of range");
    // canonical placements: sorted unique snapshot positions; names outside the snapshot → uflag bit 1
    std::vector<int32_t> cnt((size_t)W + 1, 0);
    std::vector<uint8_t> uflag((size_t)W);
    std::vector<int32_t> ids((size_t)NP);
    host_parallel(W, [&](int lo, int hi) {
      for (int w = lo; w < hi; w++) {
        int32_t* b = ids.data() + st->place_off[w];
        const int m = st->place_off[w + 1] - st->place_off[w];
        std::copy(st->place_cluster + st->place_off[w], st->place_cluster + st->place_off[w + 1], b);
        std::sort(b, b + m);
        const int u = (int)(std::unique(b, b + m) - b);
        const bool unknown = u > 0 && b[0] < 0;
        cnt[(size_t)w + 1] = unknown ? u - 1 : u;
        if (unknown) std::copy(b + 1, b + u, b);  // drop the -1
        uflag[w] = (uint8_t)((st->place_has[w] ? 1 : 0) | (unknown ? 2 : 0));
      }
    });
    std::vector<int32_t> pl_off((size_t)W + 1, 0);
    for (int w = 0; w < W; w++) pl_off[(size_t)w + 1] = pl_off[w] + cnt[(size_t)w + 1];
    std::vector<int32_t> pl_id((size_t)pl_off[W] + 1);
    host_parallel(W, [&](int lo, int hi) {
      for (int w = lo; w < hi; w++)
        std::copy(ids.data() + st->place_off[w], ids.data() + st->place_off[w] + cnt[(size_t)w + 1], pl_id.data() + pl_off[w]);
    });
    // one device buffer: [pl_off | pl_id | ov_off | ov_id | ov_val | uflag | ov_kind | out], 256-B aligned parts
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t b_ploff = 0, b_plid = al(b_ploff + 4 * ((size_t)W + 1)), b_ovoff = al(b_plid + 4 * pl_id.size()),
                 b_ovid = al(b_ovoff + 4 * ((size_t)W + 1)), b_ovval = al(b_ovid + 4 * (size_t)(NO + 1)),
                 b_uf = al(b_ovval + 8 * (size_t)(NO + 1)), b_ovk = al(b_uf + (size_t)W), b_out = al(b_ovk + (size_t)NO + 1),
                 total = al(b_out + 4 * (size_t)W);
    HIPCHK(c, hipSetDevice(c->device));
    if (int r = grow(c, &c->d_diff, &c->diff_cap, total)) return r;
    char* d = static_cast<char*>(c->d_diff);
    auto up = [&](size_t off, const void* h, size_t n) {
      return n ? hipMemcpyAsync(d + off, h, n, hipMemcpyHostToDevice, c->stream) : hipSuccess;
    };
    HIPCHK(c, up(b_ploff, pl_off.data(), 4 * ((size_t)W + 1)));
    HIPCHK(c, up(b_plid, pl_id.data(), 4 * (size_t)pl_off[W]));
    HIPCHK(c, up(b_ovoff, st->ovr_off, 4 * ((size_t)W + 1)));
    HIPCHK(c, up(b_ovid, st->ovr_cluster, 4 * (size_t)NO));
    HIPCHK(c, up(b_ovval, st->ovr_value, 8 * (size_t)NO));
    HIPCHK(c, up(b_uf, uflag.data(), (size_t)W));
    HIPCHK(c, up(b_ovk, st->ovr_kind, (size_t)NO));
    ResultDiffDev dd{};
    dd.W = W;
    dd.status = c->d_status;
    dd.count = c->d_count;
    const OutDev od = out_dev(c);
    dd.cluster = od.cluster;
    dd.replicas = od.replicas;
    dd.out_off = c->bd.out_off;
    dd.pl_off = reinterpret_cast<const int32_t*>(d + b_ploff);
    dd.pl_id = reinterpret_cast<const int32_t*>(d + b_plid);
    dd.uflag = reinterpret_cast<const uint8_t*>(d + b_uf);
    dd.ov_off = reinterpret_cast<const int32_t*>(d + b_ovoff);
    dd.ov_id = reinterpret_cast<const int32_t*>(d + b_ovid);
    dd.ov_val = reinterpret_cast<const int64_t*>(d + b_ovval);
    dd.ov_kind = reinterpret_cast<const uint8_t*>(d + b_ovk);
    dd.out = reinterpret_cast<uint32_t*>(d + b_out);
    HIPCHK(c, launch_result_diff(dd, c->stream));
    HIPCHK(c, hipMemcpyAsync(out, dd.out, 4 * (size_t)W, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // the caller's state arrays are free on return
    return KAD_OK;
  });
}

static int path_counts_locked(kad_ctx* c, int32_t* out);

int kad_path_counts(kad_ctx* c, int32_t* out) {
  if (!c || !out) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return path_counts_locked(c, out);
}

static int path_counts_locked(kad_ctx* c, int32_t* out) {
  if (!c->ran) return fail(c, KAD_ESTATE, "nothing ran");
  int32_t h[4] = {0, 0, 0, 0};
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemcpyAsync(h, c->d_defer, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  out[0] = (int32_t)c->unit_n;
  out[1] = h[0];  // defer_n: units the full kernel (schedule_kernel) took
  out[2] = c->bd.use_rows ? h[2] : 0;  // rows_n: units schedule_row_kernel took
  out[3] = (int32_t)c->plan_rows.size();  // Divide units handed to the planner
  return KAD_OK;
}

int kad_snapshot_paths(kad_ctx* c, int32_t* out) {
  return guarded(c, [&]() -> int {
    if (!c || !out) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->have_snapshot) return fail(c, KAD_ESTATE, "no snapshot");
    out[0] = c->clean_kind;
    out[1] = c->sd.clean;
    out[2] = wide_path(c->sd) ? 1 : 0;
    out[3] = c->sd.fold;
    out[4] = c->sd.fitfold;
    return KAD_OK;
  });
}

int kad_debug_inject_fault(kad_ctx* c, int where) {
  if (!c || where < 0 || where > 1) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->inject_fault = where;
  return KAD_OK;
}

int kad_debug_plan_force_workspace(kad_ctx* c, int on) {
  if (!c || on < 0 || on > 2) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->plan_force_ws = on;
  return KAD_OK;
}

int kad_debug_scores(kad_ctx* c, const kad_profile* p, uint8_t* feasible, int64_t* total) {
  return guarded(c, [&]() -> int {
    if (!c || !feasible || !total) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    const size_t n = (size_t)c->batch_hdr.n_units * c->sd.C;
    uint8_t* df = nullptr;
    int64_t* dt = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMalloc(&df, n ? n : 1));
    HIPCHK(c, hipMalloc(&dt, (n ? n : 1) * 8));
    HIPCHK(c, hipMemsetAsync(df, 0, n ? n : 1, c->stream));
    HIPCHK(c, hipMemsetAsync(dt, 0, (n ? n : 1) * 8, c->stream));
    int r = schedule_locked(c, p, df, dt);
    if (r == 0 && n) {
      HIPCHK(c, hipMemcpyAsync(feasible, df, n, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipMemcpyAsync(total, dt, n * 8, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    (void)hipFree(df);
    (void)hipFree(dt);
    return r;
  });
}


int kad_select_rows(kad_ctx* c, int n_rows, const int32_t* row_off, const int64_t* scores, const int64_t* maxc,
                    uint32_t pflags, int32_t* out_count, int32_t* out_sel, int32_t* out_status) {
  return guarded(c, [&]() -> int {
    if (!c || n_rows < 0) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    const size_t tot = row_off[n_rows];
    int kmax = 1;
    for (int r = 0; r < n_rows; r++) {
      const int k = row_off[r + 1] - row_off[r];
      if (k > 65535) return fail(c, KAD_EINVAL, "row longer than 65535");
      kmax = k > kmax ? k : kmax;
    }
    std::vector<void*> owned;
    int32_t *d_off, *d_cnt, *d_sel, *d_st;
    int64_t *d_sc, *d_mc;
    int r = 0;
    if ((r = to_dev(c, row_off, n_rows + 1, &d_off, owned)) || (r = to_dev(c, scores, tot, &d_sc, owned)) ||
        (r = to_dev(c, maxc, n_rows, &d_mc, owned)) || (r = to_dev<int32_t>(c, nullptr, n_rows, &d_cnt, owned)) ||
        (r = to_dev<int32_t>(c, nullptr, tot, &d_sel, owned)) || (r = to_dev<int32_t>(c, nullptr, n_rows, &d_st, owned))) {
      for (void* p : owned) (void)hipFree(p);
      return r;
    }
    void* scr = nullptr;
    size_t scr_bytes = 0;
    const size_t wb = select_wave_bytes(kmax);
    if (wb > 64 * 1024) {
      scr_bytes = wb * (size_t)(n_rows < 4096 ? n_rows : 4096);
      HIPCHK(c, hipMalloc(&scr, scr_bytes));
      owned.push_back(scr);
    }
    hipError_t e = launch_select_rows(n_rows, d_off, d_sc, d_mc, pflags, kmax, d_cnt, d_sel, d_st, scr, scr_bytes, c->stream);
    if (e == hipSuccess) {
      (void)hipMemcpyAsync(out_count, d_cnt, n_rows * 4, hipMemcpyDeviceToHost, c->stream);
      if (tot) (void)hipMemcpyAsync(out_sel, d_sel, tot * 4, hipMemcpyDeviceToHost, c->stream);
      (void)hipMemcpyAsync(out_status, d_st, n_rows * 4, hipMemcpyDeviceToHost, c->stream);
      e = hipStreamSynchronize(c->stream);
    }
    for (void* p : owned) (void)hipFree(p);
    if (e != hipSuccess) return fail(c, KAD_EHIP, hipGetErrorString(e));
    return KAD_OK;
  });
}

int kad_plan_rows(kad_ctx* c, int n_rows, const int32_t* row_off, const uint32_t* hash, const int64_t* weight,
                  const int64_t* min_r, const int64_t* max_r, const int64_t* cap, const int64_t* current,
                  const uint32_t* elem_flags, const int64_t* total, const uint32_t* row_flags, int64_t* out_plan,
                  int64_t* out_overflow) {
  return guarded(c, [&]() -> int {
    if (!c || n_rows < 0) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    const size_t tot = row_off[n_rows];
    int kmax = 1;
    for (int r = 0; r < n_rows; r++) {
      const int k = row_off[r + 1] - row_off[r];
      kmax = k > kmax ? k : kmax;
    }
    std::vector<void*> owned;
    PlanRowsDev R{};
    R.n_rows = n_rows;
    int32_t* d_off;
    uint32_t *d_hash, *d_ef, *d_rf;
    int64_t *d_w, *d_mn, *d_mx, *d_cap, *d_cur, *d_tot, *d_plan, *d_over;
    int r = 0;
    if ((r = to_dev(c, row_off, n_rows + 1, &d_off, owned)) || (r = to_dev(c, hash, tot, &d_hash, owned)) ||
        (r = to_dev(c, weight, tot, &d_w, owned)) || (r = to_dev(c, min_r, tot, &d_mn, owned)) ||
        (r = to_dev(c, max_r, tot, &d_mx, owned)) || (r = to_dev(c, cap, tot, &d_cap, owned)) ||
        (r = to_dev(c, current, tot, &d_cur, owned)) || (r = to_dev(c, elem_flags, tot, &d_ef, owned)) ||
        (r = to_dev(c, total, n_rows, &d_tot, owned)) || (r = to_dev(c, row_flags, n_rows, &d_rf, owned)) ||
        (r = to_dev<int64_t>(c, nullptr, tot, &d_plan, owned)) || (r = to_dev<int64_t>(c, nullptr, tot, &d_over, owned))) {
      for (void* p : owned) (void)hipFree(p);
      return r;
    }
    R.row_off = d_off;
    R.hash = d_hash;
    R.weight = d_w;
    R.min_r = d_mn;
    R.max_r = d_mx;
    R.cap = d_cap;
    R.current = d_cur;
    R.elem_flags = d_ef;
    R.total = d_tot;
    R.row_flags = d_rf;
    R.out_plan = d_plan;
    R.out_overflow = d_over;
    void* scr = nullptr;
    size_t scr_bytes = 0;
    const size_t wb = plan_wave_bytes(kmax);
    if (wb > 64 * 1024) {
      scr_bytes = wb * (size_t)(n_rows < 4096 ? n_rows : 4096);
      HIPCHK(c, hipMalloc(&scr, scr_bytes));
      owned.push_back(scr);
    }
    hipError_t e = launch_plan_rows(R, kmax, c->plan_force_ws, scr, scr_bytes, c->stream);
    if (e == hipSuccess) {
      if (tot) {
        (void)hipMemcpyAsync(out_plan, d_plan, tot * 8, hipMemcpyDeviceToHost, c->stream);
        (void)hipMemcpyAsync(out_overflow, d_over, tot * 8, hipMemcpyDeviceToHost, c->stream);
      }
      e = hipStreamSynchronize(c->stream);
    }
    for (void* p : owned) (void)hipFree(p);
    if (e != hipSuccess) return fail(c, KAD_EHIP, hipGetErrorString(e));
    return KAD_OK;
  });
}

/* ------------------------------------------------ scheduling-trigger hashes */
static int trigger_suffix_upload_locked(kad_ctx* c, const uint8_t* suffix, size_t nbytes) {
  HIPCHK(c, hipSetDevice(c->device));
  int r = grow(c, &c->t_suffix, &c->t_suffix_cap, ((nbytes + 63) & ~(size_t)63) + 64);
  if (r) return r;
  const int64_t ntab = trigger_table_count((int64_t)nbytes);
  r = grow(c, &c->t_tabs, &c->t_tabs_cap, (size_t)ntab * 256 * 4 + (size_t)ntab * 4 + 256);
  if (r) return r;
  if (nbytes) HIPCHK(c, hipMemcpyAsync(c->t_suffix, suffix, nbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  TriggerDev& t = c->td;
  t.suffix = static_cast<const uint32_t*>(c->t_suffix);
  t.suffix_len = (int64_t)nbytes;
  t.tables = static_cast<uint32_t*>(c->t_tabs);
  t.powers = t.tables + (size_t)ntab * 256;
  c->t_suffix_len = (int64_t)nbytes;
  c->t_ran = false;
  return KAD_OK;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static int trigger_prefixes_upload_locked(kad_ctx* c, int n, const int64_t* prefix_off, const uint8_t* prefix) {
  for (int i = 0; i < n; i++)
    if (prefix_off[i + 1] < prefix_off[i]) return fail(c, KAD_EINVAL, "prefix_off must be non-decreasing");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t nbytes = (size_t)prefix_off[n];
  int r = grow(c, &c->t_prefix, &c->t_prefix_cap, nbytes + 64);
  if (r) return r;
  const size_t nn = (size_t)(n > 0 ? n : 1);
  const size_t o_out = align256((nn + 1) * 8);
  r = grow(c, &c->t_work, &c->t_work_cap, o_out + align256(nn * 4));
  if (r) return r;
  char* w = static_cast<char*>(c->t_work);
  if (nbytes) HIPCHK(c, hipMemcpyAsync(c->t_prefix, prefix, nbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(w, prefix_off, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  TriggerDev& t = c->td;
  t.n = n;
  t.prefix = static_cast<const uint8_t*>(c->t_prefix);
  t.prefix_off = reinterpret_cast<const int64_t*>(w);
  t.out = reinterpret_cast<uint32_t*>(w + o_out);
  c->t_n = n;
  c->t_ran = false;
  return KAD_OK;
}

static int trigger_run_locked(kad_ctx* c) {
  if (c->t_suffix_len < 0 || c->t_n < 0) return fail(c, KAD_ESTATE, "upload the trigger suffix and prefixes first");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventRecord(c->tev[0], c->stream));
  HIPCHK(c, launch_trigger_summary(c->td, c->stream));
  HIPCHK(c, hipEventRecord(c->tev[1], c->stream));
  HIPCHK(c, launch_trigger_objects(c->td, c->stream));
  HIPCHK(c, hipEventRecord(c->tev[2], c->stream));
  c->t_ran = true;
  return KAD_OK;
}

int kad_trigger_timing(kad_ctx* c, float ms[2]) {
  if (!c || !ms) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->t_ran) return fail(c, KAD_ESTATE, "no trigger run");
  HIPCHK(c, hipEventSynchronize(c->tev[2]));
  HIPCHK(c, hipEventElapsedTime(&ms[0], c->tev[0], c->tev[2]));
  HIPCHK(c, hipEventElapsedTime(&ms[1], c->tev[0], c->tev[1]));
  return KAD_OK;
}

static int trigger_download_locked(kad_ctx* c, uint32_t* out_hash) {
  if (!c->t_ran) return fail(c, KAD_ESTATE, "no trigger run");
  HIPCHK(c, hipSetDevice(c->device));
  if (c->t_n > 0 && out_hash)
    HIPCHK(c, hipMemcpyAsync(out_hash, c->td.out, (size_t)c->t_n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return KAD_OK;
}

int kad_trigger_suffix_upload(kad_ctx* c, const uint8_t* suffix, size_t nbytes) {
  return guarded(c, [&]() -> int {
    if (!c || (!suffix && nbytes)) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return trigger_suffix_upload_locked(c, suffix, nbytes);
  });
}

int kad_trigger_prefixes_upload(kad_ctx* c, int n, const int64_t* prefix_off, const uint8_t* prefix) {
  return guarded(c, [&]() -> int {
    if (!c || n < 0 || !prefix_off || prefix_off[0] != 0) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return trigger_prefixes_upload_locked(c, n, prefix_off, prefix);
  });
}

int kad_trigger_run(kad_ctx* c) {
  if (!c) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return trigger_run_locked(c);
}

int kad_trigger_download(kad_ctx* c, uint32_t* out_hash) {
  if (!c) return KAD_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  return trigger_download_locked(c, out_hash);
}

// one critical section (see kad_schedule_batch)
int kad_trigger_hashes(kad_ctx* c, int n, const int64_t* prefix_off, const uint8_t* prefix, const uint8_t* suffix,
                       size_t suffix_len, uint32_t* out_hash) {
  return guarded(c, [&]() -> int {
    if (!c || (!suffix && suffix_len) || n < 0 || !prefix_off || prefix_off[0] != 0) return KAD_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    int r = trigger_suffix_upload_locked(c, suffix, suffix_len);
    if (!r) r = trigger_prefixes_upload_locked(c, n, prefix_off, prefix);
    if (!r) r = trigger_run_locked(c);
    if (!r) r = trigger_download_locked(c, out_hash);
    return r;
  });
}

}  // extern "C"

// ------------------------------------------------------------ multi-GPU group (kad_group_*)
// One process, N GPUs (the reference's single scheduler process with --worker-count goroutines,
// worker.go:132-134, calling Schedule at scheduler.go:507): units are independent given the read-only
// snapshot (scheduler.go:246-309), so the batch splits into contiguous unit ranges, one per member
// context, with no exchange while scheduling. Each member is a full kad_ctx on its device; a host pool
// with one thread per member issues every member's uploads / launches / copies concurrently.
struct kad_group {
  std::vector<kad_ctx*> m;
  kadpool::Pool* pool = nullptr;  // n - 1 workers + the calling thread: member i runs on thread i
  std::mutex mu;
  std::string err;
  std::vector<int64_t> unit_lo, slot_lo;  // [n + 1] the resident batch's split (kad_batch_split)
  bool have_batch = false, ran = false;
};

static int gfail(kad_group* g, int code, const std::string& msg) {
  if (g) g->err = msg;
  return code;
}

// f(i, member i) on every member concurrently; the first failure (lowest member) is the group's error
template <class F>
static int each_member(kad_group* g, F f) {
  const int n = (int)g->m.size();
  std::vector<int> rc((size_t)n, 0);
  try {
    g->pool->run(n, [&](int i) {
      kad_ctx* c = g->m[(size_t)i];
      rc[(size_t)i] = guarded(c, [&]() -> int {
        std::lock_guard<std::mutex> lk(c->mu);
        return f(i, c);
      });
    });
  } catch (const std::exception& e) {
    return gfail(g, KAD_EHOST, std::string("host error: ") + e.what());
  }
  for (int i = 0; i < n; i++)
    if (rc[(size_t)i]) return gfail(g, rc[(size_t)i], "member " + std::to_string(i) + ": " + g->m[(size_t)i]->err);
  return KAD_OK;
}

template <class F>
static int gguarded(kad_group* g, F f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return gfail(g, KAD_ENOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    return gfail(g, KAD_EHOST, std::string("host error: ") + e.what());
  } catch (...) {
    return gfail(g, KAD_EHOST, "host error: unknown exception");
  }
}

static void split_ranges(const int64_t* out_off, int64_t W, int n, int64_t* unit_lo, int64_t* slot_lo) {
  for (int i = 0; i <= n; i++) {
    unit_lo[i] = W * i / n;
    slot_lo[i] = out_off[unit_lo[i]];
  }
}

extern "C" {

int kad_batch_split(const void* blob, size_t nbytes, int n, int64_t* unit_lo, int64_t* slot_lo) {
  if (!blob || n < 1 || !unit_lo || !slot_lo || nbytes < sizeof(kad_batch_header)) return KAD_EINVAL;
  kad_batch_header h;
  std::memcpy(&h, blob, sizeof(h));
  if (h.magic != KAD_BATCH_MAGIC || h.abi_version != KAD_ABI_VERSION || h.total_bytes != nbytes || h.n_units < 0)
    return KAD_EINVAL;
  const uint64_t o = h.off[KAD_B_OUT_OFF], len = ((uint64_t)h.n_units + 1) * 8;
  if (o > nbytes || (o & 7) || len > nbytes - o) return KAD_EINVAL;
  const int64_t* oo = at<int64_t>(blob, h.off, KAD_B_OUT_OFF);
  for (int64_t w = 0; w < h.n_units; w++)
    if (oo[w + 1] < oo[w]) return KAD_EINVAL;
  split_ranges(oo, h.n_units, n, unit_lo, slot_lo);
  return KAD_OK;
}

int kad_group_create(const int* hip_devices, int n, kad_group** out) {
  if (!out || !hip_devices || n < 1 || n > 64) return KAD_EINVAL;
  *out = nullptr;
  auto* g = new (std::nothrow) kad_group();
  if (!g) return KAD_ENOMEM;
  for (int i = 0; i < n; i++) {
    kad_ctx* c = nullptr;
    if (int r = kad_ctx_create(hip_devices[i], &c)) {
      kad_group_destroy(g);
      return r;
    }
    g->m.push_back(c);
  }
  // direct peer access for the snapshot copies from member 0 (hipMemcpyPeerAsync works without it, staged)
  for (int i = 1; i < n; i++) {
    const int d = hip_devices[i], d0 = hip_devices[0];
    int can = 0;
    if (d != d0 && hipDeviceCanAccessPeer(&can, d, d0) == hipSuccess && can && hipSetDevice(d) == hipSuccess) {
      const hipError_t e = hipDeviceEnablePeerAccess(d0, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
    }
  }
  try {
    g->pool = new kadpool::Pool(n - 1);
  } catch (...) {
    kad_group_destroy(g);
    return KAD_EHOST;
  }
  *out = g;
  return KAD_OK;
}

int kad_group_destroy(kad_group* g) {
  if (!g) return KAD_OK;
  delete g->pool;  // joins its threads: nothing of the group runs after this
  for (kad_ctx* c : g->m) kad_ctx_destroy(c);
  delete g;
  return KAD_OK;
}

const char* kad_group_last_error(kad_group* g) { return g ? g->err.c_str() : "null group"; }

int kad_group_size(kad_group* g) { return g ? (int)g->m.size() : KAD_EINVAL; }

int kad_group_member(kad_group* g, int i, kad_ctx** out) {
  if (!g || !out || i < 0 || i >= (int)g->m.size()) return KAD_EINVAL;
  *out = g->m[(size_t)i];
  return KAD_OK;
}

int kad_group_snapshot_upload(kad_group* g, const void* blob, size_t nbytes) {
  return gguarded(g, [&]() -> int {
    if (!g || !blob) return KAD_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);
    g->have_batch = g->ran = false;
    for (kad_ctx* c : g->m) {  // a failure below must leave no member with a usable old state
      std::lock_guard<std::mutex> l2(c->mu);
      invalidate_snapshot(c);
    }
    kad_ctx* c0 = g->m[0];
    {
      std::lock_guard<std::mutex> l0(c0->mu);
      if (int r = guarded(c0, [&] { return snapshot_upload_locked(c0, blob, nbytes); }))
        return gfail(g, r, "member 0: " + c0->err);
    }
    return each_member(g, [&](int i, kad_ctx* c) { return i == 0 ? KAD_OK : snapshot_from_peer_locked(c, c0); });
  });
}

int kad_group_snapshot_update(kad_group* g, const void* delta, size_t nbytes) {
  return gguarded(g, [&]() -> int {
    if (!g || !delta) return KAD_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);
    const int r = each_member(g, [&](int, kad_ctx* c) { return snapshot_update_locked(c, delta, nbytes); });
    if (r) g->have_batch = g->ran = false;  // some member dropped its snapshot (and batch)
    return r;
  });
}

// the group's steps with g->mu held by the caller: kad_group_schedule_batch runs all three in one critical
// section (as kad_schedule_batch does for a ctx), so concurrent callers cannot interleave and download each
// other's batches
static int group_batch_upload_locked(kad_group* g, const void* blob, size_t nbytes) {
  g->have_batch = g->ran = false;
  const int n = (int)g->m.size();
  kad_ctx* c0 = g->m[0];
  kad_batch_header h;
  {
    // one validation of the whole blob (member 0's snapshot: every member holds the same one)
    std::lock_guard<std::mutex> l0(c0->mu);
    if (!c0->have_snapshot) return gfail(g, KAD_ESTATE, "no snapshot uploaded");
    if (nbytes < sizeof(h)) return gfail(g, KAD_EINVAL, "batch too small");
    std::memcpy(&h, blob, sizeof(h));
    if (h.magic != KAD_BATCH_MAGIC || h.abi_version != KAD_ABI_VERSION || h.total_bytes != nbytes)
      return gfail(g, KAD_EINVAL, "bad batch header");
    if (int r = guarded(c0, [&] { return validate_batch(c0, blob, nbytes, h); })) return gfail(g, r, c0->err);
  }
  g->unit_lo.assign((size_t)n + 1, 0);
  g->slot_lo.assign((size_t)n + 1, 0);
  split_ranges(at<int64_t>(blob, h.off, KAD_B_OUT_OFF), h.n_units, n, g->unit_lo.data(), g->slot_lo.data());
  if (int r = each_member(g, [&](int i, kad_ctx* c) {
        return batch_upload_locked(c, blob, nbytes, g->unit_lo[(size_t)i], g->unit_lo[(size_t)i + 1], true);
      }))
    return r;
  g->have_batch = true;
  return KAD_OK;
}

static int group_schedule_locked(kad_group* g, const kad_profile* p) {
  if (!g->have_batch) return gfail(g, KAD_ESTATE, "snapshot and batch must be uploaded first");
  if (int r = each_member(g, [&](int, kad_ctx* c) { return schedule_locked(c, p, nullptr, nullptr); })) return r;
  g->ran = true;
  return KAD_OK;
}

static int group_results_download_locked(kad_group* g, const kad_result_view* out) {
  if (!g->ran) return gfail(g, KAD_ESTATE, "nothing ran");
  return each_member(g, [&](int, kad_ctx* c) { return results_download_locked(c, out, true); });
}

int kad_group_batch_upload(kad_group* g, const void* blob, size_t nbytes) {
  return gguarded(g, [&]() -> int {
    if (!g || !blob) return KAD_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);
    return group_batch_upload_locked(g, blob, nbytes);
  });
}

int kad_group_schedule(kad_group* g, const kad_profile* p) {
  return gguarded(g, [&]() -> int {
    if (!g) return KAD_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);
    return group_schedule_locked(g, p);
  });
}

int kad_group_sync(kad_group* g) {
  return gguarded(g, [&]() -> int {
    if (!g) return KAD_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);
    return each_member(g, [&](int, kad_ctx* c) -> int {
      HIPCHK(c, hipSetDevice(c->device));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      return KAD_OK;
    });
  });
}

int kad_group_results_download(kad_group* g, const kad_result_view* out) {
  return gguarded(g, [&]() -> int {
    if (!g || !out) return KAD_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);
    return group_results_download_locked(g, out);
  });
}

// one critical section from upload to download (kad_schedule_batch's contract, per group)
int kad_group_schedule_batch(kad_group* g, const kad_profile* p, const void* blob, size_t nbytes,
                             const kad_result_view* out) {
  return gguarded(g, [&]() -> int {
    if (!g || !p || !blob || !out) return KAD_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);
    if (int r = group_batch_upload_locked(g, blob, nbytes)) return r;
    if (int r = group_schedule_locked(g, p)) return r;
    return group_results_download_locked(g, out);
  });
}

int kad_group_ranges(kad_group* g, int64_t* unit_lo, int64_t* slot_lo) {
  if (!g || !unit_lo || !slot_lo) return KAD_EINVAL;
  std::lock_guard<std::mutex> lk(g->mu);
  if (!g->have_batch) return gfail(g, KAD_ESTATE, "no batch uploaded");
  std::copy(g->unit_lo.begin(), g->unit_lo.end(), unit_lo);
  std::copy(g->slot_lo.begin(), g->slot_lo.end(), slot_lo);
  return KAD_OK;
}

int kad_group_path_counts(kad_group* g, int32_t* out) {
  return gguarded(g, [&]() -> int {
    if (!g || !out) return KAD_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->ran) return gfail(g, KAD_ESTATE, "nothing ran");
    std::vector<int32_t> per(4 * g->m.size(), 0);
    if (int r = each_member(g, [&](int i, kad_ctx* c) { return path_counts_locked(c, per.data() + 4 * (size_t)i); }))
      return r;
    for (int k = 0; k < 4; k++) {
      out[k] = 0;
      for (size_t i = 0; i < g->m.size(); i++) out[k] += per[4 * i + (size_t)k];
    }
    return KAD_OK;
  });
}

int kad_group_set_timing(kad_group* g, int on) {
  if (!g) return KAD_EINVAL;
  for (kad_ctx* c : g->m) kad_set_timing(c, on);
  return KAD_OK;
}

}  // extern "C"

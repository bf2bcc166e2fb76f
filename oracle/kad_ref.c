/*
 * kad_ref.c — C restatement of KubeAdmiral's genericScheduler.Schedule over the
 * packed snapshot / batch blobs of include/kad_sched.h.
 *
 * ORACLE HEADER — TEST INFRASTRUCTURE ONLY. This is the parity checker for the
 * HIP path at sizes the Python oracle cannot reach, and the timed CPU baseline
 * ("port") of bench.py. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it. It is written in the reference's structure: one
 * SchedulingUnit at a time (like one reconcile on a --worker-count goroutine,
 * pkg/controllers/util/worker/worker.go:132-134), clusters × filter plugins
 * with short-circuit, then score plugins × feasible clusters with
 * DefaultNormalizeScore, then Go 1.19 sort.Slice (pdqsort) in MaxCluster, then
 * ClusterCapacityWeight + planner.Plan with sort.Sort.
 *
 * It shares only the blob layout with the product; the host-side object →
 * blob packing it relies on is checked against the object-level Python oracle
 * (oracle/kad_oracle.py, pinned by tests/golden/) in tests/test_c_oracle.py.
 *
 * Deterministic rules where the reference is not:
 * AvailableToPercentage's remainder goes to the tied maximum with the lowest
 * snapshot index; planner preferences enter sort.Sort in ascending snapshot
 * index (Go: random map order; identical unless (weight, FNV) collide).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/kad_sched.h"

typedef struct {
  int C, GW, TW, K, S;
  const int64_t *alloc_cpu, *alloc_mem, *used_cpu, *used_mem, *alloc_s, *used_s, *alloc_cores, *avail_cores;
  const uint64_t *gvk, *nsne, *ne, *pns;
  const int32_t* lval;
  const int64_t* lint;
  const uint8_t* lok;
  const uint32_t* name_fnv;
} snap_t;

typedef struct {
  int W, NT, TW;
  const uint32_t* flags;
  const int32_t *gvk, *tolset;
  const int64_t *req_cpu, *req_mem, *desired, *maxc;
  const uint64_t *tol_all, *tol_pns;
  const int32_t *sreq_off, *sreq_id;
  const int64_t* sreq_val;
  const int32_t *fprog_off, *fprog, *sprog_off, *sprog, *place_off, *place, *cur_off, *cur_id;
  const int64_t* cur_rep;
  const int32_t *pref_off, *pref_id;
  const void *pref_w, *pref_min, *pref_max, *pref_cap; /* i64[], or i32[] with KAD_BATCH_NARROW_PREFS */
  int pref_narrow;
  const uint32_t* pref_fl;
  const int32_t* key_off;
  const uint8_t* key;
  const int64_t* out_off;
  const int32_t *req_off, *req;
} batch_t;

#define PTR(base, hdr, i) ((const void*)((const uint8_t*)(base) + (hdr)->off[i]))

static int parse_snap(const void* blob, snap_t* s) {
  const kad_snapshot_header* h = (const kad_snapshot_header*)blob;
  if (h->magic != KAD_SNAPSHOT_MAGIC) return -1;
  s->C = h->n_clusters; s->GW = h->n_gvk_words; s->TW = h->n_taint_words; s->K = h->n_label_keys; s->S = h->n_scalar;
  s->alloc_cpu = PTR(blob, h, KAD_S_ALLOC_CPU); s->alloc_mem = PTR(blob, h, KAD_S_ALLOC_MEM);
  s->used_cpu = PTR(blob, h, KAD_S_USED_CPU); s->used_mem = PTR(blob, h, KAD_S_USED_MEM);
  s->alloc_s = PTR(blob, h, KAD_S_ALLOC_SCALAR); s->used_s = PTR(blob, h, KAD_S_USED_SCALAR);
  s->alloc_cores = PTR(blob, h, KAD_S_ALLOC_CORES); s->avail_cores = PTR(blob, h, KAD_S_AVAIL_CORES);
  s->gvk = PTR(blob, h, KAD_S_GVK); s->nsne = PTR(blob, h, KAD_S_TAINT_NSNE); s->ne = PTR(blob, h, KAD_S_TAINT_NE);
  s->pns = PTR(blob, h, KAD_S_TAINT_PNS); s->lval = PTR(blob, h, KAD_S_LABEL_VAL); s->lint = PTR(blob, h, KAD_S_LABEL_INT);
  s->lok = PTR(blob, h, KAD_S_LABEL_INT_OK); s->name_fnv = PTR(blob, h, KAD_S_NAME_FNV);
  return 0;
}

/* preference column q's entry k in the batch's width */
static inline int64_t pref_val(const batch_t* b, const void* col, int k) {
  return b->pref_narrow ? (int64_t)((const int32_t*)col)[k] : ((const int64_t*)col)[k];
}

static int parse_batch(const void* blob, batch_t* b) {
  const kad_batch_header* h = (const kad_batch_header*)blob;
  if (h->magic != KAD_BATCH_MAGIC) return -1;
  b->W = h->n_units; b->NT = h->n_tolsets; b->TW = h->n_taint_words;
  b->flags = PTR(blob, h, KAD_B_FLAGS); b->gvk = PTR(blob, h, KAD_B_GVK);
  b->req_cpu = PTR(blob, h, KAD_B_REQ_CPU); b->req_mem = PTR(blob, h, KAD_B_REQ_MEM);
  b->desired = PTR(blob, h, KAD_B_DESIRED); b->maxc = PTR(blob, h, KAD_B_MAX_CLUSTERS);
  b->tolset = PTR(blob, h, KAD_B_TOLSET); b->tol_all = PTR(blob, h, KAD_B_TOL_ALL); b->tol_pns = PTR(blob, h, KAD_B_TOL_PNS);
  b->sreq_off = PTR(blob, h, KAD_B_SREQ_OFF); b->sreq_id = PTR(blob, h, KAD_B_SREQ_ID); b->sreq_val = PTR(blob, h, KAD_B_SREQ_VAL);
  b->fprog_off = PTR(blob, h, KAD_B_FPROG_OFF); b->fprog = PTR(blob, h, KAD_B_FPROG);
  b->sprog_off = PTR(blob, h, KAD_B_SPROG_OFF); b->sprog = PTR(blob, h, KAD_B_SPROG);
  b->place_off = PTR(blob, h, KAD_B_PLACE_OFF); b->place = PTR(blob, h, KAD_B_PLACE);
  b->cur_off = PTR(blob, h, KAD_B_CUR_OFF); b->cur_id = PTR(blob, h, KAD_B_CUR_ID); b->cur_rep = PTR(blob, h, KAD_B_CUR_REP);
  b->pref_off = PTR(blob, h, KAD_B_PREF_OFF); b->pref_id = PTR(blob, h, KAD_B_PREF_ID);
  b->pref_w = PTR(blob, h, KAD_B_PREF_W); b->pref_min = PTR(blob, h, KAD_B_PREF_MIN);
  b->pref_max = PTR(blob, h, KAD_B_PREF_MAX); b->pref_cap = PTR(blob, h, KAD_B_PREF_CAP);
  b->pref_fl = PTR(blob, h, KAD_B_PREF_FLAGS);
  b->pref_narrow = (h->flags & KAD_BATCH_NARROW_PREFS) != 0;
  b->key_off = PTR(blob, h, KAD_B_KEY_OFF); b->key = PTR(blob, h, KAD_B_KEY); b->out_off = PTR(blob, h, KAD_B_OUT_OFF);
  b->req_off = PTR(blob, h, KAD_B_REQ_OFF); b->req = PTR(blob, h, KAD_B_REQ);
  return 0;
}

/* ------------------------------------------------------------ Go semantics */
static inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static inline int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
static inline int64_t gdiv(int64_t a, int64_t b) { /* Go: truncation; MinInt64/-1 wraps */
  if (b == -1) return (int64_t)(0 - (uint64_t)a);
  return a / b;
}
static inline int64_t go_f2i(double x) { /* amd64 CVTTSD2SQ */
  if (isnan(x) || x >= 9223372036854775808.0 || x < -9223372036854775808.0) return INT64_MIN;
  return (int64_t)x;
}
static inline double go_round(double x) { return round(x); } /* half away from zero, same as math.Round */
static inline uint32_t fnv_cont(uint32_t h, const uint8_t* p, int n) {
  for (int i = 0; i < n; i++) { h *= 16777619u; h ^= p[i]; }
  return h;
}

/* ---------------------------------------------------------- Go 1.19 pdqsort */
typedef struct {
  int (*less)(void* ctx, int i, int j);
  void (*swap)(void* ctx, int i, int j);
  void* ctx;
  int xs_b, xs_c; /* xorshift triple (13, xs_b, xs_c) */
} gosort_t;

#define LESS(i, j) (d->less(d->ctx, (i), (j)))
#define SWAP(i, j) (d->swap(d->ctx, (i), (j)))

static int bits_len(unsigned long long x) { int n = 0; while (x) { n++; x >>= 1; } return n; }

static void insertion_sort(gosort_t* d, int a, int b) {
  for (int i = a + 1; i < b; i++)
    for (int j = i; j > a && LESS(j, j - 1); j--) SWAP(j, j - 1);
}
static void sift_down(gosort_t* d, int lo, int hi, int first) {
  int root = lo;
  for (;;) {
    int child = 2 * root + 1;
    if (child >= hi) return;
    if (child + 1 < hi && LESS(first + child, first + child + 1)) child++;
    if (!LESS(first + root, first + child)) return;
    SWAP(first + root, first + child);
    root = child;
  }
}
static void heap_sort(gosort_t* d, int a, int b) {
  int first = a, lo = 0, hi = b - a;
  for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(d, i, hi, first);
  for (int i = hi - 1; i >= 0; i--) { SWAP(first, first + i); sift_down(d, lo, i, first); }
}
static int partial_insertion_sort(gosort_t* d, int a, int b) {
  const int maxSteps = 5, shortestShifting = 50;
  int i = a + 1;
  for (int j = 0; j < maxSteps; j++) {
    while (i < b && !LESS(i, i - 1)) i++;
    if (i == b) return 1;
    if (b - a < shortestShifting) return 0;
    SWAP(i, i - 1);
    if (i - a >= 2) {
      for (int k = i - 1; k >= 1; k--) { /* sic: Go's bound is 1 */
        if (!LESS(k, k - 1)) break;
        SWAP(k, k - 1);
      }
    }
    if (b - i >= 2) {
      for (int k = i + 1; k < b; k++) {
        if (!LESS(k, k - 1)) break;
        SWAP(k, k - 1);
      }
    }
  }
  return 0;
}
static void break_patterns(gosort_t* d, int a, int b) {
  int length = b - a;
  if (length >= 8) {
    uint64_t r = (uint64_t)length;
    unsigned long long modulus = 1ull << bits_len((unsigned long long)length);
    int idx = a + (length / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
      r ^= r << 13; r ^= r >> d->xs_b; r ^= r << d->xs_c;
      int other = (int)((unsigned long long)r & (modulus - 1));
      if (other >= length) other -= length;
      SWAP(idx - 1 + i, a + other);
    }
  }
}
static void order2(gosort_t* d, int* a, int* b, int* swaps) {
  if (LESS(*b, *a)) { int t = *a; *a = *b; *b = t; (*swaps)++; }
}
static int median(gosort_t* d, int a, int b, int c, int* swaps) {
  order2(d, &a, &b, swaps); order2(d, &b, &c, swaps); order2(d, &a, &b, swaps);
  return b;
}
static int choose_pivot(gosort_t* d, int a, int b, int* hint) {
  int l = b - a, swaps = 0;
  int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
  if (l >= 8) {
    if (l >= 50) {
      i = median(d, i - 1, i, i + 1, &swaps);
      j = median(d, j - 1, j, j + 1, &swaps);
      k = median(d, k - 1, k, k + 1, &swaps);
    }
    j = median(d, i, j, k, &swaps);
  }
  *hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
  return j;
}
static void reverse_range(gosort_t* d, int a, int b) {
  for (int i = a, j = b - 1; i < j; i++, j--) SWAP(i, j);
}
static int partition_equal(gosort_t* d, int a, int b, int pivot) {
  SWAP(a, pivot);
  int i = a + 1, j = b - 1;
  for (;;) {
    while (i <= j && !LESS(a, i)) i++;
    while (i <= j && LESS(a, j)) j--;
    if (i > j) break;
    SWAP(i, j); i++; j--;
  }
  return i;
}
static int partition(gosort_t* d, int a, int b, int pivot, int* already) {
  SWAP(a, pivot);
  int i = a + 1, j = b - 1;
  while (i <= j && LESS(i, a)) i++;
  while (i <= j && !LESS(j, a)) j--;
  if (i > j) { SWAP(j, a); *already = 1; return j; }
  SWAP(i, j); i++; j--;
  for (;;) {
    while (i <= j && LESS(i, a)) i++;
    while (i <= j && !LESS(j, a)) j--;
    if (i > j) break;
    SWAP(i, j); i++; j--;
  }
  SWAP(j, a);
  *already = 0;
  return j;
}
static void pdqsort(gosort_t* d, int a, int b, int limit) {
  int wasBalanced = 1, wasPartitioned = 1;
  for (;;) {
    int length = b - a;
    if (length <= 12) { insertion_sort(d, a, b); return; }
    if (limit == 0) { heap_sort(d, a, b); return; }
    if (!wasBalanced) { break_patterns(d, a, b); limit--; }
    int hint;
    int pivot = choose_pivot(d, a, b, &hint);
    if (hint == 2) { reverse_range(d, a, b); pivot = (b - 1) - (pivot - a); hint = 1; }
    if (wasBalanced && wasPartitioned && hint == 1) {
      if (partial_insertion_sort(d, a, b)) return;
    }
    if (a > 0 && !LESS(a - 1, pivot)) { a = partition_equal(d, a, b, pivot); continue; }
    int already;
    int mid = partition(d, a, b, pivot, &already);
    wasPartitioned = already;
    int leftLen = mid - a, rightLen = b - mid, balanceThreshold = length / 8;
    if (leftLen < rightLen) {
      wasBalanced = leftLen >= balanceThreshold;
      pdqsort(d, a, mid, limit);
      a = mid + 1;
    } else {
      wasBalanced = rightLen >= balanceThreshold;
      pdqsort(d, mid + 1, b, limit);
      b = mid;
    }
  }
}
static void go_sort(gosort_t* d, int n) { pdqsort(d, 0, n, bits_len((unsigned long long)n)); }

/* --------------------------------------------------- predicate programs */
/* labels.Requirement.Matches / fields one-term selectors on cluster c for the
 * interned requirement `id` (apimachinery v0.26.6). */
static int eval_req(const snap_t* s, const batch_t* b, int id, int c) {
  const int32_t* p = b->req + b->req_off[id];
  int op = p[0] & 0xff, n = p[0] >> 8, key = p[1];
  switch (op) {
    case KAD_OP_TRUE: return 1;
    case KAD_OP_FALSE: return 0;
    case KAD_OP_NAME_EQ: return c == key;
    case KAD_OP_NAME_NE: return c != key;
    default: break;
  }
  int32_t v = s->lval[(size_t)key * s->C + c];
  switch (op) {
    case KAD_OP_EXISTS: return v >= 0;
    case KAD_OP_DNE: return v < 0;
    case KAD_OP_EQ:
    case KAD_OP_IN:
      if (v < 0) return 0;
      for (int i = 0; i < n; i++) if (p[2 + i] == v) return 1;
      return 0;
    case KAD_OP_NOTIN:
      if (v < 0) return 1;
      for (int i = 0; i < n; i++) if (p[2 + i] == v) return 0;
      return 1;
    case KAD_OP_GT:
    case KAD_OP_LT: {
      if (v < 0 || !s->lok[(size_t)key * s->C + c]) return 0;
      int64_t thr = (int64_t)(((uint64_t)(uint32_t)p[3] << 32) | (uint32_t)p[2]);
      int64_t lv = s->lint[(size_t)key * s->C + c];
      return op == KAD_OP_GT ? lv > thr : lv < thr;
    }
  }
  return 0;
}

/* clusterselector.MatchClusterSelectorTerms + ClusterAffinity.Filter (cluster_affinity.go:50-94) */
static int filter_affinity(const snap_t* s, const batch_t* b, const int32_t* p, int c) {
  int pc = 0;
  int n_sel = p[pc++];
  for (int i = 0; i < n_sel; i++)
    if (!eval_req(s, b, p[pc + i], c)) return 0; /* SelectorFromSet: every (k, v) must match */
  pc += n_sel;
  int present = p[pc++];
  if (!present) return 1;
  int n_terms = p[pc++];
  for (int t = 0; t < n_terms; t++) {
    int tf = p[pc], ne = p[pc + 1], nf = p[pc + 2];
    const int32_t* ids = p + pc + 3;
    pc += 3 + ne + nf;
    if (!(tf & KAD_TERM_HAS_EXPR) && !(tf & KAD_TERM_HAS_FIELD)) continue;
    if (tf & KAD_TERM_HAS_EXPR) {
      if (!(tf & KAD_TERM_EXPR_VALID)) return 0; /* error ⇒ false */
      int m = 1;
      for (int i = 0; i < ne && m; i++) m = eval_req(s, b, ids[i], c);
      if (!m) continue;
    }
    if (tf & KAD_TERM_HAS_FIELD) {
      if (!(tf & KAD_TERM_FIELD_VALID)) return 0;
      int m = 1;
      for (int i = 0; i < nf && m; i++) m = eval_req(s, b, ids[ne + i], c);
      if (!m) continue;
    }
    return 1;
  }
  return 0;
}

static int64_t score_affinity(const snap_t* s, const batch_t* b, const int32_t* p, int c) {
  int pc = 0;
  int n_terms = p[pc++];
  int64_t score = 0;
  for (int t = 0; t < n_terms; t++) {
    int32_t w = p[pc], ne = p[pc + 1];
    const int32_t* ids = p + pc + 2;
    pc += 2 + ne;
    int m = 1;
    for (int i = 0; i < ne && m; i++) m = eval_req(s, b, ids[i], c);
    if (m) score = wadd(score, w);
  }
  return score;
}

/* -------------------------------------------------------------- filters */
static int has_current(const batch_t* b, int w, int c) {
  for (int i = b->cur_off[w]; i < b->cur_off[w + 1]; i++) if (b->cur_id[i] == c) return 1;
  return 0;
}

static int run_filter(const snap_t* s, const batch_t* b, int w, int c, int plugin) {
  uint32_t f = b->flags[w];
  switch (plugin) {
    case KAD_PL_API_RESOURCES: { /* apiresources.go:25-43 */
      int g = b->gvk[w];
      if (g < 0) return 0;
      return (int)((s->gvk[(size_t)(g / 64) * s->C + c] >> (g % 64)) & 1);
    }
    case KAD_PL_TAINT_TOLERATION: { /* taint_toleration.go:44-89 */
      int scheduled = (f & KAD_W_HAS_CURRENT) && has_current(b, w, c);
      const uint64_t* tol = b->tol_all + (size_t)b->tolset[w] * b->TW;
      for (int i = 0; i < s->TW; i++) {
        uint64_t m = scheduled ? s->ne[(size_t)i * s->C + c] : s->nsne[(size_t)i * s->C + c];
        if (m & ~tol[i]) return 0;
      }
      return 1;
    }
    case KAD_PL_CLUSTER_RESOURCES_FIT: { /* fit.go:73-134 */
      if (!(f & KAD_W_FIT_NONZERO)) return 1;
      int ok = 1;
      if (s->alloc_cpu[c] < wadd(b->req_cpu[w], s->used_cpu[c])) ok = 0;
      if (s->alloc_mem[c] < wadd(b->req_mem[w], s->used_mem[c])) ok = 0;
      for (int i = b->sreq_off[w]; i < b->sreq_off[w + 1]; i++) {
        int sid = b->sreq_id[i];
        int64_t a = sid >= 0 ? s->alloc_s[(size_t)sid * s->C + c] : 0;
        int64_t u = sid >= 0 ? s->used_s[(size_t)sid * s->C + c] : 0;
        if (a < wadd(b->sreq_val[i], u)) ok = 0;
      }
      return ok;
    }
    case KAD_PL_PLACEMENT_FILTER: { /* placement/filter.go:37-57 */
      if (!(f & KAD_W_HAS_PLACEMENT)) return 1;
      for (int i = b->place_off[w]; i < b->place_off[w + 1]; i++) if (b->place[i] == c) return 1;
      return 0;
    }
    case KAD_PL_CLUSTER_AFFINITY:
      return filter_affinity(s, b, b->fprog + b->fprog_off[w], c);
  }
  return 1;
}

/* --------------------------------------------------------------- scores */
static int64_t least_requested(int64_t req, int64_t cap) { /* least_allocated.go:88-94 */
  if (cap == 0 || req > cap) return 0;
  return gdiv(wmul(wsub(cap, req), 100), cap);
}
static int64_t most_requested(int64_t req, int64_t cap) { /* most_allocated.go:90-97 */
  if (cap == 0 || req > cap) return 0;
  return gdiv(wmul(req, 100), cap);
}
static double fraction(int64_t req, int64_t cap) { return cap == 0 ? 1.0 : (double)req / (double)cap; }

static int64_t run_score(const snap_t* s, const batch_t* b, int w, int c, int plugin) {
  int64_t rc = wadd(s->used_cpu[c], b->req_cpu[w]), rm = wadd(s->used_mem[c], b->req_mem[w]);
  int64_t cc = s->alloc_cpu[c], cm = s->alloc_mem[c];
  switch (plugin) {
    case KAD_PL_TAINT_TOLERATION: { /* taint_toleration.go:91-113, 145-159 */
      const uint64_t* tol = b->tol_pns + (size_t)b->tolset[w] * b->TW;
      int64_t n = 0;
      for (int i = 0; i < s->TW; i++) n += __builtin_popcountll(s->pns[(size_t)i * s->C + c] & ~tol[i]);
      return n;
    }
    case KAD_PL_LEAST_ALLOCATED:
      return gdiv(wadd(least_requested(rm, cm), least_requested(rc, cc)), 2);
    case KAD_PL_MOST_ALLOCATED:
      return gdiv(wadd(most_requested(rm, cm), most_requested(rc, cc)), 2);
    case KAD_PL_BALANCED_ALLOCATION: { /* balanced_allocation.go:45-76 */
      double cf = fraction(rc, cc), mf = fraction(rm, cm);
      if (cf >= 1 || mf >= 1) return 0;
      double diff = fabs(cf - mf);
      volatile double one_minus = 1 - diff; /* no contraction */
      return go_f2i(one_minus * 100.0);
    }
    case KAD_PL_CLUSTER_AFFINITY:
      return score_affinity(s, b, b->sprog + b->sprog_off[w], c);
  }
  return 0;
}

static void default_normalize(int64_t maxp, int reverse, int64_t* sc, int n) { /* framework/util.go:455-483 */
  int64_t mx = 0;
  for (int i = 0; i < n; i++) if (sc[i] > mx) mx = sc[i];
  if (mx == 0) {
    if (reverse) for (int i = 0; i < n; i++) sc[i] = maxp;
    return;
  }
  for (int i = 0; i < n; i++) {
    int64_t v = gdiv(wmul(maxp, sc[i]), mx);
    if (reverse) v = maxp - v;
    sc[i] = v;
  }
}

/* ---------------------------------------------------------- MaxCluster */
typedef struct { int32_t cid; int64_t score; } cscore_t;
static int cs_less(void* ctx, int i, int j) { cscore_t* a = ctx; return a[i].score > a[j].score; }
static void cs_swap(void* ctx, int i, int j) { cscore_t* a = ctx; cscore_t t = a[i]; a[i] = a[j]; a[j] = t; }

/* -------------------------------------------------------------- planner */
typedef struct {
  int32_t cid;
  uint32_t hash;
  int64_t weight, min, max;
  int has_max;
} npref_t;
static int np_less(void* ctx, int i, int j) { /* planner.go:64-66 */
  npref_t* a = ctx;
  return a[i].weight > a[j].weight || (a[i].weight == a[j].weight && a[i].hash < a[j].hash);
}
static void np_swap(void* ctx, int i, int j) { npref_t* a = ctx; npref_t t = a[i]; a[i] = a[j]; a[j] = t; }

/* per-row scratch indexed by position in the selected list */
typedef struct {
  int n;
  int32_t cid[1]; /* flexible */
} dummy_t;

static int pos_of(const int32_t* cids, int n, int32_t cid) {
  for (int i = 0; i < n; i++) if (cids[i] == cid) return i;
  return -1;
}

/* getDesiredPlan (planner.go:211-304). prefs sorted; plan/overflow indexed by
 * position in `cids` (the selected list); cap: has_cap/capv by position.    */
static void get_desired_plan(npref_t* prefs, int np, const int32_t* cids, int n, const int* has_cap,
                             const int64_t* capv, int64_t total, int keep, int64_t* plan, int64_t* overflow,
                             int* has_plan, int* has_over, int64_t* remaining_out, npref_t* tmp) {
  int64_t remaining = total;
  for (int i = 0; i < np; i++) {
    int p = pos_of(cids, n, prefs[i].cid);
    int64_t mn = prefs[i].min < remaining ? prefs[i].min : remaining;
    if (has_cap && has_cap[p] && capv[p] < mn) {
      overflow[p] = mn - capv[p]; has_over[p] = 1;
      mn = capv[p];
    }
    remaining = wsub(remaining, mn);
    plan[p] = mn; has_plan[p] = 1;
  }
  int modified = 1;
  while (modified && remaining > 0) {
    modified = 0;
    int64_t wsum = 0;
    for (int i = 0; i < np; i++) wsum = wadd(wsum, prefs[i].weight);
    if (wsum <= 0) break;
    int nn = 0;
    int64_t distribute = remaining;
    for (int i = 0; i < np; i++) {
      int p = pos_of(cids, n, prefs[i].cid);
      int64_t start = plan[p];
      int64_t extra = gdiv(wsub(wadd(wmul(distribute, prefs[i].weight), wsum), 1), wsum);
      if (remaining < extra) extra = remaining;
      int64_t tot = wadd(start, extra);
      int full = 0;
      if (prefs[i].has_max && tot > prefs[i].max) { tot = prefs[i].max; full = 1; }
      if (has_cap && has_cap[p] && tot > capv[p]) {
        overflow[p] = wadd(has_over[p] ? overflow[p] : 0, tot - capv[p]); has_over[p] = 1;
        tot = capv[p]; full = 1;
      }
      if (!full) tmp[nn++] = prefs[i];
      remaining = wsub(remaining, wsub(tot, start));
      plan[p] = tot;
      if (tot > start) modified = 1;
    }
    memcpy(prefs, tmp, sizeof(npref_t) * nn);
    np = nn;
  }
  if (!keep) {
    for (int p = 0; p < n; p++) {
      if (!has_over[p]) continue;
      int64_t v = overflow[p] < remaining ? overflow[p] : remaining;
      if (v > 0) overflow[p] = v; else has_over[p] = 0;
    }
  }
  *remaining_out = remaining;
}

typedef struct {
  int xs_b, xs_c;
} sortcfg_t;

/* ClusterCapacityWeight.ReplicaScheduling (rsp.go:65-181) over the selected
 * clusters `cids` (n). Writes (cid, replicas>0) pairs sorted by cid.        */
static int replica_scheduling(const snap_t* s, const batch_t* b, int w, const int32_t* sel, int n, int32_t* out_c,
                              int64_t* out_r, uint32_t* rflags, sortcfg_t sc) {
  uint32_t f = b->flags[w];
  int32_t* cids = malloc(sizeof(int32_t) * (n + 1));
  for (int i = 0; i < n; i++) cids[i] = sel[i];
  /* ascending snapshot order (input order of the Go maps is random) */
  for (int i = 1; i < n; i++) { int32_t x = cids[i]; int j = i - 1; while (j >= 0 && cids[j] > x) { cids[j + 1] = cids[j]; j--; } cids[j + 1] = x; }
  int64_t *weight = calloc(n + 1, 8), *minr = calloc(n + 1, 8), *maxr = calloc(n + 1, 8), *capv = calloc(n + 1, 8),
          *cur = calloc(n + 1, 8), *plan = calloc(n + 1, 8), *over = calloc(n + 1, 8), *dplan = calloc(n + 1, 8),
          *dover = calloc(n + 1, 8), *tmpv = calloc(n + 1, 8);
  int *has_max = calloc(n + 1, sizeof(int)), *has_cap = calloc(n + 1, sizeof(int)), *hp = calloc(n + 1, sizeof(int)),
      *ho = calloc(n + 1, sizeof(int)), *dhp = calloc(n + 1, sizeof(int)), *dho = calloc(n + 1, sizeof(int));
  uint32_t* hash = calloc(n + 1, 4);
  npref_t *np = calloc(n + 1, sizeof(npref_t)), *tmp = calloc(n + 1, sizeof(npref_t));
  int64_t total = (f & KAD_W_HAS_DESIRED) ? b->desired[w] : 0;
  const uint8_t* key = b->key + b->key_off[w];
  int klen = b->key_off[w + 1] - b->key_off[w];

  for (int i = 0; i < n; i++) {
    int c = cids[i];
    hash[i] = fnv_cont(s->name_fnv[c], key, klen);
    for (int k = b->pref_off[w]; k < b->pref_off[w + 1]; k++) {
      if (b->pref_id[k] != c) continue;
      uint32_t pf = b->pref_fl[k];
      weight[i] = (pf & KAD_PREF_HAS_WEIGHT) ? pref_val(b, b->pref_w, k) : 0;
      minr[i] = pref_val(b, b->pref_min, k);
      if (pf & KAD_PREF_HAS_MAX) { has_max[i] = 1; maxr[i] = pref_val(b, b->pref_max, k); }
      if (pf & KAD_PREF_HAS_CAP) { has_cap[i] = 1; capv[i] = pref_val(b, b->pref_cap, k); }
    }
    cur[i] = 0;
    for (int k = b->cur_off[w]; k < b->cur_off[w + 1]; k++) if (b->cur_id[k] == c) cur[i] = b->cur_rep[k];
  }
  if (f & KAD_W_DYNAMIC_WEIGHTS) {
    /* CalcWeightLimit (rsp.go:183-213) */
    double sum = 0.0;
    for (int i = 0; i < n; i++) sum += (double)s->alloc_cores[cids[i]];
    for (int i = 0; i < n; i++) {
      if (sum == 0) tmpv[i] = go_f2i(go_round(1000.0 / (double)n));
      else tmpv[i] = go_f2i(go_round((double)s->alloc_cores[cids[i]] / sum * 1000.0 * 1.4));
    }
    /* AvailableToPercentage (rsp.go:215-272) */
    double suma = 0.0;
    for (int i = 0; i < n; i++) if (s->avail_cores[cids[i]] > 0) suma += (double)s->avail_cores[cids[i]];
    if (suma == 0) {
      for (int i = 0; i < n; i++) weight[i] = go_f2i(go_round(1000.0 / (double)n));
    } else {
      int64_t sumtmp = 0;
      for (int i = 0; i < n; i++) {
        double v = (double)s->avail_cores[cids[i]];
        if (v < 0.0) v = 0.0;
        int64_t wt = go_f2i(go_round(v / suma * 1000.0));
        if (wt > tmpv[i]) wt = tmpv[i];
        weight[i] = wt;
        sumtmp = wadd(sumtmp, wt);
      }
      int64_t other = 0, maxw = 0;
      int maxi = -1, ties = 0;
      for (int i = 0; i < n; i++) {
        int64_t wt = go_f2i(go_round((double)weight[i] / (double)sumtmp * 1000.0));
        weight[i] = wt;
        if (wt > maxw) { maxw = wt; maxi = i; ties = 0; }
        else if (wt == maxw && maxw > 0) ties = 1;
        other = wadd(other, wt);
      }
      if (ties) *rflags |= KAD_RF_REMAINDER_TIE;
      if (maxi >= 0) weight[maxi] = wadd(weight[maxi], wsub(1000, other));
    }
  }
  /* planner.Plan (planner.go:83-177) */
  gosort_t d = {np_less, np_swap, np, sc.xs_b, sc.xs_c};
  for (int i = 0; i < n; i++) { np[i].cid = cids[i]; np[i].hash = hash[i]; np[i].weight = weight[i]; np[i].min = minr[i]; np[i].max = maxr[i]; np[i].has_max = has_max[i]; }
  if (n > 1) go_sort(&d, n);
  for (int i = 1; i < n; i++) if (np[i].weight == np[i - 1].weight && np[i].hash == np[i - 1].hash) *rflags |= KAD_RF_HASH_TIE;
  int avoid = (f & KAD_W_AVOID_DISRUPTION) != 0;
  int keep = (f & KAD_W_KEEP_UNSCHED) != 0;
  if (!avoid) keep = 1;
  int64_t rem;
  get_desired_plan(np, n, cids, n, has_cap, capv, total, keep, dplan, dover, dhp, dho, &rem, tmp);
  if (!avoid) {
    for (int i = 0; i < n; i++) { plan[i] = dplan[i]; over[i] = dho[i] ? dover[i] : 0; }
  } else {
    int64_t cur_total = 0, des_total = 0;
    for (int i = 0; i < n; i++) {
      int64_t r = cur[i];
      if (has_cap[i] && capv[i] < r) r = capv[i];
      plan[i] = r;
      cur_total = wadd(cur_total, r);
      des_total = wadd(des_total, dplan[i]);
    }
    for (int i = 0; i < n; i++) over[i] = dho[i] ? dover[i] : 0;
    if (cur_total != des_total) {
      int up = cur_total < des_total;
      int64_t count = up ? des_total - cur_total : cur_total - des_total;
      int m = 0;
      for (int i = 0; i < n; i++) {
        int64_t dsr = dplan[i], c = plan[i];
        if (up ? dsr > c : dsr < c) {
          np[m].cid = cids[i]; np[m].hash = hash[i];
          np[m].weight = up ? dsr - c : c - dsr;
          np[m].min = 0;
          if (up) { np[m].has_max = has_max[i]; np[m].max = has_max[i] ? maxr[i] - c : 0; }
          else { np[m].has_max = 1; np[m].max = c; }
          m++;
        }
      }
      d.ctx = np;
      if (m > 1) go_sort(&d, m);
      int64_t* sp = calloc(n + 1, 8);
      int64_t* so = calloc(n + 1, 8);
      int *shp = calloc(n + 1, sizeof(int)), *sho = calloc(n + 1, sizeof(int));
      int64_t r2;
      get_desired_plan(np, m, cids, n, NULL, NULL, count, 0, sp, so, shp, sho, &r2, tmp);
      for (int i = 0; i < n; i++) if (shp[i]) plan[i] = up ? wadd(plan[i], sp[i]) : wsub(plan[i], sp[i]);
      free(sp); free(so); free(shp); free(sho);
    }
  }
  int cnt = 0;
  for (int i = 0; i < n; i++) {
    int64_t r = wadd(plan[i], over[i]);
    if (r == 0) continue;
    out_c[cnt] = cids[i]; out_r[cnt] = r; cnt++;
  }
  free(cids); free(weight); free(minr); free(maxr); free(capv); free(cur); free(plan); free(over); free(dplan);
  free(dover); free(tmpv); free(has_max); free(has_cap); free(hp); free(ho); free(dhp); free(dho); free(hash);
  free(np); free(tmp);
  return cnt;
}

/* -------------------------------------------------------------- Schedule */
static const int FILTER_ORDER[5] = {KAD_PL_API_RESOURCES, KAD_PL_TAINT_TOLERATION, KAD_PL_CLUSTER_RESOURCES_FIT,
                                    KAD_PL_PLACEMENT_FILTER, KAD_PL_CLUSTER_AFFINITY};
static const int SCORE_ORDER[5] = {KAD_PL_TAINT_TOLERATION, KAD_PL_BALANCED_ALLOCATION, KAD_PL_LEAST_ALLOCATED,
                                   KAD_PL_MOST_ALLOCATED, KAD_PL_CLUSTER_AFFINITY};

static int cmp_i32(const void* a, const void* b) { int32_t x = *(const int32_t*)a, y = *(const int32_t*)b; return (x > y) - (x < y); }

/* genericScheduler.Schedule (core/generic_scheduler.go:92-150) for unit w. */
static void schedule_one(const snap_t* s, const batch_t* b, const kad_profile* prof, int w, int32_t* status,
                         int32_t* count, uint32_t* rflags, int32_t* out_c, int64_t* out_r, uint8_t* dbg_feas,
                         int64_t* dbg_total) {
  uint32_t f = b->flags[w];
  int C = s->C;
  *rflags = 0;
  *count = 0;
  if (f & KAD_W_STICKY) { *status = KAD_ST_STICKY; return; }
  cscore_t* fs = malloc(sizeof(cscore_t) * (C + 1));
  int n = 0;
  for (int c = 0; c < C; c++) { /* findClustersThatFitWorkload :152-169 */
    int ok = 1;
    for (int k = 0; k < 5 && ok; k++)
      if (prof->filter_mask & (1u << FILTER_ORDER[k])) ok = run_filter(s, b, w, c, FILTER_ORDER[k]);
    if (dbg_feas) dbg_feas[(size_t)w * C + c] = (uint8_t)ok;
    if (ok) { fs[n].cid = c; fs[n].score = 0; n++; }
  }
  if (n == 0) { *status = KAD_ST_NO_FEASIBLE; free(fs); return; }
  int64_t* sc = malloc(sizeof(int64_t) * n);
  for (int k = 0; k < 5; k++) { /* RunScorePlugins (runtime/framework.go:139-181) */
    int pl = SCORE_ORDER[k];
    if (!(prof->score_mask & (1u << pl))) continue;
    if (pl == KAD_PL_CLUSTER_AFFINITY && (f & KAD_W_SCORE_ERROR)) {
      *status = KAD_ST_ERR_SCORE; free(sc); free(fs); return;
    }
    for (int i = 0; i < n; i++) sc[i] = run_score(s, b, w, fs[i].cid, pl);
    if (pl == KAD_PL_TAINT_TOLERATION) default_normalize(100, 1, sc, n);
    if (pl == KAD_PL_CLUSTER_AFFINITY) default_normalize(100, 0, sc, n);
    for (int i = 0; i < n; i++) fs[i].score = wadd(fs[i].score, sc[i]);
  }
  free(sc);
  if (dbg_total) for (int i = 0; i < n; i++) dbg_total[(size_t)w * C + fs[i].cid] = fs[i].score;
  int k = n;
  if (prof->select_plugin == KAD_PL_MAX_CLUSTER) { /* max_cluster.go:42-66 */
    if ((f & KAD_W_HAS_MAX_CLUSTERS) && b->maxc[w] < 0) { *status = KAD_ST_ERR_SELECT; free(fs); return; }
    gosort_t d = {cs_less, cs_swap, fs, 17, 5};
    if (prof->flags & KAD_PROFILE_XORSHIFT_GO121) { d.xs_b = 7; d.xs_c = 17; }
    /* detect whether the cut lands inside a run of equal scores (diagnostic flag) */
    go_sort(&d, n);
    if ((f & KAD_W_HAS_MAX_CLUSTERS) && b->maxc[w] < k) k = (int)b->maxc[w];
    if (k > 0 && k < n && fs[k - 1].score == fs[k].score) *rflags |= KAD_RF_TIE_STRADDLE;
  }
  int32_t* sel = malloc(sizeof(int32_t) * (k + 1));
  for (int i = 0; i < k; i++) sel[i] = fs[i].cid;
  qsort(sel, k, sizeof(int32_t), cmp_i32);
  free(fs);
  *status = KAD_ST_OK;
  if (f & KAD_W_DUPLICATE) {
    for (int i = 0; i < k; i++) { out_c[i] = sel[i]; out_r[i] = -1; }
    *count = k;
    free(sel);
    return;
  }
  /* RunReplicasPlugin (runtime/framework.go:211-249) */
  if (k == 0 || !(f & KAD_W_HAS_DESIRED) || b->desired[w] <= 0 || prof->replicas_plugin != KAD_PL_CLUSTER_CAPACITY_WEIGHT) {
    free(sel);
    return;
  }
  sortcfg_t cfg = {17, 5};
  if (prof->flags & KAD_PROFILE_XORSHIFT_GO121) { cfg.xs_b = 7; cfg.xs_c = 17; }
  *count = replica_scheduling(s, b, w, sel, k, out_c, out_r, rflags, cfg);
  free(sel);
}

typedef struct {
  const snap_t* s;
  const batch_t* b;
  const kad_profile* prof;
  int begin, end, stride;
  int32_t *status, *count, *cluster;
  uint32_t* flags;
  int64_t* replicas;
  uint8_t* dbg_feas;
  int64_t* dbg_total;
} job_t;

static void* worker(void* arg) {
  job_t* j = arg;
  for (int w = j->begin; w < j->end; w += j->stride) {
    int64_t o = j->b->out_off[w];
    int64_t cap = j->b->out_off[w + 1] - o;
    int32_t* oc = malloc(sizeof(int32_t) * (j->s->C + 1));
    int64_t* orr = malloc(sizeof(int64_t) * (j->s->C + 1));
    schedule_one(j->s, j->b, j->prof, w, &j->status[w], &j->count[w], &j->flags[w], oc, orr, j->dbg_feas, j->dbg_total);
    int cnt = j->count[w];
    if (cnt > cap) { j->status[w] = -100; cnt = (int)cap; } /* bound violated: packer bug */
    for (int i = 0; i < cnt; i++) { j->cluster[o + i] = oc[i]; j->replicas[o + i] = orr[i]; }
    free(oc); free(orr);
  }
  return NULL;
}

/* Schedule units [begin, end) of the batch with n_threads workers (one unit
 * per worker at a time, like --worker-count goroutines). Outputs follow the
 * kad_result_view layout (indexed by the batch's OUT_OFF).                  */
int kad_ref_schedule(const void* snap_blob, const void* batch_blob, const kad_profile* prof, int begin, int end,
                     int n_threads, int32_t* status, int32_t* count, uint32_t* flags, int32_t* cluster,
                     int64_t* replicas, uint8_t* dbg_feas, int64_t* dbg_total) {
  snap_t s;
  batch_t b;
  if (parse_snap(snap_blob, &s) || parse_batch(batch_blob, &b)) return -1;
  if (end > b.W) end = b.W;
  if (n_threads < 1) n_threads = 1;
  pthread_t* th = malloc(sizeof(pthread_t) * n_threads);
  job_t* jobs = malloc(sizeof(job_t) * n_threads);
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (job_t){&s, &b, prof, begin + t, end, n_threads, status, count, cluster, flags, replicas, dbg_feas, dbg_total};
  }
  int* started = calloc(n_threads, sizeof(int));
  for (int t = 0; t < n_threads; t++) {
    if (n_threads > 1 && pthread_create(&th[t], NULL, worker, &jobs[t]) == 0) started[t] = 1;
    else worker(&jobs[t]); /* single thread, or thread creation refused: run inline */
  }
  for (int t = 0; t < n_threads; t++) if (started[t]) pthread_join(th[t], NULL);
  free(started);
  free(th);
  free(jobs);
  return 0;
}

/* MaxCluster over explicit score rows (max_cluster_test.go shape): selected
 * input positions, in sorted (selection) order.                              */
int kad_ref_select_row(int n, const int64_t* scores, int64_t max_clusters, int has_max, uint32_t pflags,
                       int32_t* out_pos) {
  if (has_max && max_clusters < 0) return -1;
  cscore_t* fs = malloc(sizeof(cscore_t) * (n + 1));
  for (int i = 0; i < n; i++) { fs[i].cid = i; fs[i].score = scores[i]; }
  gosort_t d = {cs_less, cs_swap, fs, 17, 5};
  if (pflags & KAD_PROFILE_XORSHIFT_GO121) { d.xs_b = 7; d.xs_c = 17; }
  go_sort(&d, n);
  int k = n;
  if (has_max && max_clusters < k) k = (int)max_clusters;
  for (int i = 0; i < k; i++) out_pos[i] = fs[i].cid;
  free(fs);
  return k;
}

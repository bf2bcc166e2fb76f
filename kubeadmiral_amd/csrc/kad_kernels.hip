// HIP kernels of libkad.so for gfx950 (MI355X, CDNA4).
//
// schedule_kernel — one 64-lane wavefront per SchedulingUnit:
//   filters (ballot bitmask) → raw scores → per-row max → normalisation →
//   totals → MaxCluster first-k set (radix select + restricted pdqsort replay)
//   → ascending cluster-id output via ballot compaction.
//   Reference: genericScheduler.Schedule, core/generic_scheduler.go:92-150.
// plan_kernel — one wavefront per Divide-mode unit with ≥1 selected cluster:
//   ClusterCapacityWeight (rsp.go:65-181) + planner.Plan (planner.go:83-366).
//
// Nothing here is a dense contraction (no MFMA). Cluster attributes are read
// attribute-major (attr[i*C + c]) so each wave's 64 lanes read 64 consecutive
// clusters: one coalesced 512-B access per i64 attribute. Per-row state lives
// in LDS (per-wave region) when it fits, else in a per-wave global scratch slab.
#include <cstdlib>

#include <type_traits>

#include "kad_device.h"
#include "kad_plan.h"
#include "kad_select.h"
#include "kad_wave.h"

namespace kad {

// Phase profiling (only in builds with -DKAD_PHASE_PROF; scripts/phase_prof.py):
// per-phase s_memtime cycles summed over units, plus event counters.
// Accumulated per wave in registers, flushed once at wave exit into one of
// 256 stripes (a shared counter per phase would serialise the waves).
#ifdef KAD_PHASE_PROF
constexpr int KAD_PSLOTS = 40;  // per-block phase slots (scripts/phase_prof.py NAMES)
__device__ unsigned long long g_phase[256 * KAD_PSLOTS];
// lean kernel: (start, end) s_memtime of every wave of the last launch, for the wave-lifetime split
__device__ unsigned long long g_wavetime[8192 * 2];
// wide kernel: per wave (units taken, the longest unit's s_memtime cycles, realtime of the last dequeue, units
// that straddled a tie, HW_ID, XCC_ID)
__device__ unsigned long long g_wavex[8192 * 6];
// wide kernel, per unit of the last launch (units < 2^20): realtime start; (duration in realtime ticks,
// feasible count n << 32, straddle << 47, global wave << 48) — scripts/unit_trace.py
constexpr int KAD_UTRACE_MAX = 1 << 20;
__device__ unsigned long long g_ustart[KAD_UTRACE_MAX];
__device__ unsigned long long g_uinfo[KAD_UTRACE_MAX];
#define KAD_PT(v) const unsigned long long v = __builtin_readcyclecounter()
#define KAD_PACC uint32_t pacc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}
#define KAD_PADD(i, x) pacc[i] += (uint32_t)(x)
#define KAD_PFLUSH                                                                       \
  if (lane_id() == 0)                                                                    \
    for (int i_ = 0; i_ < 10; ++i_) atomicAdd(&g_phase[(blockIdx.x & 255) * KAD_PSLOTS + i_], pacc[i_])
// lean / wide kernel: slots 10..15 (A, B, D, E, straddles, D on straddles), 24..29 (replay: setup,
// partitions, pivots, insertion sorts, #partitions, feasible count of replayed units)
#define KAD_PFLUSH_LEAN                                                                  \
  if (lane_id() == 0) {                                                                  \
    for (int i_ = 0; i_ < 6; ++i_) atomicAdd(&g_phase[(blockIdx.x & 255) * KAD_PSLOTS + 10 + i_], pacc[i_]); \
    for (int i_ = 6; i_ < 12; ++i_) atomicAdd(&g_phase[(blockIdx.x & 255) * KAD_PSLOTS + 18 + i_], pacc[i_]); \
  }
// plan kernel: slots 16..23 (setup, dynamic weights, first plan, avoid-disruption, output, units)
#define KAD_PFLUSH_PLAN                                                                  \
  if (lane_id() == 0)                                                                    \
    for (int i_ = 0; i_ < 6; ++i_) atomicAdd(&g_phase[(blockIdx.x & 255) * KAD_PSLOTS + 16 + i_], pacc[i_])
// row kernel (thread 0, block-synchronous phases): slots 9 (units), 20 (compaction), 22 (scores),
// 23 (normalise), 30 (select: radix + counts), 31 (pdqsort replay); within the scores 32 (preferred-term
// words) and 33 (thread 0's position loop)
#define KAD_PFLUSH_ROW                                                                   \
  if (threadIdx.x == 0) {                                                                \
    const int sl_[8] = {9, 20, 22, 23, 30, 31, 32, 33};                                  \
    for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_phase[(blockIdx.x & 255) * KAD_PSLOTS + sl_[i_]], pacc[i_]); \
  }
#else
#define KAD_PFLUSH_ROW
#define KAD_PFLUSH_LEAN
#define KAD_PFLUSH_PLAN
#define KAD_PT(v)
#define KAD_PACC
#define KAD_PADD(i, x)
#define KAD_PFLUSH
#endif

// ----------------------------------------------------------- per-wave layout
struct RowLayout {
  size_t tot, fx, idx, perm, posl, posr, feas, sel, place, cur, hist, bytes;
};
__host__ __device__ inline RowLayout row_layout(int C) {
  const size_t Cp = (size_t)((C + 63) & ~63);
  const size_t nw = Cp / 64;
  RowLayout L;
  L.tot = 0;                                     // i64[Cp] total per feasible position
  L.fx = L.tot + 8 * Cp;                         // u32[Cp] fixed scores | TT raw << 16
  L.idx = L.fx + 4 * Cp;                         // u16[Cp] feasible position → cluster id
  L.perm = L.idx + 2 * Cp;                       // u16[Cp] pdqsort replay permutation
  L.posl = L.perm + 2 * Cp;                      // u16[Cp] replay scratch (partition stoppers)
  L.posr = L.posl + 2 * Cp + 128;                // u16[Cp] (posl: Cp + 64 entries, PdqWave)
  L.feas = (L.posr + 2 * Cp + 15) & ~(size_t)15;  // u64[nw] feasibility by cluster
  L.sel = L.feas + 8 * nw;                       // u64[nw] selection by position
  L.place = L.sel + 8 * nw;
  L.cur = L.place + 8 * nw;
  L.hist = L.cur + 8 * nw;
  L.bytes = (L.hist + 4 * 256 + 15) & ~(size_t)15;
  return L;
}
size_t select_wave_bytes(int C) { return row_layout(C).bytes; }
// GSCR rows (state in a global slab): the small per-wave arrays that take atomics — selection, placement
// and current-cluster bitmaps, the radix histogram — stay in LDS (dynamic LDS of the 1-wave blocks)
struct SmallLayout {
  size_t sel, place, cur, hist, bytes;
};
__host__ __device__ inline SmallLayout small_layout(int C) {
  const size_t nw = (size_t)((C + 63) / 64);
  SmallLayout L;
  L.sel = 0;
  L.place = 8 * nw;
  L.cur = 16 * nw;
  L.hist = 24 * nw;
  L.bytes = L.hist + 4 * 256;
  return L;
}

// ---------------------------------------------------------- predicate programs
// labels.Requirement.Matches / fields one-term selectors (apimachinery v0.26.6) per interned
// requirement and cluster. Requirement × cluster bitmask rows: M[r][ch] bit l = requirement r holds on
// cluster 64*ch + l. Every distinct requirement of the batch is evaluated once per cluster here, instead
// of once per (unit, cluster) pair.
// req_mask_kernel: one wave per (segment of <= 64 requirements on ONE label key, group of REQ_G
// consecutive chunks). The wave loads the key's label-value ids (and, when the segment has Gt/Lt, the
// parsed integers) of its REQ_G chunks once — one coalesced row load per chunk for the whole segment,
// not per requirement — and the segment's requirement words into lanes (lane i = requirement i: op,
// count, first four value ids / the threshold), so the per-requirement loop reads its operands with
// v_readlane: compares, one ballot per chunk, one coalesced store of the REQ_G words (lane j = chunk).
constexpr int REQ_G = REQ_SEG_G;
__global__ __launch_bounds__(256) void req_mask_kernel(SnapDev s, BatchDev b, int ngrp) {
  const int lane = lane_id();
  const int C = s.C, nch = (C + 63) >> 6;
  const long gw = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= (long)b.n_seg * ngrp) return;
  const int sg = (int)(gw / ngrp), g0 = (int)(gw % ngrp) * REQ_G;
  const int ng = nch - g0 < REQ_G ? nch - g0 : REQ_G;
  const int key = ldc(&b.req_seg[sg].x), first = ldc(&b.req_seg[sg].y), cnt = ldc(&b.req_seg[sg].z);
  // lane i < cnt: requirement i of the segment (id, word offset, op | n << 8, key word, payload 0..3)
  const bool li = lane < cnt;
  const int4* ent = reinterpret_cast<const int4*>(b.req_perm) + 2 * (size_t)(first + (li ? lane : 0));
  const int4 e0 = ent[0], e1 = ent[1];
  const int rid = e0.x, off = e0.y, w0 = li ? e0.z : 0, kw = e0.w;
  const int pv[4] = {e1.x, e1.y, e1.z, e1.w};
  uint64_t* out = b.req_mask;
  // every segment holds requirements on one label key (key >= 0): the label-free ops (TRUE / FALSE /
  // metadata.name =, !=) always take req_row_kernel (kad_batch_upload's routing)
  int32_t lv[REQ_G];
#pragma unroll
  for (int j = 0; j < REQ_G; ++j) {
    const int c = (g0 + j) * WAVE + lane;
    lv[j] = (j < ng && c < C) ? ldg(s.lval, (uint32_t)(key * C + c)) : -1;
  }
  const int op_l = w0 & 0xff;
  const bool has_int = ballot(li && (op_l == KAD_OP_GT || op_l == KAD_OP_LT)) != 0;
  int64_t lint[REQ_G];
  bool lok[REQ_G];
#pragma unroll
  for (int j = 0; j < REQ_G; ++j) {
    lint[j] = 0;
    lok[j] = false;
  }
  if (has_int) {
#pragma unroll
    for (int j = 0; j < REQ_G; ++j) {
      const int c = (g0 + j) * WAVE + lane;
      const uint32_t cc = (j < ng && c < C) ? (uint32_t)(key * C + c) : 0u;
      lint[j] = ldg(s.lint, cc);
      lok[j] = ldg(s.lok, cc) != 0;
    }
  }
  for (int i = 0; i < cnt; ++i) {
    const int wi = __builtin_amdgcn_readlane(w0, i);
    const int op = wi & 0xff, n = (int)((uint32_t)wi >> 8);
    const int r = __builtin_amdgcn_readlane(rid, i);
    bool hit[REQ_G];
    if (op == KAD_OP_GT || op == KAD_OP_LT) {
      const int64_t thr = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(pv[1], i) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane(pv[0], i));
#pragma unroll
      for (int j = 0; j < REQ_G; ++j) hit[j] = lv[j] >= 0 && lok[j] && (op == KAD_OP_GT ? lint[j] > thr : lint[j] < thr);
    } else if (op == KAD_OP_EXISTS || op == KAD_OP_DNE) {
#pragma unroll
      for (int j = 0; j < REQ_G; ++j) hit[j] = (lv[j] >= 0) == (op == KAD_OP_EXISTS);
    } else {  // IN / NOTIN / EQ: value ids of this key (>= 0; a missing label is -1)
#pragma unroll
      for (int j = 0; j < REQ_G; ++j) hit[j] = false;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < n) {
          const int a = __builtin_amdgcn_readlane(pv[t], i);
#pragma unroll
          for (int j = 0; j < REQ_G; ++j) hit[j] |= lv[j] == a;
        }
      if (n > 4) {
        const int offi = __builtin_amdgcn_readlane(off, i);
        for (int t = 4; t < n; ++t) {
          const int a = ldc(b.req + offi + 2 + t);
#pragma unroll
          for (int j = 0; j < REQ_G; ++j) hit[j] |= lv[j] == a;
        }
      }
      if (op == KAD_OP_NOTIN)
#pragma unroll
        for (int j = 0; j < REQ_G; ++j) hit[j] = !hit[j];  // NotIn: a missing label matches too
    }
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < REQ_G; ++j) {
      const int c = (g0 + j) * WAVE + lane;
      const uint64_t m = ballot(hit[j] && c < C && j < ng);
      acc = lane == j ? m : acc;
    }
    if (lane < ng) out[(size_t)r * nch + g0 + lane] = acc;
  }
}

// req_row_kernel: one lane per (value-row requirement, REQ_RC consecutive chunks): In / Equals = OR of the
// value rows, NotIn = its complement (a missing label matches), Exists / DoesNotExist = the key row or its
// complement; TRUE / FALSE / metadata.name =, != are constants or one bit (no loads). The requirement's
// 32-B entry is read once per lane for its REQ_RC words (C5: 100k requirements x 157 chunks).
constexpr int REQ_RC = 4;
__global__ __launch_bounds__(256) void req_row_kernel(SnapDev s, BatchDev b, int zero_rows) {
  const int nch = (s.C + 63) >> 6;
  const int nq = (nch + REQ_RC - 1) / REQ_RC;
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  // the row list (rows_n, rows_head) emptied before prep_kernel appends to it (early routing): here
  // instead of a separate memset launch
  if (zero_rows && g < 2) b.rows_n[g] = 0;
  if (g >= (long)b.n_rowreq * nq) return;
  const int i = (int)(g / nq), ch0 = (int)(g - (long)i * nq) * REQ_RC;
  const int4 e0 = b.req_rows[2 * (size_t)i], e1 = b.req_rows[2 * (size_t)i + 1];
  const int rid = e0.x, op = e0.y & 0xff, n = (int)((uint32_t)e0.y >> 8), key = e0.z;
  const int v[VR_MAX_VALS] = {e0.w, e1.x, e1.y, e1.z, e1.w};
  const uint64_t tail = (s.C & 63) ? (1ull << (s.C & 63)) - 1 : ~0ull;  // clusters past C: never
  uint64_t* out = b.req_mask + (size_t)rid * nch;
  if (op == KAD_OP_TRUE || op == KAD_OP_FALSE || op == KAD_OP_NAME_EQ || op == KAD_OP_NAME_NE) {
    // label-free: metadata.name = / != the cluster with snapshot id `key` (-1: no such cluster)
#pragma unroll
    for (int k = 0; k < REQ_RC; ++k) {
      const int ch = ch0 + k;
      if (ch >= nch) break;
      const uint64_t one = (key >= 0 && (key >> 6) == ch) ? 1ull << (key & 63) : 0ull;
      uint64_t acc = op == KAD_OP_TRUE ? ~0ull : op == KAD_OP_FALSE ? 0ull : op == KAD_OP_NAME_EQ ? one : ~one;
      if (ch == nch - 1) acc &= tail;
      out[ch] = acc;
    }
    return;
  }
  const uint64_t* kr = s.vrows + (size_t)key * (VR_SLOTS + 1) * nch;
  uint64_t acc[REQ_RC];
#pragma unroll
  for (int k = 0; k < REQ_RC; ++k) acc[k] = 0;
  auto or_row = [&](const uint64_t* row) {  // the lane's REQ_RC words of one value row, loads issued together
    uint64_t w[REQ_RC];
#pragma unroll
    for (int k = 0; k < REQ_RC; ++k) w[k] = ch0 + k < nch ? row[ch0 + k] : 0ull;
#pragma unroll
    for (int k = 0; k < REQ_RC; ++k) acc[k] |= w[k];
  };
  if (op == KAD_OP_EXISTS || op == KAD_OP_DNE) {
    or_row(kr + (size_t)VR_SLOTS * nch);
  } else {
#pragma unroll
    for (int t = 0; t < VR_MAX_VALS; ++t)
      if (t < n) or_row(kr + (size_t)v[t] * nch);
  }
  const bool neg = op == KAD_OP_NOTIN || op == KAD_OP_DNE;
#pragma unroll
  for (int k = 0; k < REQ_RC; ++k) {
    const int ch = ch0 + k;
    if (ch >= nch) break;
    uint64_t x = neg ? ~acc[k] : acc[k];
    if (ch == nch - 1) x &= tail;
    out[ch] = x;
  }
}

// SnapDev::res4 / res_iv (clean snapshots): the same expressions as the wide kernel's block cache
__global__ __launch_bounds__(256) void res_cols_kernel(SnapDev s, double4* r4, float2* iv, ulonglong4* p4) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= s.C) return;
  double capc, avc, capm, avm;
  score_res(s.alloc_cpu[c], s.used_cpu[c], capc, avc);
  score_res(s.alloc_mem[c], s.used_mem[c], capm, avm);
  r4[c] = make_double4(avc, avm, capc, capm);
  iv[c] = make_float2((float)(100.0 / capc), (float)(100.0 / capm));
  if (p4) {
    const int TW = s.TW;
    p4[c] = make_ulonglong4(TW > 0 ? s.pns[c] : 0ull, TW > 1 ? s.pns[(size_t)s.C + c] : 0ull,
                            TW > 2 ? s.pns[2 * (size_t)s.C + c] : 0ull, TW > 3 ? s.pns[3 * (size_t)s.C + c] : 0ull);
  }
}

// SnapDev::vrows: one wave per (key, chunk), lane = cluster; lane s < VR_SLOTS collects value s's word
__global__ __launch_bounds__(256) void value_rows_kernel(SnapDev s, uint64_t* out) {
  const int lane = lane_id();
  const int nch = (s.C + 63) >> 6;
  const long gw = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= (long)s.K * nch) return;
  const int k = (int)(gw / nch), ch = (int)(gw % nch);
  const int c = ch * WAVE + lane;
  const int v = c < s.C ? ldg(s.lval, (uint32_t)(k * s.C + c)) : -1;
  uint64_t mine = 0;
  for (int t = 0; t < VR_SLOTS; ++t) {
    const uint64_t m = ballot(v == t);
    mine = lane == t ? m : mine;
  }
  const uint64_t has = ballot(v >= 0);
  uint64_t* kr = out + (size_t)k * (VR_SLOTS + 1) * nch + ch;
  kr[(size_t)lane * nch] = mine;
  if (lane == 0) kr[(size_t)VR_SLOTS * nch] = has;
}

// A unit's program (filter / score words) held in VGPR lanes: word i < 64 is
// read with v_readlane (no memory latency on the interpretation chain);
// longer programs fall back to scalar loads for the tail.
struct ProgRegs {
  const int32_t* p;
  int v;  // lane l holds p[l] (l < len)
  __device__ __forceinline__ int operator[](int i) const {
    return i < WAVE ? __builtin_amdgcn_readlane(v, i) : ldc(p + i);
  }
};
__device__ __forceinline__ ProgRegs load_prog(const int32_t* p, int len) {
  const int l = lane_id();
  return ProgRegs{p, l < len ? ldg(p, (uint32_t)l) : 0};
}

// ClusterAffinity.Filter (cluster_affinity.go:50-94) with
// clusterselector.MatchClusterSelectorTerms (clusterselector/util.go:97-132)
// over requirement bitmask rows, one lane per 64-cluster chunk: lane l
// returns the affinity word of chunk ch0 + l (every cluster evaluated
// independently, so the result ANDs with the other filters afterwards).
__device__ uint64_t affinity_filter_chunks(const uint64_t* rows, const ProgRegs& P, int nch, int ch0) {
  const int ch = ch0 + lane_id();
  const uint32_t chc = ch < nch ? (uint32_t)ch : 0u;
  auto row = [&](int id) { return ldg(rows, (uint32_t)id * (uint32_t)nch + chc); };
  auto and_rows = [&](uint64_t m, int at, int n) {
    int i = 0;
    for (; i + 4 <= n; i += 4) {  // four independent loads in flight
      const uint64_t r0 = row(P[at + i]), r1 = row(P[at + i + 1]), r2 = row(P[at + i + 2]), r3 = row(P[at + i + 3]);
      m &= r0 & r1 & r2 & r3;
    }
    for (; i < n; ++i) m &= row(P[at + i]);
    return m;
  };
  int pc = 0;
  const int n_sel = P[pc++];
  uint64_t m = and_rows(~0ull, pc, n_sel);  // SelectorFromSet
  pc += n_sel;
  if (!P[pc++]) return m;  // Required == nil: Success
  const int n_terms = P[pc++];
  uint64_t matched = 0, undecided = m;
  for (int t = 0; t < n_terms; t++) {
    if (!ballot(undecided != 0)) break;
    const int tf = P[pc], ne = P[pc + 1], nf = P[pc + 2];
    const int at = pc + 3;
    pc += 3 + ne + nf;
    if (!(tf & (KAD_TERM_HAS_EXPR | KAD_TERM_HAS_FIELD))) continue;  // nil/empty term selects nothing
    uint64_t cand = undecided;
    if (tf & KAD_TERM_HAS_EXPR) {
      if (!(tf & KAD_TERM_EXPR_VALID)) break;  // invalid selector reached: false for every undecided cluster
      cand = and_rows(cand, at, ne);
    }
    if (tf & KAD_TERM_HAS_FIELD) {
      if (!(tf & KAD_TERM_FIELD_VALID)) {  // reached only where the expressions matched
        undecided &= ~cand;
        continue;
      }
      cand = and_rows(cand, at + ne, nf);
    }
    matched |= cand;
    undecided &= ~cand;
  }
  return matched;
}

// ClusterAffinity.Score raw (cluster_affinity.go:96-135) for cluster c (per lane).
__device__ int64_t affinity_score(const uint64_t* rows, const int32_t* p, int nch, int c) {
  int pc = 0;
  const int n_terms = ldc(p + pc++);
  int64_t score = 0;
  const int ch = c >> 6, bit = c & 63;
  for (int t = 0; t < n_terms; t++) {
    const int32_t wgt = ldc(p + pc), ne = ldc(p + pc + 1);
    const int32_t* ids = p + pc + 2;
    pc += 2 + ne;
    bool m = true;
    for (int i = 0; i < ne; i++) m = m && ((ldg(rows, (uint32_t)ldc(ids + i) * (uint32_t)nch + ch) >> bit) & 1);
    if (m) score = wadd(score, wgt);
  }
  return score;
}

// The same score with the unit's program words 0..63 in the lanes of `pv` (one vector load of the window at
// the program's offset; the batch buffer has 256 B of slack past the blob, BatchDev): the program is parsed
// with v_readlane, and each term's expression rows load together, four at a time (the AND of a term's rows
// at c is the AND of their bits) — one memory round trip per term instead of a scalar load chain through
// the program plus one load per expression. Words past 63 are read from memory (sp = the program).
__device__ __forceinline__ int64_t affinity_score_pv(const uint64_t* rows, uint32_t pv, const int32_t* sp, int nch,
                                                     int c) {
  auto pw = [&](int i) -> int { return i < WAVE ? __builtin_amdgcn_readlane((int)pv, i) : ldc(sp + i); };
  const int n_terms = pw(0);
  int pc = 1;
  int64_t score = 0;
  const uint32_t ch = (uint32_t)(c >> 6);
  const int bit = c & 63;
  for (int t = 0; t < n_terms; t++) {
    const int32_t wgt = pw(pc), ne = pw(pc + 1);
    const int at = pc + 2;
    pc += 2 + ne;
    uint64_t all = ~0ull;
    for (int i0 = 0; i0 < ne; i0 += 4) {
      uint64_t r[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int i = i0 + u < ne ? i0 + u : ne - 1;  // (repeats past ne: AND is idempotent)
        r[u] = ldg(rows, (uint32_t)pw(at + i) * (uint32_t)nch + ch);
      }
      all &= r[0] & r[1] & r[2] & r[3];
    }
    if ((all >> bit) & 1) score = wadd(score, wgt);
  }
  return score;
}

// least_allocated.go:88-94 / most_allocated.go:90-97:
//   capacity == 0 || requested > capacity ? 0 : (x * 100) / capacity
// with x = capacity - requested (least) or requested (most). Fast path for
// 0 <= requested <= capacity < 2^46 (every real cluster): x*100 < 2^53 and the
// quotient is in [0, 100], so an f64 reciprocal estimate corrected twice with
// exact f64 products gives the exact integer quotient; anything else takes the
// Go-wrapping int64 path.
__device__ __forceinline__ int64_t alloc_score(int64_t req, int64_t cap, bool most) {
  if (cap == 0 || req > cap) return 0;
  if (cap > 0 && req >= 0 && cap < (1ll << 46)) {
    const double cd = (double)cap;
    const double ad = (double)(most ? req : cap - req) * 100.0;  // exact
    int q = (int)(ad * __builtin_amdgcn_rcp(cd));
    double r = ad - (double)q * cd;  // exact: q * cd < 2^53
    q += (r >= cd) - (r < 0.0);
    r = ad - (double)q * cd;
    q += (r >= cd) - (r < 0.0);
    return q;
  }
  const int64_t num = wmul(most ? req : wsub(cap, req), 100);
  return go_div(num, cap);
}
// floor(100 x / cap) for integer-valued 0 <= x <= cap, 1 <= cap < 2^46 (the
// lean kernel's clean-snapshot path): the f32 estimate x * (100/cap) is within
// 1e-4 of the quotient (<= 100), so one exact f64 correction (100x and q*cap
// are integers < 2^53) gives the exact Go integer quotient
__device__ __forceinline__ int quot100(double x, double cap, float inv100) {
  int q = (int)((float)x * inv100);
  const double r = __builtin_fma(-(double)q, cap, x * 100.0);
  q += (int)(r >= cap) - (int)(r < 0.0);
  return q;
}
__device__ __forceinline__ int64_t least_requested(int64_t req, int64_t cap) { return alloc_score(req, cap, false); }
__device__ __forceinline__ int64_t most_requested(int64_t req, int64_t cap) { return alloc_score(req, cap, true); }
// balanced_allocation.go:45-88 — IEEE float64, no contraction (-ffp-contract=off)
__device__ __forceinline__ int64_t balanced_d(double cf, double mf) {
  if (cf >= 1 || mf >= 1) return 0;
  const double diff = fabs(cf - mf);
  const double one_minus = 1 - diff;
  return go_f2i(one_minus * 100.0);
}
__device__ __forceinline__ int64_t balanced(int64_t rc, int64_t cc, int64_t rm, int64_t cm) {
  const double cf = cc == 0 ? 1.0 : (double)rc / (double)cc;
  const double mf = cm == 0 ? 1.0 : (double)rm / (double)cm;
  if (cf >= 1 || mf >= 1) return 0;
  const double diff = fabs(cf - mf);
  const double one_minus = 1 - diff;
  return go_f2i(one_minus * 100.0);
}

constexpr uint32_t BIT(int pl) { return 1u << pl; }

// ========================================================= schedule kernel
// The kernel takes one by-value argument block and reads it through the
// kernarg segment pointer, laundered per phase (kargs()): argument loads then
// sit next to their uses instead of being hoisted to the entry, where ~60
// live pointers overflow the SGPR file and spill to VGPR lanes.
struct SchedArgs {
  SnapDev s;
  BatchDev b;
  OutDev o;
  ProfDev p;
  char* gscratch;
  int wave_bytes, waves_per_block, w_stride;
  const int32_t* list;    // non-null: schedule units list[0 .. *list_n) (the lean kernel's defer list)
  const int32_t* list_n;
};
typedef const __attribute__((address_space(4))) SchedArgs* KArgs;
__device__ __forceinline__ KArgs kargs() {
  return (KArgs)opq((uintptr_t)__builtin_amdgcn_kernarg_segment_ptr());
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
// q = num / den for Go int64 when 0 <= num < 2^24, den > 0 (f32 path), else go_div
__device__ __forceinline__ int64_t div_fast(int64_t num, int64_t den) {
  if (num >= 0 && num < (1 << 24) && den > 0) return small_quot(num, den);
  return go_div(num, den);
}

__device__ __forceinline__ void unit_status(KArgs a, int w, int32_t st) {
  if (lane_id() == 0) {
    a->o.status[w] = st;
    a->o.count[w] = 0;
    a->o.flags[w] = 0;
  }
}

template <bool GSCR>
__global__ __launch_bounds__(256) void schedule_kernel(SchedArgs args) {
  (void)args;  // read through kargs()
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: per-unit loads go scalar
  int gw, w_stride, C, TW, W;
  char* region;
  uint32_t fm, sm;
  int xs_b, xs_c;
  {
    KArgs a = kargs();
    const int wpb = a->waves_per_block, wbytes = a->wave_bytes;
    gw = blockIdx.x * wpb + wv;
    w_stride = a->w_stride;
    region = GSCR ? a->gscratch + (size_t)gw * wbytes : smem + (size_t)wv * wbytes;
    C = a->s.C;
    TW = a->s.TW;
    W = a->list ? *a->list_n : a->b.W;
    fm = a->p.filter_mask;
    sm = a->p.score_mask;
    xs_b = (a->p.flags & KAD_PROFILE_XORSHIFT_GO121) ? 7 : 17;
    xs_c = (a->p.flags & KAD_PROFILE_XORSHIFT_GO121) ? 17 : 5;
  }
  const RowLayout L = row_layout(C);
  int64_t* tot = (int64_t*)(region + L.tot);
  uint32_t* fx = (uint32_t*)(region + L.fx);
  uint16_t* idx = (uint16_t*)(region + L.idx);
  uint16_t* perm = (uint16_t*)(region + L.perm);
  const SmallLayout SL = small_layout(C);
  uint64_t* selb = (uint64_t*)(GSCR ? smem + SL.sel : region + L.sel);
  uint64_t* plb = (uint64_t*)(GSCR ? smem + SL.place : region + L.place);
  uint64_t* curb = (uint64_t*)(GSCR ? smem + SL.cur : region + L.cur);
  uint32_t* hist = (uint32_t*)(GSCR ? smem + SL.hist : region + L.hist);
  uint16_t* posl = (uint16_t*)(region + L.posl);
  uint16_t* posr = (uint16_t*)(region + L.posr);
  const int nch = (C + 63) >> 6;
  const bool f_taint = fm & BIT(KAD_PL_TAINT_TOLERATION), f_api = fm & BIT(KAD_PL_API_RESOURCES);
  const bool f_aff = fm & BIT(KAD_PL_CLUSTER_AFFINITY), f_place = fm & BIT(KAD_PL_PLACEMENT_FILTER);

  KAD_PACC;
  for (int wi = gw; wi < W; wi += w_stride) {
    KAD_PT(t0);
    KArgs a = kargs();
    const int w = a->list ? ldc(a->list + wi) : wi;
    const uint32_t f = ldc(a->b.flags + w);
    if (f & KAD_W_STICKY) {  // generic_scheduler.go:101-104
      unit_status(a, w, KAD_ST_STICKY);
      continue;
    }
    const bool use_place = f_place && (f & KAD_W_HAS_PLACEMENT);
    const bool use_cur = f_taint && (f & KAD_W_HAS_CURRENT);
    if (use_place || use_cur) {
      for (int i = lane; i < nch; i += WAVE) {
        plb[i] = 0;
        curb[i] = 0;
      }
      wsync<GSCR>();
      if (use_place) {
        const int32_t* pl = a->b.place;
        for (int j = ldc(a->b.place_off + w) + lane; j < ldc(a->b.place_off + w + 1); j += WAVE) {
          const int c = ldg(pl, (uint32_t)j);
          atomicOr((unsigned long long*)&plb[c >> 6], 1ull << (c & 63));
        }
      }
      if (use_cur) {
        const int32_t* cu = a->b.cur_id;
        for (int j = ldc(a->b.cur_off + w) + lane; j < ldc(a->b.cur_off + w + 1); j += WAVE) {
          const int c = ldg(cu, (uint32_t)j);
          atomicOr((unsigned long long*)&curb[c >> 6], 1ull << (c & 63));
        }
      }
      wsync<GSCR>();
    }
    const int gv = ldc(a->b.gvk + w);
    const int ts = ldc(a->b.tolset + w);
    const int64_t rq_cpu = ldc(a->b.req_cpu + w), rq_mem = ldc(a->b.req_mem + w);
    const bool fit_on = (fm & BIT(KAD_PL_CLUSTER_RESOURCES_FIT)) && (f & KAD_W_FIT_NONZERO);
    const int s0 = ldc(a->b.sreq_off + w), s1 = ldc(a->b.sreq_off + w + 1);
    ProgRegs FP{nullptr, 0};
    if (f_aff) {
      const int fo = ldc(a->b.fprog_off + w), fl = ldc(a->b.fprog_off + w + 1) - fo;
      FP = load_prog(a->b.fprog + fo, fl);
    }

    // ---------------- A: filters → compacted feasible list (findClustersThatFitWorkload, :152-169)
    // Per chunk of 64 clusters every attribute load is unconditional, so one
    // memory round trip serves all filters; ClusterAffinity comes from the
    // lane-per-chunk bitmask evaluation.
    int n = 0;
    uint64_t affv = ~0ull;
    for (int ch = 0; ch < nch; ++ch) {
      KArgs ac = kargs();
      if (f_aff && (ch & 63) == 0) affv = affinity_filter_chunks(ac->b.req_mask, FP, nch, ch);
      const int c = ch * WAVE + lane;
      const uint32_t cl = c < C ? (uint32_t)c : 0u;
      bool ok = c < C;
      if (f_aff) ok &= (readlane64(affv, ch & 63) >> lane) & 1;
      if (use_place) ok &= (plb[ch] >> lane) & 1;
      if (f_taint) {  // taint_toleration.go:50-77: NoSchedule/NoExecute (NoExecute only if not yet scheduled)
        const uint64_t* tolA = ac->b.tol_all + (size_t)ts * TW;
        const uint64_t* nsne = ac->s.nsne;
        const uint64_t* ne = ac->s.ne;
        const bool sch = use_cur && ((curb[ch] >> lane) & 1);
        for (int t = 0; t < TW; ++t) {
          uint64_t x = ldg(nsne, (uint32_t)(t * C) + cl);
          if (use_cur) {
            const uint64_t y = ldg(ne, (uint32_t)(t * C) + cl);
            x = sch ? y : x;
          }
          ok &= (x & ~ldc(tolA + t)) == 0;
        }
      }
      if (f_api) {  // api_resources.go:42-63
        if (gv >= 0)
          ok &= (ldg(ac->s.gvk, (uint32_t)((gv >> 6) * C) + cl) >> (gv & 63)) & 1;
        else
          ok = false;
      }
      if (fit_on) {  // cluster_resources_fit.go:48-90
        const int64_t acpu = ldg(ac->s.alloc_cpu, cl), ucpu = ldg(ac->s.used_cpu, cl);
        const int64_t amem = ldg(ac->s.alloc_mem, cl), umem = ldg(ac->s.used_mem, cl);
        ok &= (int)(acpu >= wadd(rq_cpu, ucpu)) & (int)(amem >= wadd(rq_mem, umem));
        for (int j = s0; j < s1; ++j) {
          KArgs aj = kargs();
          const int sid = ldc(aj->b.sreq_id + j);
          const int64_t v = ldc(aj->b.sreq_val + j);
          int64_t al = 0, us = 0;
          if (sid >= 0) {
            al = ldg(aj->s.alloc_s, (uint32_t)(sid * C) + cl);
            us = ldg(aj->s.used_s, (uint32_t)(sid * C) + cl);
          }
          ok &= al >= wadd(v, us);
        }
      }
      const uint64_t m = ballot(ok);
      if (ok) idx[n + mbcnt(m)] = (uint16_t)c;  // compact feasible clusters, snapshot order
      n += popc64(m);
      uint8_t* dbg = ac->o.dbg_feas;
      if (dbg && c < C) dbg[(size_t)w * C + c] = ok;
    }
    KAD_PT(t1);
    KAD_PADD(0, t1 - t0);
    if (n == 0) {  // generic_scheduler.go:112-114
      unit_status(kargs(), w, KAD_ST_NO_FEASIBLE);
      continue;
    }
    if ((sm & BIT(KAD_PL_CLUSTER_AFFINITY)) && (f & KAD_W_SCORE_ERROR)) {  // framework.go:149-159
      unit_status(kargs(), w, KAD_ST_ERR_SCORE);
      continue;
    }
    wsync<GSCR>();

    // ---------------- B: raw scores on the compacted feasible list (RunScorePlugins, framework.go:139-181)
    int ttmax = 0;
    int64_t affmax = 0;
    {
      KArgs ab = kargs();
      const uint64_t* tolP = ab->b.tol_pns + (size_t)ts * TW;
      const int32_t* sp = ab->b.sprog + ldc(ab->b.sprog_off + w);
      for (int j = lane; j < n; j += WAVE) {
        const uint32_t c = idx[j];
        int64_t fixed = 0;
        if (sm & (BIT(KAD_PL_LEAST_ALLOCATED) | BIT(KAD_PL_MOST_ALLOCATED) | BIT(KAD_PL_BALANCED_ALLOCATION))) {
          const int64_t rc = wadd(ldg(ab->s.used_cpu, c), rq_cpu), rm = wadd(ldg(ab->s.used_mem, c), rq_mem);
          const int64_t cc = ldg(ab->s.alloc_cpu, c), cm = ldg(ab->s.alloc_mem, c);
          if (sm & BIT(KAD_PL_LEAST_ALLOCATED))
            fixed += go_div(wadd(least_requested(rm, cm), least_requested(rc, cc)), 2);
          if (sm & BIT(KAD_PL_MOST_ALLOCATED))
            fixed += go_div(wadd(most_requested(rm, cm), most_requested(rc, cc)), 2);
          if (sm & BIT(KAD_PL_BALANCED_ALLOCATION)) fixed += balanced(rc, cc, rm, cm);
        }
        int tt = 0;
        if (sm & BIT(KAD_PL_TAINT_TOLERATION))
          for (int t = 0; t < TW; ++t) tt += popc64(ldg(ab->s.pns, (uint32_t)(t * C) + c) & ~ldc(tolP + t));
        int64_t aff = 0;
        if (sm & BIT(KAD_PL_CLUSTER_AFFINITY)) aff = affinity_score(ab->b.req_mask, sp, nch, c);
        fx[j] = (uint32_t)fixed | ((uint32_t)tt << 16);
        tot[j] = aff;
        ttmax = tt > ttmax ? tt : ttmax;
        affmax = aff > affmax ? aff : affmax;
      }
    }
    if (sm & BIT(KAD_PL_TAINT_TOLERATION)) ttmax = wave_max_u_i32(ttmax);
    if (sm & BIT(KAD_PL_CLUSTER_AFFINITY)) affmax = wave_max_u_i64(affmax);
    wsync<GSCR>();
    KAD_PT(t2);
    KAD_PADD(1, t2 - t1);

    // ---------------- C: DefaultNormalizeScore (framework/util.go:455-483) + sum
    int64_t rmin = I64_MAX, rmax = I64_MIN;
    {
      int64_t* dbt = kargs()->o.dbg_total;
      for (int j = lane; j < n; j += WAVE) {
        const uint32_t x = fx[j];
        int64_t t = (int64_t)(x & 0xFFFF);
        if (sm & BIT(KAD_PL_TAINT_TOLERATION))
          t += ttmax == 0 ? 100 : 100 - (int64_t)small_quot(100 * (int)(x >> 16), ttmax);
        if (sm & BIT(KAD_PL_CLUSTER_AFFINITY)) {
          const int64_t av = tot[j];
          t = wadd(t, affmax == 0 ? av : div_fast(wmul(100, av), affmax));
        }
        tot[j] = t;
        rmin = t < rmin ? t : rmin;
        rmax = t > rmax ? t : rmax;
        if (dbt) dbt[(size_t)w * C + idx[j]] = t;
      }
    }
    rmin = wave_min_u_i64(rmin);
    rmax = wave_max_u_i64(rmax);
    wsync<GSCR>();
    KAD_PT(t3);
    KAD_PADD(2, t3 - t2);

    // ---------------- D: select (framework.go:183-209, max_cluster.go:42-66)
    int64_t k = n;
    {
      KArgs ad = kargs();
      if (ad->p.select_plugin == KAD_PL_MAX_CLUSTER) {
        const bool hm = f & KAD_W_HAS_MAX_CLUSTERS;
        const int64_t mc = ldc(ad->b.maxc + w);
        if (hm && mc < 0) {
          unit_status(ad, w, KAD_ST_ERR_SELECT);
          continue;
        }
        if (hm && mc < k) k = mc;
      }
    }
    SelWs ws{tot, selb, perm, hist, posl, posr};
    const uint32_t rflags = select_topk<GSCR>(ws, n, k, rmin, rmax, xs_b, xs_c);
    KAD_PT(t4);
    KAD_PADD(3, t4 - t3);
    KAD_PADD(6, 1);
    KAD_PADD(7, n);
    if (rflags & KAD_RF_TIE_STRADDLE) {
      KAD_PADD(5, 1);
      KAD_PADD(8, t4 - t3);
    }

    // ---------------- E: output, ascending cluster id (idx is ascending in j)
    {
      KArgs ae = kargs();
      const bool dup = f & KAD_W_DUPLICATE;
      const bool replicas = !dup && ae->p.replicas_plugin == KAD_PL_CLUSTER_CAPACITY_WEIGHT &&
                            (f & KAD_W_HAS_DESIRED) && ldc(ae->b.desired + w) > 0 && k > 0;
      if (dup || replicas) {
        const int64_t off = ldc(ae->b.out_off + w);
        int32_t* oc = ae->o.cluster + off;
        int64_t* orp = ae->o.replicas + off;
        int base = 0;
        for (int jc = 0; jc < ((n + 63) >> 6); ++jc) {
          const uint64_t m = selb[jc];
          if ((m >> lane) & 1) {
            const uint32_t at = (uint32_t)(base + mbcnt(m));
            stg(oc, at, (int32_t)idx[jc * WAVE + lane]);
            stg(orp, at, (int64_t)(dup ? -1 : 0));
          }
          base += popc64(m);
        }
      }
      if (lane == 0) {
        ae->o.status[w] = KAD_ST_OK;
        ae->o.count[w] = (dup || replicas) ? (int32_t)k : 0;  // Divide without replicas plugin: empty map
        ae->o.flags[w] = rflags;
      }
    }
    wsync<GSCR>();
    KAD_PT(t5);
    KAD_PADD(4, t5 - t4);
  }
  KAD_PFLUSH;
}

// ============================================================ prep kernel
// One lane per (unit, PREP_CPL consecutive 64-cluster chunks), every launch,
// before the schedule kernel:
//  * the unit's first lane writes its 64-B UnitRec, routing units that use a
//    feature the lean kernel leaves out (scalar resource requests, more than
//    64 taint ids or GVKs, debug capture) to schedule_kernel (REC_FULL);
//  * every lane writes the unit's static filter words for its chunks: the
//    ClusterAffinity filter (cluster_affinity.go:50-94,
//    MatchClusterSelectorTerms clusterselector/util.go:97-132) evaluated over
//    the requirement rows, ANDed with the PlacementFilter's ClusterNames
//    bitmap (placement/filter.go:37-57); and, for units with
//    CurrentClusters, the current-cluster word (TaintToleration's NoExecute
//    rule, taint_toleration.go:64-78).
// This takes the program → requirement-row load chain off every unit's
// critical path in the schedule kernel.
// p(i): word i of the unit's filter program (prep_kernel stages the first words in LDS). The CPL
// chunks ch0 .. ch0+CPL-1 are evaluated together (their row loads are independent); chunks past
// nch read chunk nch-1 and are never stored.
template <int CPL, class Prog, bool WAVE_ANY = false>
__device__ __forceinline__ void affinity_words(const uint64_t* rows, Prog p, uint32_t nch, uint32_t ch0,
                                               uint64_t (&out)[CPL], uint32_t cst = 1) {
  uint32_t cc[CPL];
#pragma unroll
  for (int k = 0; k < CPL; k++) cc[k] = ch0 + k * cst < nch ? ch0 + k * cst : nch - 1;
  auto and_row = [&](uint64_t (&v)[CPL], int id) {
    uint64_t r[CPL];
#pragma unroll
    for (int k = 0; k < CPL; k++) r[k] = ldg(rows, (uint32_t)id * nch + cc[k]);
#pragma unroll
    for (int k = 0; k < CPL; k++) v[k] &= r[k];
  };
  auto any = [](const uint64_t (&v)[CPL]) {
    uint64_t o = 0;
#pragma unroll
    for (int k = 0; k < CPL; k++) o |= v[k];
    if constexpr (WAVE_ANY) return ballot(o != 0) != 0;  // (one unit per wave: uniform control flow)
    return o != 0;
  };
  int pc = 0;
  const int n_sel = p(pc++);
  uint64_t m[CPL];  // SelectorFromSet: AND of the ClusterSelector entries
#pragma unroll
  for (int k = 0; k < CPL; k++) m[k] = ~0ull;
  for (int i = 0; i < n_sel; i++) and_row(m, p(pc + i));
  pc += n_sel;
#pragma unroll
  for (int k = 0; k < CPL; k++) out[k] = m[k];
  if (!p(pc++)) return;  // Required == nil: Success
  const int n_terms = p(pc++);
  uint64_t matched[CPL], undecided[CPL], cand[CPL];
#pragma unroll
  for (int k = 0; k < CPL; k++) matched[k] = 0, undecided[k] = m[k];
  for (int t = 0; t < n_terms && any(undecided); t++) {
    const int tf = p(pc), ne = p(pc + 1), nf = p(pc + 2);
    const int at = pc + 3;
    pc += 3 + ne + nf;
    if (!(tf & (KAD_TERM_HAS_EXPR | KAD_TERM_HAS_FIELD))) continue;  // nil/empty term selects nothing
#pragma unroll
    for (int k = 0; k < CPL; k++) cand[k] = undecided[k];
    if (tf & KAD_TERM_HAS_EXPR) {
      if (!(tf & KAD_TERM_EXPR_VALID)) break;  // invalid selector reached: false for every undecided cluster
      for (int i = 0; i < ne; i++) and_row(cand, p(at + i));
    }
    if (tf & KAD_TERM_HAS_FIELD) {
      if (!(tf & KAD_TERM_FIELD_VALID)) {  // reached only where the expressions matched
#pragma unroll
        for (int k = 0; k < CPL; k++) undecided[k] &= ~cand[k];
        continue;
      }
      for (int i = 0; i < nf; i++) and_row(cand, p(at + ne + i));
    }
#pragma unroll
    for (int k = 0; k < CPL; k++) matched[k] |= cand[k], undecided[k] &= ~cand[k];
  }
#pragma unroll
  for (int k = 0; k < CPL; k++) out[k] = matched[k];
}


// the words of chunks ch0 .. ch0+CPL-1 of the sorted cluster-id list ids[lo, hi): one lower bound of the
// first chunk's base, then the ids inside the CPL chunks four at a time (independent loads)
template <int CPL>
__device__ __forceinline__ void id_list_words(const int32_t* ids, int lo, int hi, uint32_t ch0, uint64_t (&out)[CPL]) {
#pragma unroll
  for (int k = 0; k < CPL; k++) out[k] = 0;
  const int base = (int)ch0 * WAVE, end = base + CPL * WAVE;
  int a = lo, b = hi;
  while (a < b) {  // lower bound of base
    const int mid = (a + b) >> 1;
    if (ids[mid] < base)
      a = mid + 1;
    else
      b = mid;
  }
  for (int j = a; j < hi; j += 4) {
    int v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = j + u < hi ? ids[j + u] : INT32_MAX;
    bool past = false;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int d = v[u] - base;
      if (d >= 0 && d < CPL * WAVE) {
#pragma unroll
        for (int k = 0; k < CPL; k++)
          if ((d >> 6) == k) out[k] |= 1ull << (d & 63);
      }
      past |= v[u] >= end;
    }
    if (past) break;
  }
}

// the words of chunks ch0 + k*cst (k < CPL) of the sorted cluster-id list ids[lo, hi): per chunk one lower
// bound of its base, then the ids inside it four at a time (prep_wave_kernel's strided chunks)
template <int CPL>
__device__ __forceinline__ void id_list_words_strided(const int32_t* ids, int lo, int hi, uint32_t ch0, uint32_t cst,
                                                      uint64_t (&out)[CPL]) {
#pragma unroll
  for (int k = 0; k < CPL; k++) {
    out[k] = 0;
    const int base = (int)(ch0 + k * cst) * WAVE, end = base + WAVE;
    int a = lo, b = hi;
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (ids[mid] < base)
        a = mid + 1;
      else
        b = mid;
    }
    for (int j = a; j < hi; j += 4) {
      int v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) v[u] = j + u < hi ? ids[j + u] : INT32_MAX;
      bool past = false;
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int d = v[u] - base;
        if (d >= 0 && d < WAVE) out[k] |= 1ull << d;
        past |= v[u] >= end;
      }
      if (past) break;
    }
  }
}

// SnapDev::slices row r (r < 64*TW: NoSchedule|NoExecute taint id r; r < 128*TW: NoExecute taint id
// r - 64*TW; else GVK id r - 128*TW, any of the GW words), chunk ch: one wave per (row, ch), lane = cluster
__global__ __launch_bounds__(256) void slice_kernel(SnapDev s, uint64_t* out) {
  const int lane = lane_id();
  const int nch = (s.C + 63) >> 6;
  const int TW = s.TW;
  const long gw = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= (128L * TW + 64L * s.GW) * nch) return;
  const int ch = (int)(gw % nch), r = (int)(gw / nch);
  const int c = ch * WAVE + lane;
  const uint32_t cl = c < s.C ? (uint32_t)c : 0u;
  uint64_t word;
  int bit;
  if (r < 128 * TW) {
    const int t = r % (64 * TW);
    const uint32_t at = (uint32_t)(t >> 6) * (uint32_t)s.C + cl;
    word = r < 64 * TW ? ldg(s.nsne, at) : ldg(s.ne, at);
    bit = t & 63;
  } else {
    const int g = r - 128 * TW;
    word = ldg(s.gvk, (uint32_t)(g >> 6) * (uint32_t)s.C + cl);
    bit = g & 63;
  }
  const uint64_t m = ballot(c < s.C && ((word >> bit) & 1));
  if (lane == 0) out[(size_t)r * nch + ch] = m;
}

// SnapDev::taint_tab: lane per (tbl, g, sub, ch); OR over the set bits of sub of slice 8g + b of table tbl
__global__ __launch_bounds__(256) void taint_table_kernel(SnapDev s, uint64_t* tab) {
  const uint32_t nch = (uint32_t)((s.C + 63) >> 6);
  const uint32_t ng = 8u * (uint32_t)s.TW;  // 8-id groups per table
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g >= 2u * ng * 256 * nch) return;
  const uint32_t ch = g % nch, e = g / nch, sub = e & 255u, grp = (e >> 8) % ng, tbl = (e >> 8) / ng;
  uint64_t m = 0;
  for (uint32_t r = sub; r; r &= r - 1) m |= s.slices[((size_t)tbl * 8 * ng + grp * 8 + __builtin_ctz(r)) * nch + ch];
  tab[g] = m;
}

// TaintToleration.Filter (taint_toleration.go:44-89) and APIResources.Filter (apiresources.go:25-43) of
// unit w on chunks cc[0..CPL) (TW <= TFOLD_MAX_TW): clusters with a NoSchedule|NoExecute taint the unit
// does not tolerate are out — only NoExecute ones on its CurrentClusters (cw) — and clusters without its
// GVK. The untolerated present taints are looked up 8 ids at a time in SnapDev::taint_tab, each lookup
// serving the lane's CPL chunks (independent loads).
template <int CPL>
__device__ __forceinline__ void folded_words(const SnapDev& s, uint32_t fm, uint32_t f, int gvk, const uint64_t* tol,
                                             const uint64_t (&cw)[CPL], uint32_t nch, const uint32_t (&cc)[CPL],
                                             uint64_t (&out)[CPL]) {
#pragma unroll
  for (int k = 0; k < CPL; k++) out[k] = ~0ull;
  if (fm & (1u << KAD_PL_TAINT_TOLERATION)) {
    const bool cur = f & KAD_W_HAS_CURRENT;
    const int TW = s.TW;
    const size_t ng = (size_t)8 * TW;
    uint64_t bad_ns[CPL], bad_ne[CPL];
#pragma unroll
    for (int k = 0; k < CPL; k++) bad_ns[k] = bad_ne[k] = 0;
    for (int tw = 0; tw < TW; tw++) {
      const uint64_t u = s.present_taints[tw] & ~tol[tw];
#pragma unroll
      for (int gi = 0; gi < 8; gi++) {
        const uint32_t sub = (uint32_t)(u >> (8 * gi)) & 255u;
        if (sub) {
          const uint64_t* rn = s.taint_tab + ((size_t)(8 * tw + gi) * 256 + sub) * nch;
          uint64_t x[CPL];
#pragma unroll
          for (int k = 0; k < CPL; k++) x[k] = rn[cc[k]];
#pragma unroll
          for (int k = 0; k < CPL; k++) bad_ns[k] |= x[k];
          if (cur) {
            const uint64_t* re = s.taint_tab + ((ng + 8 * tw + gi) * 256 + sub) * nch;
#pragma unroll
            for (int k = 0; k < CPL; k++) x[k] = re[cc[k]];
#pragma unroll
            for (int k = 0; k < CPL; k++) bad_ne[k] |= x[k];
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < CPL; k++) out[k] = cur ? ((cw[k] & ~bad_ne[k]) | (~cw[k] & ~bad_ns[k])) : ~bad_ns[k];
  }
  if (fm & (1u << KAD_PL_API_RESOURCES)) {  // any GVK id of the snapshot's GW words (-1: no cluster has it)
    const bool has = gvk >= 0 && gvk < 64 * s.GW;
    const uint64_t* rg = s.slices + ((size_t)128 * s.TW + (has ? gvk : 0)) * nch;
#pragma unroll
    for (int k = 0; k < CPL; k++) out[k] &= has ? rg[cc[k]] : 0ull;
  }
}

// #(fit_vals[r] < x) for r = 0, 1 (x0, x1): 8 levels over the LDS fences (fence i = value (i+1)*S - 1,
// S = fit_mp / FIT_FENCES), then log2(S) levels in global memory; both searches interleaved
__device__ __forceinline__ int2 fit_ranks(const SnapDev& s, const int64_t (*fences)[FIT_FENCES], int64_t x0, int64_t x1) {
  int f0 = 0, f1 = 0;
#pragma unroll
  for (int st = FIT_FENCES / 2; st >= 1; st >>= 1) {
    f0 = fences[0][f0 + st - 1] < x0 ? f0 + st : f0;
    f1 = fences[1][f1 + st - 1] < x1 ? f1 + st : f1;
  }
  const int S = s.fit_mp / FIT_FENCES;
  int b0 = f0 * S, b1 = f1 * S;  // the answer lies in [b, b + S - 1]: value b + S - 1 >= x
  for (int st = S >> 1; st >= 1; st >>= 1) {
    const int64_t v0 = ldg(s.fit_vals[0], (uint32_t)(b0 + st - 1)), v1 = ldg(s.fit_vals[1], (uint32_t)(b1 + st - 1));
    b0 = v0 < x0 ? b0 + st : b0;
    b1 = v1 < x1 ? b1 + st : b1;
  }
  return make_int2(b0, b1);
}

#ifndef KAD_PREP_CPL
#define KAD_PREP_CPL 4
#endif
constexpr int PREP_CPL = KAD_PREP_CPL;                 // chunks per lane
#ifndef KAD_PREP_MINW
#define KAD_PREP_MINW 1
#endif
__global__ __launch_bounds__(256, KAD_PREP_MINW) void prep_kernel(SnapDev s, BatchDev b, ProfDev p, int force_full) {
  constexpr int CPL = PREP_CPL;
  __shared__ int32_t prog_words[256 * CPL];  // words CPL*l .. CPL*l+CPL-1 of its unit's filter program, per lane
  const uint32_t nch = (uint32_t)((s.C + 63) >> 6);
  const uint32_t per = nch > 0 ? (nch + CPL - 1) / CPL : 1u;  // lanes per unit
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g == 0) {
    *b.defer_n = 0;
    *b.work_n = 0;
    if (!b.early_rows) {  // early_rows: this kernel appends to rows (the host zeroes both before it runs)
      *b.rows_n = 0;
      *b.rows_head = 0;
    }
  }
  if (g < (uint32_t)WQ_HEADS) b.wq[g * WQ_STRIDE] = 0u;  // the schedule kernels' work heads
  // one block per 256 lanes (a persistent grid striding over the batch measured equal at C3, 188 vs 187 us,
  // and its loop cost C4's 2-lane units 17 us: profiles/r06/ab_c3_prep_persistent.txt)
  const bool live = g < (uint32_t)b.W * per;
  const uint32_t w = live ? g / per : 0u, l = g - w * per, ch0 = l * CPL;
  // the unit's lanes load its program words 0 .. CPL*per-1 with coalesced
  // loads into LDS: the interpreter's word → row chain then runs on LDS
  // reads, not on dependent global loads
  const int32_t fpo = live ? b.fprog_off[w] : 0;
  const int32_t plen = live ? b.fprog_off[w + 1] - fpo : 0;
#pragma unroll
  for (int k = 0; k < CPL; k++) {
    const int i = (int)ch0 + k;
    prog_words[threadIdx.x * CPL + k] = i < plen ? b.fprog[fpo + i] : 0;
  }
  __shared__ int64_t fences[2][FIT_FENCES];  // SnapDev::fitfold: every S-th fit value per resource
  if (s.fitfold) {
    const int S = s.fit_mp / FIT_FENCES;
    for (int i = threadIdx.x; i < 2 * FIT_FENCES; i += 256)
      fences[i / FIT_FENCES][i % FIT_FENCES] = s.fit_vals[i / FIT_FENCES][(i % FIT_FENCES + 1) * S - 1];
  }
  __syncthreads();
  if (!live) return;
  // every per-unit load is issued up front by every lane (the lanes of a
  // unit share its cache lines), so the record lane's chain and the affinity
  // chain below overlap instead of running one after the other
  const uint32_t f = b.flags[w];
  const uint32_t fm = p.filter_mask;
  const int32_t gvk = b.gvk[w], tolset = b.tolset[w], sprog = b.sprog_off[w];
  const int64_t rqc = b.req_cpu[w], rqm = b.req_mem[w], maxc = b.maxc[w], desired = b.desired[w];
  const int64_t oo = b.out_off[w];
  const int32_t so0 = b.sreq_off[w], so1 = b.sreq_off[w + 1];
  const uint64_t tol0 = b.tol_all[(size_t)tolset * b.TW], tolp0 = b.tol_pns[(size_t)tolset * b.TW];
  bool full = force_full != 0;
  // the unfolded schedule kernels cache GVK word 0 only; folded snapshots take every GVK id from the slices
  if ((fm & (1u << KAD_PL_API_RESOURCES)) && gvk >= 64 && !s.fold) full = true;
  if ((fm & (1u << KAD_PL_CLUSTER_RESOURCES_FIT)) && (f & KAD_W_FIT_NONZERO) && so0 < so1) full = true;
  const uint32_t rflags = f | (((f & KAD_W_HAS_DESIRED) && desired > 0) ? REC_DESIRED_POS : 0u) | (full ? REC_FULL : 0u);
  const bool act = ch0 < nch && !(f & KAD_W_STICKY);
  int cnt = 0;  // feasible clusters among this lane's chunks (early_rows)
  if (act) {
    uint64_t m[CPL];
#pragma unroll
    for (int k = 0; k < CPL; k++) m[k] = ~0ull;
    if (fm & (1u << KAD_PL_CLUSTER_AFFINITY)) {
      const int32_t* gp = b.fprog + fpo;
      const int base = ((int)threadIdx.x - (int)l) * CPL;  // the unit's program word 0 in this block (may be < 0)
      auto word = [&](int i) -> int32_t {
        const int t = base + i;
        return (i < (int)(per * CPL) && t >= 0 && t < 256 * CPL) ? prog_words[t] : gp[i];
      };
      affinity_words<CPL>(b.req_mask, word, nch, ch0, m);
    }
    if (s.fitfold && (fm & (1u << KAD_PL_CLUSTER_RESOURCES_FIT)) && (f & KAD_W_FIT_NONZERO)) {
      // fit.go:73-134 (cpu, memory) by threshold rows: clusters whose available amount >= the request
      const int2 j = fit_ranks(s, fences, rqc, rqm);
      const int jc = j.x, jm = j.y;
#pragma unroll
      for (int k = 0; k < CPL; k++) {
        const uint32_t ch = ch0 + k < nch ? ch0 + k : nch - 1;
        m[k] &= ldg(s.fit_rows[0], (uint32_t)jc * nch + ch) & ldg(s.fit_rows[1], (uint32_t)jm * nch + ch);
      }
    }
    const bool place = (fm & (1u << KAD_PL_PLACEMENT_FILTER)) && (f & KAD_W_HAS_PLACEMENT);
    const bool curw = (fm & (1u << KAD_PL_TAINT_TOLERATION)) && (f & KAD_W_HAS_CURRENT);
    uint64_t pw[CPL], cwv[CPL];
    if (place) {
      id_list_words<CPL>(b.place, b.place_off[w], b.place_off[w + 1], ch0, pw);
#pragma unroll
      for (int k = 0; k < CPL; k++) m[k] &= pw[k];
    }
#pragma unroll
    for (int k = 0; k < CPL; k++) cwv[k] = 0;
    if (curw) id_list_words<CPL>(b.cur_id, b.cur_off[w], b.cur_off[w + 1], ch0, cwv);
    if (s.fold) {
      uint32_t cc[CPL];
#pragma unroll
      for (int k = 0; k < CPL; k++) cc[k] = ch0 + k < nch ? ch0 + k : nch - 1;
      uint64_t tw[TFOLD_MAX_TW];
      tw[0] = tol0;
      for (int t = 1; t < s.TW && t < TFOLD_MAX_TW; t++) tw[t] = b.tol_all[(size_t)tolset * b.TW + t];
      uint64_t fw[CPL];
      folded_words<CPL>(s, fm, f, gvk, tw, cwv, nch, cc, fw);
#pragma unroll
      for (int k = 0; k < CPL; k++) m[k] &= fw[k];
    }
#pragma unroll
    for (int k = 0; k < CPL; k++) {
      const uint32_t ch = ch0 + k;
      if (ch >= nch) break;
      if (curw) b.cw[(size_t)w * nch + ch] = cwv[k];
      if (ch == nch - 1 && (s.C & 63)) m[k] &= (1ull << (s.C & 63)) - 1;  // clusters past C: never feasible
      b.sw[(size_t)w * nch + ch] = m[k];
      cnt += popc64(m[k]);
    }
  }
  // early_rows: in the wide kernel's FITF mode (fold + fitfold) the static words are the whole filter, so
  // the unit's feasible count is their popcount (summed over its `per` lanes: a power of two, one wave);
  // a unit the wide kernel would hand to rows (past its sticky / defer checks, more than WIDE_P clusters)
  // is routed here, before the wide kernel starts
  bool route = false;
  if (b.early_rows) {
    for (uint32_t o = 1; o < per; o <<= 1) cnt += __shfl_xor(cnt, (int)o);
    route = act && !(rflags & REC_FULL) && !(f & KAD_W_WIDE_SCORES) && (uint64_t)rqc < (1ull << 46) &&
            (uint64_t)rqm < (1ull << 46) && cnt > WIDE_P;
  }
  if (l == 0) {
    UnitRec r;
    r.flags = rflags | (route ? REC_ROW : 0u);
    r.gvk = gvk;
    r.tolset = tolset;
    r.sprog_off = sprog;
    r.req_cpu = rqc;
    r.req_mem = rqm;
    r.maxc = maxc;
    r.out_off = oo;
    r.tol0 = tol0;
    r.tolp0 = tolp0;
    b.rec[w] = r;
    if (route) b.rows[atomicAdd(b.rows_n, 1)] = (int32_t)w;
  }
}

// prep_wave_kernel<CW> — prep_kernel for wide snapshots (64 < ceil(C/64) <= 64*CW chunks, C5's 10 000
// clusters): one unit per wave, lane l owning chunks l, l+64, ... (CW of them). prep_kernel's lanes pack
// CPL consecutive chunks and ceil(nch/CPL) lanes per unit, so a wave holds parts of two or three units whose
// filter programs diverge (every loop runs the longest unit's trips under exec masks) and a load
// instruction reads every CPL-th word of a row; here the unit's program, tolerations and taint groups are
// wave-uniform (scalar branches; the program words are v_readlane reads of one window load) and every row
// load reads 64 consecutive words. Same outputs as prep_kernel.
template <int CW>
__global__ __launch_bounds__(256) void prep_wave_kernel(SnapDev s, BatchDev b, ProfDev p, int force_full) {
  const uint32_t nch = (uint32_t)((s.C + 63) >> 6);
  const int lane = lane_id();
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g == 0) {
    *b.defer_n = 0;
    *b.work_n = 0;
    if (!b.early_rows) {
      *b.rows_n = 0;
      *b.rows_head = 0;
    }
  }
  if (g < (uint32_t)WQ_HEADS) b.wq[g * WQ_STRIDE] = 0u;
  __shared__ int64_t fences[2][FIT_FENCES];
  if (s.fitfold) {
    const int S = s.fit_mp / FIT_FENCES;
    const int64_t* fv0 = s.fit_vals[0];
    const int64_t* fv1 = s.fit_vals[1];
    for (int i = threadIdx.x; i < FIT_FENCES; i += 256) {
      const int64_t a0 = fv0[(i + 1) * S - 1], a1 = fv1[(i + 1) * S - 1];
      fences[0][i] = a0;
      fences[1][i] = a1;
    }
  }
  __syncthreads();
  // one unit per wave, grid = units / 4 (a unit loop here, even at one trip per wave, took C5's prep
  // 540 -> 588 us: profiles/r06/bisect_c5_prep.txt)
  const int w = __builtin_amdgcn_readfirstlane((int)(g >> 6));
  if (w >= b.W) return;
  const uint32_t f = (uint32_t)ldc(b.flags + w);
  const uint32_t fm = p.filter_mask;
  const int32_t gvk = ldc(b.gvk + w), tolset = ldc(b.tolset + w), sprog = ldc(b.sprog_off + w);
  const int64_t rqc = ldc(b.req_cpu + w), rqm = ldc(b.req_mem + w), maxc = ldc(b.maxc + w), desired = ldc(b.desired + w);
  const int64_t oo = ldc(b.out_off + w);
  const int32_t so0 = ldc(b.sreq_off + w), so1 = ldc(b.sreq_off + w + 1);
  const int32_t fpo = ldc(b.fprog_off + w), plen = ldc(b.fprog_off + w + 1) - fpo;
  const uint64_t tol0 = ldc(b.tol_all + (size_t)tolset * b.TW), tolp0 = ldc(b.tol_pns + (size_t)tolset * b.TW);
  bool full = force_full != 0;
  if ((fm & (1u << KAD_PL_API_RESOURCES)) && gvk >= 64 && !s.fold) full = true;
  if ((fm & (1u << KAD_PL_CLUSTER_RESOURCES_FIT)) && (f & KAD_W_FIT_NONZERO) && so0 < so1) full = true;
  const uint32_t rflags = f | (((f & KAD_W_HAS_DESIRED) && desired > 0) ? REC_DESIRED_POS : 0u) | (full ? REC_FULL : 0u);
  const bool act = !(f & KAD_W_STICKY);
  int cnt = 0;
  if (act) {
    uint32_t cc[CW];
#pragma unroll
    for (int k = 0; k < CW; k++) cc[k] = (uint32_t)(lane + 64 * k) < nch ? (uint32_t)(lane + 64 * k) : nch - 1;
    uint64_t m[CW];
#pragma unroll
    for (int k = 0; k < CW; k++) m[k] = ~0ull;
    if (fm & (1u << KAD_PL_CLUSTER_AFFINITY)) {
      // program words 0..63 in the lanes (one load; the batch buffer's slack covers a window past the blob)
      const int32_t* gp = b.fprog + fpo;
      const int32_t pv = ldg(gp, (uint32_t)lane);
      auto word = [&](int i) -> int32_t { return i < WAVE ? __builtin_amdgcn_readlane(pv, i) : ldc(gp + i); };
      affinity_words<CW, decltype(word), true>(b.req_mask, word, nch, (uint32_t)lane, m, 64u);
    }
    if (s.fitfold && (fm & (1u << KAD_PL_CLUSTER_RESOURCES_FIT)) && (f & KAD_W_FIT_NONZERO)) {
      const int2 j = fit_ranks(s, fences, rqc, rqm);
      const int jc = __builtin_amdgcn_readfirstlane(j.x), jm = __builtin_amdgcn_readfirstlane(j.y);
#pragma unroll
      for (int k = 0; k < CW; k++)
        m[k] &= ldg(s.fit_rows[0], (uint32_t)jc * nch + cc[k]) & ldg(s.fit_rows[1], (uint32_t)jm * nch + cc[k]);
    }
    const bool place = (fm & (1u << KAD_PL_PLACEMENT_FILTER)) && (f & KAD_W_HAS_PLACEMENT);
    const bool curw = (fm & (1u << KAD_PL_TAINT_TOLERATION)) && (f & KAD_W_HAS_CURRENT);
    uint64_t cwv[CW];
#pragma unroll
    for (int k = 0; k < CW; k++) cwv[k] = 0;
    if (place) {
      uint64_t pw[CW];
      id_list_words_strided<CW>(b.place, ldc(b.place_off + w), ldc(b.place_off + w + 1), (uint32_t)lane, 64u, pw);
#pragma unroll
      for (int k = 0; k < CW; k++) m[k] &= pw[k];
    }
    if (curw) id_list_words_strided<CW>(b.cur_id, ldc(b.cur_off + w), ldc(b.cur_off + w + 1), (uint32_t)lane, 64u, cwv);
    if (s.fold) {
      uint64_t tw[TFOLD_MAX_TW];
      tw[0] = tol0;
      for (int t = 1; t < s.TW && t < TFOLD_MAX_TW; t++) tw[t] = ldc(b.tol_all + (size_t)tolset * b.TW + t);
      uint64_t fw[CW];
      folded_words<CW>(s, fm, f, gvk, tw, cwv, nch, cc, fw);
#pragma unroll
      for (int k = 0; k < CW; k++) m[k] &= fw[k];
    }
#pragma unroll
    for (int k = 0; k < CW; k++) {
      const uint32_t ch = (uint32_t)(lane + 64 * k);
      if (ch >= nch) break;
      if (curw) b.cw[(size_t)w * nch + ch] = cwv[k];
      if (ch == nch - 1 && (s.C & 63)) m[k] &= (1ull << (s.C & 63)) - 1;
      b.sw[(size_t)w * nch + ch] = m[k];
      cnt += popc64(m[k]);
    }
  }
  bool route = false;
  if (b.early_rows) {
    cnt = wave_sum_i32(cnt);
    route = act && !(rflags & REC_FULL) && !(f & KAD_W_WIDE_SCORES) && (uint64_t)rqc < (1ull << 46) &&
            (uint64_t)rqm < (1ull << 46) && cnt > WIDE_P;
  }
  if (lane == 0) {
    UnitRec r;
    r.flags = rflags | (route ? REC_ROW : 0u);
    r.gvk = gvk;
    r.tolset = tolset;
    r.sprog_off = sprog;
    r.req_cpu = rqc;
    r.req_mem = rqm;
    r.maxc = maxc;
    r.out_off = oo;
    r.tol0 = tol0;
    r.tolp0 = tolp0;
    b.rec[w] = r;
    if (route) b.rows[atomicAdd(b.rows_n, 1)] = (int32_t)w;
  }
}

int prep_lanes_per_unit(int C) {
  const int nch = (C + 63) >> 6;
  return nch > 0 ? (nch + PREP_CPL - 1) / PREP_CPL : 1;
}

// ====================================================== unit work queue
constexpr int WQ_BATCH = 4;  // units per dequeue
static_assert(WQ_HEADS == 64, "drained-head set is one u64; heads map to XCDs by h & 7");
// Work queue: WQ_HEADS = 64 heads; head h hands out the batches of the h-th contiguous 64th of the
// units. 64 counters (not 8) spread the returning atomics over as many lines: the device-scope
// atomics of 8 XCDs on a few addresses serialise. A wave of block b starts at head b & 63 (blocks go
// round-robin over the 8 XCDs, so head h is started by XCD h & 7) and, when it is drained, moves to
// the next head of its own XCD (h + 8, h + 16, ...) that still has batches, then to any other. A ticket is one
// returning atomicAdd (lane 0), resolved into a batch one batch later, so its latency hides behind a
// batch of work. Every wave's first batch is static (no atomic): wave wv of block b takes batch
// (b >> 6) * wpb + wv of head b & 63, and that head's atomics count on from its static_batches.
// Every wave ends once all heads are drained.
struct WorkTicket {
  int x;             // head of the pending ticket
  int i;             // its atomicAdd result (lane 0); batch index = i + static_batches(x)
  int wpb, nblocks;  // waves per block, grid size: the static first round
  int B;             // units per batch (<= WQ_BATCH): small enough that a wave takes >= ~12 batches
};
// the static first-round batches of head x: one per wave of every block b < nblocks with b & 63 == x
__device__ __forceinline__ int static_batches(const WorkTicket& t, int x) { return t.wpb * ((t.nblocks - x + 63) >> 6); }
__device__ __forceinline__ WorkTicket wq_start(int wpb, int B = WQ_BATCH) {
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  WorkTicket t{(int)(blockIdx.x & (WQ_HEADS - 1)), 0, wpb, (int)gridDim.x, B};
  t.i = (int)(blockIdx.x >> 6) * wpb + wv - static_batches(t, t.x);
  return t;
}
__device__ __forceinline__ void wq_issue(uint32_t* heads, WorkTicket& t) {
  if (lane_id() == 0) t.i = (int)atomicAdd(heads + t.x * WQ_STRIDE, 1u);
}
__device__ __forceinline__ int wq_head_batches(int W, int x, int B) {
  const int s0 = (int)((int64_t)W * x / WQ_HEADS), s1 = (int)((int64_t)W * (x + 1) / WQ_HEADS);
  return (s1 - s0 + B - 1) / B;
}
// the batch [first, first + count) of a ticket; count 0 = queue drained. A drained head costs one
// wave-wide look at all 64 counters (lane l loads head l, device-coherent) and one atomic on a head
// that still has batches — not a walk over the heads with one atomic round trip each.
__device__ __forceinline__ int2 wq_resolve(uint32_t* heads, int W, WorkTicket& t) {
  const int lane = lane_id();
  for (;;) {
    const int x = t.x;
    const int bi = __builtin_amdgcn_readfirstlane(t.i) + static_batches(t, x);
    if (bi < wq_head_batches(W, x, t.B)) {
      const int s0 = (int)((int64_t)W * x / WQ_HEADS), s1 = (int)((int64_t)W * (x + 1) / WQ_HEADS);
      const int first = s0 + bi * t.B;
      return make_int2(first, (s1 - first) < t.B ? (s1 - first) : t.B);
    }
    const uint32_t taken = __hip_atomic_load(heads + lane * WQ_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t open = ballot((int)taken + static_batches(t, lane) < wq_head_batches(W, lane, t.B));
    if (!open) return make_int2(0, 0);
    // same XCD first (heads x & 7 + 8j), in rotation order after x; then the lowest open head
    const uint64_t same = open & (0x0101010101010101ull << (x & 7));
    int nx;
    if (same) {
      const int sh = (x + 1) & 63;
      const uint64_t rot = sh ? (same >> sh) | (same << (64 - sh)) : same;
      nx = (x + 1 + __builtin_ctzll(rot)) & 63;
    } else {
      nx = __builtin_ctzll(open);
    }
    t.x = nx;
    if (lane == 0) t.i = (int)atomicAdd(heads + nx * WQ_STRIDE, 1u);
  }
}

// ================================================= lean schedule kernel
// schedule_lean_kernel<NCH, CL> — the common case, used whenever C fits the
// per-wave LDS budget (fast_path). Each wave owns a run of consecutive units.
// For NCH > 0 (C <= 64*NCH) the block first copies the cluster attributes the
// path reads (fit resources, taint words, GVK word) into an LDS cache shared
// by its waves; a unit's record and static filter words arrive in VGPRs with
// one vector load per 4-unit batch (issued a batch ahead) and are read with
// v_readlane. CL (clean snapshot, SnapDev::clean, NCH > 0): the resource
// columns are cached as exact f64 (capacity, available) + f32 100/cap and
// every total fits 32 bits (see quot100).
// The feasible list is compacted into LDS (snapshot order = the reference's
// feasible list, generic_scheduler.go:152-169); then each lane owns
// positions lane + 64q (q < QMAX), and scores, normalisation and MaxCluster's
// first-k set are computed in registers:
//   * the k-th largest total T from an LDS histogram when the totals span
//     < 128 (one wave prefix sum), else by ballot bisection over [min, max];
//   * cut takes every tie (k - #(>T) == #(==T)): selection = {total >= T};
//   * n <= 12: Go's pdqsort is one stable insertionSort, so the selection is
//     {> T} plus the first k - #(>T) ties in input order;
//   * otherwise the restricted pdqsort replay (kad_select.h PdqWave) on u32
//     keys (total - row minimum) in the wave's LDS region.
// Units routed REC_FULL by prep, or (NCH == 0) with more than 64*QMAX
// feasible clusters, go to the defer list and schedule_kernel afterwards.
constexpr int LEAN_QMAX_DYN = 4;
constexpr int LEAN_BATCH = 4;  // units per work-queue batch (one VGPR of UnitRecs)
static_assert(LEAN_BATCH == WQ_BATCH, "the lean kernel dequeues WQ_BATCH units per ticket");
__host__ __device__ constexpr int lean_qmax(int nch_t) { return nch_t > 0 ? nch_t : LEAN_QMAX_DYN; }
// cached attributes: alloc/used cpu & mem, NS|NE taints, GVK word 0 (always),
// NE taints (taint filter and some unit has CurrentClusters), PNS taints (TaintToleration score)
struct LeanLayout {
  size_t key, idx, pid, posl, posr, bytes;
};
// per-wave region
__host__ __device__ inline LeanLayout lean_layout(int C, int qmax) {
 (void)C;
  const size_t P = (size_t)qmax * 64;  // positions held in registers
  LeanLayout L;
  L.key = 0;                     // u32[P] replay keys (total - row minimum)
  L.idx = L.key + 4 * P;         // u16[P] feasible position → cluster id (NCH > 0: P = Cp)
  L.posl = L.idx;                // u16[P + 64] replay scratch (partition stoppers; then ranks): idx is
                                 // dead once the scores have read the cluster ids into registers
  L.pid = L.idx + 2 * P + 128;   // u16[P] replay: original position at each position
  L.posr = L.pid + 2 * P;        // u16[P]
  L.bytes = (L.posr + 2 * P + 15) & ~(size_t)15;
  return L;
}
// block-shared cluster cache (NCH > 0): n_attrs arrays of Cp i64
__host__ __device__ inline size_t lean_cache_bytes(int C, int n_attrs) { return (size_t)n_attrs * 8 * ((C + 63) & ~63); }
static constexpr int LDS_BUDGET = 64 * 1024;  // per block
bool fast_path(int C) { return C >= 0; }  // the lean kernel runs for every C; the full kernel takes its defer list

struct LeanArgs {
  SnapDev s;
  BatchDev b;
  OutDev o;
  ProfDev p;
  int wave_bytes, waves_per_block, units_per_wave;  // units_per_wave: work-queue batch size (<= LEAN_BATCH)
  int cache_ne, cache_pn;  // optional cache arrays present
};
typedef const __attribute__((address_space(4))) LeanArgs* LArgs;
__device__ __forceinline__ LArgs largs() {
  return (LArgs)opq((uintptr_t)__builtin_amdgcn_kernarg_segment_ptr());
}
__device__ __forceinline__ void lean_status(int w, int32_t st) {
  if (lane_id() == 0) {
    LArgs a = largs();
    a->o.status[w] = st;
    a->o.count[w] = 0;
    a->o.flags[w] = 0;
  }
}
// (inline: the kernarg segment pointer is only defined inside the kernel body)
__device__ __forceinline__ void lean_defer(int w) {
  if (lane_id() == 0) {
    LArgs a = largs();
    const int slot = atomicAdd(a->b.defer_n, 1);
    a->b.defer[slot] = w;
  }
}

// feasible lists longer than the kernel's register positions: the row kernel's list when it runs
// (BatchDev::use_rows: every filter is in the static words), else the full kernel's defer list
__device__ __forceinline__ void lean_row_or_defer(int w) {
  if (lane_id() == 0) {
    LArgs a = largs();
    if (a->b.use_rows) {
      const int slot = atomicAdd(a->b.rows_n, 1);
      a->b.rows[slot] = w;
    } else {
      const int slot = atomicAdd(a->b.defer_n, 1);
      a->b.defer[slot] = w;
    }
  }
}

// CL (clean snapshot, host-checked SnapDev::clean, NCH > 0): resources as exact
// f64 columns, every total in [-2^28, 2^28] (units with wide affinity weights
// or requests outside [0, 2^46) are deferred), so totals live in 32 bits
template <typename TT>
__device__ __forceinline__ TT tadd(TT a, int64_t b) {
  if constexpr (sizeof(TT) == 8)
    return wadd(a, b);
  else
    return a + (TT)b;
}
// SM >= 0: specialised for that score-plugin mask (as schedule_wide_kernel)
template <int NCH, bool CL, int SM = -1>
__global__ __launch_bounds__(256, 6) void schedule_lean_kernel(LeanArgs args) {
  using TT = typename std::conditional<CL, int, int64_t>::type;
  (void)args;  // read through largs()
  constexpr int Q = lean_qmax(NCH);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int C, W, TWs;
  uint32_t fm, sm;
  char* region;
  {
    LArgs a = largs();
    region = smem + (size_t)wv * a->wave_bytes;
    C = a->s.C;
    TWs = a->s.TW;
    W = a->b.W;
    fm = a->p.filter_mask;
    sm = SM >= 0 ? (uint32_t)SM : a->p.score_mask;
  }
  const int nch = (C + 63) >> 6;
  const LeanLayout L = lean_layout(C, Q);
  constexpr int P = Q * 64;
  const int Cp = nch * 64;
  uint32_t* key = (uint32_t*)(region + L.key);
  uint16_t* idx = (uint16_t*)(region + L.idx);
  uint16_t* pid = (uint16_t*)(region + L.pid);
  uint16_t* posl = (uint16_t*)(region + L.posl);
  uint16_t* posr = (uint16_t*)(region + L.posr);
  uint16_t* inv = posl;  // ranks after the replay
  const bool f_taint = fm & BIT(KAD_PL_TAINT_TOLERATION), f_api = fm & BIT(KAD_PL_API_RESOURCES);
  // static filter words carry ClusterAffinity + PlacementFilter, and with SnapDev::fold also TaintToleration
  // + APIResources (prep_kernel)
  const bool fold = largs()->s.fold;
  const bool fitf = largs()->s.fitfold;  // cpu / memory fit in the static words too
  // the static words are always read: they also clear the last chunk's lanes past C (prep_kernel)
  constexpr bool f_sw = true;
  const bool f_fit = fm & BIT(KAD_PL_CLUSTER_RESOURCES_FIT);
  const bool s_res =
      sm & (BIT(KAD_PL_LEAST_ALLOCATED) | BIT(KAD_PL_MOST_ALLOCATED) | BIT(KAD_PL_BALANCED_ALLOCATION));
  const bool s_tt = sm & BIT(KAD_PL_TAINT_TOLERATION);

  // block-shared LDS cache of the cluster attributes (NCH > 0), after the wave regions
  int64_t* cache = (int64_t*)(smem + (size_t)blockDim.x / 64 * largs()->wave_bytes);
  int64_t* c_ac = cache;
  int64_t* c_uc = cache + Cp;
  int64_t* c_am = cache + 2 * Cp;
  int64_t* c_um = cache + 3 * Cp;
  uint64_t* c_ns = (uint64_t*)(cache + 4 * Cp);
  uint64_t* c_gv = (uint64_t*)(cache + 5 * Cp);
  uint64_t* c_ne = nullptr;
  uint64_t* c_pn = nullptr;
  float2* c_iv = nullptr;
  // clean snapshot (host-checked, SnapDev::clean): the resource columns are
  // cached as exact f64 capacity / available (alloc - used) plus f32 100/cap,
  // and fit / Least / Most / Balanced run in f64 compares and one correction
  constexpr bool clean = CL && NCH > 0;
  {
    LArgs a = largs();
    int nx = 6;
    if (a->cache_ne) c_ne = (uint64_t*)(cache + (nx++) * Cp);
    if (a->cache_pn) c_pn = (uint64_t*)(cache + (nx++) * Cp);
    if (clean) c_iv = (float2*)(cache + (nx++) * Cp);
  }
  if constexpr (NCH > 0) {
    LArgs a = largs();
    for (int c = threadIdx.x; c < Cp; c += blockDim.x) {
      const bool in = c < C;
      const uint32_t cl = in ? (uint32_t)c : 0u;
      const int64_t ac = in ? ldg(a->s.alloc_cpu, cl) : 1, uc = in ? ldg(a->s.used_cpu, cl) : 0;
      const int64_t am = in ? ldg(a->s.alloc_mem, cl) : 1, um = in ? ldg(a->s.used_mem, cl) : 0;
      if (clean) {
        double capc, avc, capm, avm;  // (relaxed clusters: only with the fit rows, MODE 3 below)
        score_res(ac, uc, capc, avc);
        score_res(am, um, capm, avm);
        c_ac[c] = __builtin_bit_cast(int64_t, capc);
        c_uc[c] = __builtin_bit_cast(int64_t, avc);
        c_am[c] = __builtin_bit_cast(int64_t, capm);
        c_um[c] = __builtin_bit_cast(int64_t, avm);
        c_iv[c] = make_float2((float)(100.0 / capc), (float)(100.0 / capm));
      } else {
        c_ac[c] = in ? ac : 0;
        c_uc[c] = uc;
        c_am[c] = in ? am : 0;
        c_um[c] = um;
      }
      c_ns[c] = in ? ldg(a->s.nsne, cl) : 0;
      c_gv[c] = in ? ldg(a->s.gvk, cl) : 0;
      if (c_ne) c_ne[c] = in ? ldg(a->s.ne, cl) : 0;
      if (c_pn) c_pn[c] = in ? ldg(a->s.pns, cl) : 0;
    }
    __syncthreads();
  }
  constexpr int NR = NCH > 0 ? NCH : 1;

  // UnitRecs and static filter words of a batch of up to 8 units, loaded
  // with two vector loads at the batch start into VGPRs (record dword d of
  // batch unit u in lane 16*(u&3)+d of rvA/rvB; filter word ch of unit u in
  // lanes 2*(u*nch+ch)+{0,1} of svv) and read per unit with v_readlane: no
  // scalar or vector memory round trip per unit (an SMEM load would be
  // waited by the next LDS wait; a vector load by the last unit's stores).
  // Units are dequeued in batches of LEAN_BATCH from the work heads (WorkTicket: one returning atomicAdd
  // per batch, resolved one batch later); the grid is the resident wave count (launch_schedule) and
  // every wave runs until all heads are drained, so no wave idles on a static share while others work.
  const UnitRec* recs = largs()->b.rec;
  const uint64_t* sws = largs()->b.sw;
  uint32_t* heads = largs()->b.wq;
  WorkTicket tk = wq_start((int)(blockDim.x >> 6), largs()->units_per_wave);
#ifdef KAD_PHASE_PROF
  const unsigned long long wt_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz, device-wide
#endif
  // the next batch's records are loaded one batch ahead (nrvA/nsvv): the
  // wait at a batch start then only covers the previous unit's stores
  uint32_t rvA = 0, svv = ~0u, nrvA = 0, nsvv = ~0u;
  auto fetch = [&](int wb, int nb) {
    nrvA = lane < nb * 16 ? ldg((const uint32_t*)(recs + wb), (uint32_t)lane) : 0u;
    if (NCH > 0 && f_sw) nsvv = lane < nb * 2 * nch ? ldg((const uint32_t*)(sws + (size_t)wb * nch), (uint32_t)lane) : ~0u;
  };
  int2 cb = wq_resolve(heads, W, tk);  // the static first batch; then the ticket of the one after
  if (cb.y > 0) {
    wq_issue(heads, tk);
    fetch(cb.x, cb.y);
  }
  int w = -1, bend = 0, u = 0;
  KAD_PACC;
  for (;;) {
    ++w;
    ++u;
    if (w >= bend) {  // next batch
      if (cb.y <= 0) break;
      w = cb.x;
      bend = cb.x + cb.y;
      u = 0;
      rvA = nrvA;
      svv = nsvv;
      cb = wq_resolve(heads, W, tk);
      if (cb.y > 0) {
        wq_issue(heads, tk);
        fetch(cb.x, cb.y);
      }
    }
    KAD_PT(t0);
    auto fld = [&](int d) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)rvA, (u << 4) + d); };
    auto fld64 = [&](int d) -> int64_t { return (int64_t)(((uint64_t)fld(d + 1) << 32) | fld(d)); };
    const uint32_t fc = fld(0);
    const int gvc = (int)fld(1);
    const int tsc = (int)fld(2);
    const int64_t rqc = fld64(4), rqm = fld64(6);
    const uint64_t tolc = (uint64_t)fld64(12);
    uint64_t swc[NR];
#pragma unroll
    for (int ch = 0; ch < NR; ++ch) {
      const int l = 2 * (u * nch + ch);
      swc[ch] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)svv, l + 1) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)svv, l);
    }
    if (fc & KAD_W_STICKY) {  // generic_scheduler.go:101-104
      lean_status(w, KAD_ST_STICKY);
      continue;
    }
    if ((fc & REC_FULL) ||
        (clean && ((uint64_t)rqc >= (1ull << 46) || (uint64_t)rqm >= (1ull << 46) || (fc & KAD_W_WIDE_SCORES)))) {
      lean_defer(w);  // (requests outside [0, 2^46) and wide weights set the host's batch_defer)
      continue;
    }
    const double rqcd = (double)rqc, rqmd = (double)rqm;  // exact on the clean path
    const int spo = (int)fld(3);
    const int64_t mc = fld64(8), ooff = fld64(10);
    const uint64_t tolp0 = (uint64_t)fld64(14);
    const bool use_cur = f_taint && (fc & KAD_W_HAS_CURRENT);
    const bool fit_on = f_fit && (fc & KAD_W_FIT_NONZERO);
    const uint64_t o_sw = 0ull, o_taint = f_taint ? 0ull : ~0ull, o_fit = fit_on ? 0ull : ~0ull;
    const uint64_t o_api = f_api ? 0ull : ~0ull, a_api = gvc >= 0 ? ~0ull : 0ull;  // no GVK id: no cluster has it
    const double fcpu = fit_on ? rqcd : -1.0, fmem = fit_on ? rqmd : -1.0;  // clean fit compare operands
    uint64_t dsw = ~0ull, dcw = 0;  // dynamic-NCH path: words of chunks 64g..64g+63 in lanes
    auto load_words = [&](int ch0) {
      LArgs a = largs();
      const int ch = ch0 + lane;
      dsw = (f_sw && ch < nch) ? ldg(a->b.sw, (uint32_t)(w * nch + ch)) : ~0ull;
      dcw = (use_cur && ch < nch) ? ldg(a->b.cw, (uint32_t)(w * nch + ch)) : 0ull;
    };
    if constexpr (NCH == 0) load_words(0);
    // (NCH == 0, every filter in the static words: the words of chunks 64..191 load in the same round trip)
    uint64_t dsw1 = 0, dsw2 = 0;
    if constexpr (NCH == 0) {
      if (fold && fitf && f_sw && nch > WAVE) {
        LArgs a = largs();
        const int c1 = WAVE + lane, c2 = 2 * WAVE + lane;
        dsw1 = ldg(a->b.sw, (uint32_t)(w * nch + (c1 < nch ? c1 : nch - 1)));
        dsw2 = ldg(a->b.sw, (uint32_t)(w * nch + (c2 < nch ? c2 : nch - 1)));
      }
    }

    // ---------------- filters → compacted feasible list (findClustersThatFitWorkload, :152-169)
    int n = 0;
    uint64_t mk[NR];
    const int NC = NCH > 0 ? NCH : nch;
    // NCH == 0 (no LDS cache): the attributes of chunk ch+1 are loaded while
    // chunk ch is filtered (software pipeline; one exposed round trip per unit)
    int64_t p_ac = 0, p_uc = 0, p_am = 0, p_um = 0;
    uint64_t p_ns = 0, p_ne = 0, p_gv = 0;
    // NCH == 0: the attributes of chunk cn (lanes = its clusters) that the mode's filters read: none
    // when every filter is in the static words (FITF), the resources only with FOLD
    auto load_attrs = [&](auto mode_t, int cn) {
      constexpr int MODE = decltype(mode_t)::value;
      if constexpr (MODE != 3) {
        LArgs a = largs();
        const uint32_t cl = cn < C ? (uint32_t)cn : 0u;
        p_ac = ldg(a->s.alloc_cpu, cl);
        p_uc = ldg(a->s.used_cpu, cl);
        p_am = ldg(a->s.alloc_mem, cl);
        p_um = ldg(a->s.used_mem, cl);
        if constexpr (MODE < 2) {
          p_ns = ldg(a->s.nsne, cl);
          p_ne = ldg(a->s.ne, cl);
          p_gv = ldg(a->s.gvk, cl);
        }
      }
    };
    // the chunk loop twice: FAST (no CurrentClusters, one taint word) has no
    // uniform branch inside, so the cache reads of every chunk issue together
    // MODE 2 (FOLD): taint and API filters already in the static words (prep_kernel, SnapDev::fold);
    // 1 (FAST): one taint word, no CurrentClusters; 0: general
    auto filter_chunks = [&](auto mode_t) {
      constexpr int MODE = decltype(mode_t)::value;
      constexpr bool FAST = MODE >= 1, FOLD = MODE >= 2, FITF = MODE == 3;
      if constexpr (NCH == 0 && FITF) {
        // every filter is in the static words: only the non-zero words of each 64-chunk group (one per
        // lane) are compacted — C5's median unit has 2 feasible clusters of 10 000
        for (int g = 0; g < nch; g += WAVE) {
          if (g == WAVE) dsw = f_sw ? dsw1 : ~0ull;
          else if (g == 2 * WAVE) dsw = f_sw ? dsw2 : ~0ull;
          else if (g > 0) load_words(g);
          uint64_t nz = ballot(g + lane < nch && dsw != 0);
          while (nz) {
            const int l = __builtin_ctzll(nz);
            nz &= nz - 1;
            const uint64_t m = readlane64(dsw, l);
            if (lane_on(m)) {
              const int pos = n + mbcnt(m);
              if (pos < P) idx[pos] = (uint16_t)((g + l) * WAVE + lane);  // more than P: deferred
            }
            n += popc64(m);
            if (n > P) return;
          }
        }
        return;
      }
      const bool ucur = !FAST && use_cur;
      if constexpr (NCH == 0) load_attrs(mode_t, lane);
#pragma unroll
      for (int ch = 0; ch < NC; ++ch) {
        const int c = ch * WAVE + lane;
        int64_t acpu, ucpu, amem, umem;
        uint64_t ns0, ne0, pn0, gv0, sw0, cw0;
        if constexpr (NCH > 0) {
          acpu = (clean || FITF) ? 0 : c_ac[c];
          ucpu = FITF ? 0 : c_uc[c];  // clean: available cpu as f64
          amem = (clean || FITF) ? 0 : c_am[c];
          umem = FITF ? 0 : c_um[c];
          ns0 = FOLD ? 0ull : c_ns[c];
          ne0 = ucur ? c_ne[c] : 0ull;
          pn0 = 0;
          gv0 = FOLD ? 0ull : c_gv[c];
          sw0 = swc[ch];
          cw0 = ucur ? ldc(largs()->b.cw + (size_t)w * nch + ch) : 0ull;
        } else {
          acpu = p_ac;
          ucpu = p_uc;
          amem = p_am;
          umem = p_um;
          ns0 = p_ns;
          ne0 = p_ne;
          gv0 = p_gv;
          pn0 = 0;
          if (ch + 1 < NC) load_attrs(mode_t, c + WAVE);
          if (ch > 0 && (ch & 63) == 0) load_words(ch);
          sw0 = readlane64(dsw, ch & 63);
          cw0 = readlane64(dcw, ch & 63);
        }
        // each filter as a lane mask (v_cmp → SGPR pair), combined with scalar
        // ANDs under uniform selects (no branches inside the unrolled loop)
        uint64_t m = ~0ull;  // lanes past C: cleared in the static word
        const bool sch = ucur && ((cw0 >> lane) & 1);
        const uint64_t x = sch ? ne0 : ns0;
        bool tok = (x & ~tolc) == 0;
        for (int tw = 1; tw < (FAST ? 1 : TWs); ++tw) {  // more than 64 taint ids (C5): words 1.. from global
          LArgs a = largs();
          const uint32_t cl = c < C ? (uint32_t)c : 0u;
          const uint64_t xt = sch ? ldg(a->s.ne, (uint32_t)(tw * C) + cl) : ldg(a->s.nsne, (uint32_t)(tw * C) + cl);
          tok &= (xt & ~ldc(a->b.tol_all + (size_t)tsc * TWs + tw)) == 0;
        }
        // fit.go:73-134: alloc >= req + used (clean: available - req >= 0, exact in f64; with the filter
        // off the compare is against -1, true everywhere)
        const uint64_t m_fit = FITF    ? ~0ull  // in the static words (SnapDev::fitfold)
                               : clean ? ballot(__builtin_bit_cast(double, ucpu) >= fcpu) & ballot(__builtin_bit_cast(double, umem) >= fmem)
                                       : ballot((acpu >= wadd(rqc, ucpu)) & (amem >= wadd(rqm, umem)));
        if constexpr (FOLD) {
          (void)tok;
          m &= sw0 & (clean ? m_fit : (m_fit | o_fit));
        } else {
          const uint64_t m_taint = ballot(tok);      // taint_toleration.go:50-77
          const uint64_t m_api = ballot((gv0 >> (gvc & 63)) & 1);  // apiresources.go:25-43
          // disabled filters OR in an all-ones mask (per-unit constants: two SALU ops per filter)
          m &= (sw0 | o_sw) & (m_taint | o_taint) & ((m_api & a_api) | o_api) & (m_fit | o_fit);
        }
        (void)pn0;
        if constexpr (NCH > 0) {
          mk[ch] = m;  // compaction after every chunk's mask: no LDS store between the cache reads
        } else {
          if ((m >> lane) & 1) {
            const int pos = n + mbcnt(m);
            if (pos < P) idx[pos] = (uint16_t)c;  // more than P feasible: the unit is deferred
          }
          n += popc64(m);
          if (n > P) break;  // deferred whatever the remaining chunks hold
        }
      }
    };
    if (fold && fitf)
      filter_chunks(std::integral_constant<int, 3>{});
    else if (fold)
      filter_chunks(std::integral_constant<int, 2>{});
    else if (!use_cur && TWs == 1)
      filter_chunks(std::integral_constant<int, 1>{});
    else
      filter_chunks(std::integral_constant<int, 0>{});
    if constexpr (NCH > 0) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        // every lane stores (no exec branch): infeasible lanes into pid[], rewritten before use
        idx[lane_on(mk[ch]) ? n + mbcnt(mk[ch]) : P + lane] = (uint16_t)(ch * WAVE + lane);
        n += popc64(mk[ch]);
      }
    }
    KAD_PT(t1);
    KAD_PADD(0, t1 - t0);
    if (n == 0) {  // generic_scheduler.go:112-114
      lean_status(w, KAD_ST_NO_FEASIBLE);
      continue;
    }
    if (NCH == 0 && n > P) {  // more feasible clusters than registers: the row kernel (or the full kernel)
      lean_row_or_defer(w);
      continue;
    }
    if ((sm & BIT(KAD_PL_CLUSTER_AFFINITY)) && (fc & KAD_W_SCORE_ERROR)) {  // framework.go:149-159
      lean_status(w, KAD_ST_ERR_SCORE);
      continue;
    }
    wave_sync();

    // ---------------- scores of positions 64q + lane (RunScorePlugins, framework.go:139-181)
    const int nq = (n + 63) >> 6;
    TT t[Q];
    uint32_t cid[Q];
    int ttv[Q];
    int ttmax = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      t[q] = 0;
      cid[q] = 0;
      ttv[q] = 0;
      if (q >= nq) continue;
      const int p = q * 64 + lane;
      const bool v = p < n;
      cid[q] = v ? idx[p] : 0u;
      const uint32_t cq = cid[q];
      if (s_res && clean) {
        // x = cap - req = available - request (exact); req > cap <=> x < 0 (score 0)
        const double capc = __builtin_bit_cast(double, c_ac[cq]), capm = __builtin_bit_cast(double, c_am[cq]);
        const double xc = __builtin_bit_cast(double, c_uc[cq]) - rqcd, xm = __builtin_bit_cast(double, c_um[cq]) - rqmd;
        const float2 iv = c_iv[cq];
        // branch-free: quotients of max(x, 0) (= 0 when x <= 0), masked to 0 where req > cap
        const double xcp = fmax(xc, 0.0), xmp = fmax(xm, 0.0);
        const int okc = -(int)(xc >= 0.0), okm = -(int)(xm >= 0.0);
        int x = 0;
        if (sm & BIT(KAD_PL_LEAST_ALLOCATED)) x += (quot100(xcp, capc, iv.x) + quot100(xmp, capm, iv.y)) >> 1;
        if (sm & BIT(KAD_PL_MOST_ALLOCATED))
          x += ((quot100(capc - xcp, capc, iv.x) & okc) + (quot100(capm - xmp, capm, iv.y) & okm)) >> 1;
        if (sm & BIT(KAD_PL_BALANCED_ALLOCATION)) x += (int)balanced_d((capc - xc) / capc, (capm - xm) / capm);
        t[q] = (TT)x;
      } else if (s_res) {
        int64_t cc, cm, uc, um;
        if constexpr (NCH > 0) {
          cc = c_ac[cq];
          cm = c_am[cq];
          uc = c_uc[cq];
          um = c_um[cq];
        } else {
          LArgs a = largs();
          cc = ldg(a->s.alloc_cpu, cq);
          cm = ldg(a->s.alloc_mem, cq);
          uc = ldg(a->s.used_cpu, cq);
          um = ldg(a->s.used_mem, cq);
        }
        if (!v) {
          cc = cm = 1;
          uc = um = 0;
        }
        const int64_t rc = wadd(uc, rqc), rm = wadd(um, rqm);
        int64_t x = 0;
        if (sm & BIT(KAD_PL_LEAST_ALLOCATED))
          x = wadd(x, go_div(wadd(least_requested(rm, cm), least_requested(rc, cc)), 2));
        if (sm & BIT(KAD_PL_MOST_ALLOCATED))
          x = wadd(x, go_div(wadd(most_requested(rm, cm), most_requested(rc, cc)), 2));
        if (sm & BIT(KAD_PL_BALANCED_ALLOCATION)) x = wadd(x, balanced(rc, cc, rm, cm));
        t[q] = x;
      }
      if (s_tt) {  // taint_toleration.go:91-118: PreferNoSchedule taints not tolerated
        uint64_t pn;
        if constexpr (NCH > 0)
          pn = c_pn[cq];
        else
          pn = ldg(largs()->s.pns, cq);
        int tc = popc64(pn & ~tolp0);
        for (int tw = 1; tw < TWs; ++tw) {
          LArgs a = largs();
          tc += popc64(ldg(a->s.pns, (uint32_t)(tw * C) + cq) & ~ldc(a->b.tol_pns + (size_t)tsc * TWs + tw));
        }
        ttv[q] = v ? tc : 0;
        ttmax = ttv[q] > ttmax ? ttv[q] : ttmax;
      }
    }
    if (s_tt) {  // DefaultNormalizeScore(100, reverse=true), framework/util.go:455-483
      ttmax = wave_max_u_i32(ttmax);
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (q < nq) t[q] = tadd(t[q], ttmax == 0 ? 100 : 100 - (int64_t)small_quot(100 * ttv[q], ttmax));
    }
    if (sm & BIT(KAD_PL_CLUSTER_AFFINITY)) {  // cluster_affinity.go:96-140 + DefaultNormalizeScore(100, false)
      LArgs a = largs();
      const int32_t* sp = a->b.sprog + spo;
      const uint32_t pv = ldg((const uint32_t*)sp, (uint32_t)lane);  // program words 0..63 (slack past the blob)
      if (__builtin_amdgcn_readfirstlane((int)pv) > 0) {  // units without preferred terms score 0 everywhere
        TT afs[Q];  // CL: |raw| <= sum |weight| <= 2^20 (wider units are deferred)
        TT amax = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          afs[q] = 0;
          if (q < nq && q * 64 + lane < n) afs[q] = (TT)affinity_score_pv(a->b.req_mask, pv, sp, nch, (int)cid[q]);
          amax = afs[q] > amax ? afs[q] : amax;
        }
        if constexpr (CL) {
          amax = wave_max_u_i32(amax);
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (q < nq) {
              const int num = 100 * afs[q];
              t[q] += amax == 0 ? afs[q] : (num >= 0 && num < (1 << 24) ? (int)small_quot(num, amax) : num / amax);
            }
        } else {
          amax = wave_max_u_i64(amax);
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (q < nq) t[q] = wadd(t[q], amax == 0 ? afs[q] : div_fast(wmul(100, afs[q]), amax));
        }
      }
    }
    KAD_PT(t2);
    KAD_PADD(1, t2 - t1);

    // ---------------- select (framework.go:183-209, max_cluster.go:42-66)
    LArgs ad = largs();
    int k = n;  // <= n <= 64 * Q: 32-bit counts
    if (ad->p.select_plugin == KAD_PL_MAX_CLUSTER) {
      const bool hm = fc & KAD_W_HAS_MAX_CLUSTERS;
      if (hm && mc < 0) {
        lean_status(w, KAD_ST_ERR_SELECT);
        continue;
      }
      if (hm && mc < k) k = (int)mc;
    }
    uint64_t sel[Q];
    uint32_t rflags = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) sel[q] = 0;
    if (k >= n) {
#pragma unroll
      for (int q = 0; q < Q; ++q) sel[q] = ballot(q * 64 + lane < n);
    } else if (k > 0) {
      // lanes holding a total, per position chunk
      uint64_t vm[Q];
      TT mn = CL ? (TT)INT32_MAX : (TT)I64_MAX, mx = CL ? (TT)INT32_MIN : (TT)I64_MIN;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int r = n - q * 64;
        vm[q] = q < nq ? (r >= 64 ? ~0ull : ((1ull << r) - 1)) : 0ull;
        const bool vq = lane_on(vm[q]);
        mn = (vq && t[q] < mn) ? t[q] : mn;
        mx = (vq && t[q] > mx) ? t[q] : mx;
      }
      // k-th largest total T: the largest T with #(total >= T) >= k, by
      // bisection over [min, max] — in 32 bits when every total fits (the
      // usual case: totals are sums of 0..100 plugin scores)
      const bool hv = lane < n;
      int64_t rmin, rmax, lo;
      if (!ballot(hv && (mn < INT32_MIN || mx > INT32_MAX))) {
        int mn32, mx32;
        wave_minmax_u_i32(hv ? (int)mn : INT32_MAX, hv ? (int)mx : INT32_MIN, mn32, mx32);
        int t32[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) t32[q] = (int)t[q];
        int lo32 = mn32, hi32 = mx32;
        if (Q >= 2 && (uint32_t)mx32 - (uint32_t)mn32 < 128u) {
          // totals within 128 of each other (the usual case: sums of 0..100
          // plugin scores): LDS histogram in descending bin order, one
          // prefix sum over the wave, the k-th largest from one ballot —
          // instead of a ballot-count bisection step per bit of the range
          uint32_t* hist = key;  // 128 u32; the replay rewrites key[] afterwards
          *(uint2*)(hist + 2 * lane) = make_uint2(0u, 0u);
          wave_sync();
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (q < nq) {  // exec-free: lanes past n add 0 to bin `lane` (not all to one bin)
              const bool vq = lane_on(vm[q]);
              atomicAdd(hist + (vq ? 127 - (t32[q] - mn32) : lane), vq ? 1u : 0u);
            }
          wave_sync();
          const uint2 hh = *(const uint2*)(hist + 2 * lane);  // bins 127-2l, 126-2l
          const int pre = wave_incl_sum_i32((int)(hh.x + hh.y));  // #(total >= mn + 126 - 2l)
          const int kk = (int)k;
          const int l0 = (int)__builtin_ctzll(ballot(pre >= kk));
          const int pl = __builtin_amdgcn_readlane(pre, l0);
          const int h1 = __builtin_amdgcn_readlane((int)hh.y, l0);
          lo32 = mn32 + (pl - h1 >= kk ? 127 - 2 * l0 : 126 - 2 * l0);
          hi32 = lo32;
          wave_sync();
        }
        if (nq == 1) {  // one position per lane: one ballot per step
          while (lo32 < hi32) {
            const uint32_t d = (uint32_t)hi32 - (uint32_t)lo32;
            const int mid = (int)((uint32_t)lo32 + (d >> 1) + (d & 1));
            if (popc64(ballot(t32[0] >= mid) & vm[0]) >= k)
              lo32 = mid;
            else
              hi32 = mid - 1;
          }
        } else {
          while (lo32 < hi32) {
            const uint32_t d = (uint32_t)hi32 - (uint32_t)lo32;
            const int mid = (int)((uint32_t)lo32 + (d >> 1) + (d & 1));
            int cnt = 0;
#pragma unroll
            for (int q = 0; q < Q; ++q)
              if (q < nq) cnt += popc64(ballot(t32[q] >= mid) & vm[q]);
            if (cnt >= k)
              lo32 = mid;
            else
              hi32 = mid - 1;
          }
        }
        rmin = mn32;
        rmax = mx32;
        lo = lo32;
      } else {
        rmin = wave_min_u_i64(mn);
        rmax = wave_max_u_i64(mx);
        lo = rmin;
        int64_t hi = rmax;
        while (lo < hi) {
          const uint64_t d = (uint64_t)hi - (uint64_t)lo;
          const int64_t mid = (int64_t)((uint64_t)lo + (d >> 1) + (d & 1));
          int64_t cnt = 0;
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (q < nq) cnt += popc64(ballot(t[q] >= mid) & vm[q]);
          if (cnt >= k)
            lo = mid;
          else
            hi = (int64_t)((uint64_t)mid - 1);
        }
      }
      uint64_t gm[Q], em[Q];
      int g = 0, e = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        gm[q] = ballot(t[q] > lo) & vm[q];
        em[q] = ballot(t[q] == lo) & vm[q];
        g += popc64(gm[q]);
        e += popc64(em[q]);
      }
      const int need = k - g;
      if (need == e) {  // the cut takes every tie: no sort needed
#pragma unroll
        for (int q = 0; q < Q; ++q) sel[q] = gm[q] | em[q];
      } else {
        rflags = KAD_RF_TIE_STRADDLE;
        const int xs_b = (ad->p.flags & KAD_PROFILE_XORSHIFT_GO121) ? 7 : 17;
        const int xs_c = (ad->p.flags & KAD_PROFILE_XORSHIFT_GO121) ? 17 : 5;
        if (n <= 12) {  // pdqsort_func: a single (stable) insertionSort
          sel[0] = gm[0] | ballot(lane < n && t[0] == lo && mbcnt(em[0]) < need);
        } else {
          // restricted pdqsort replay, wave-parallel (kad_select.h PdqWave), on
          // u32 keys t - min (order-preserving); rows spanning >= 2^32 go to schedule_kernel
          if ((uint64_t)rmax - (uint64_t)rmin > 0xFFFFFFFFull) {
            lean_defer(w);
            continue;
          }
          if ((uint64_t)rmax - (uint64_t)rmin < 65536u) {  // packed replay: key << 16 | position
#pragma unroll
            for (int q = 0; q < Q; ++q)
              if (q < nq && q * 64 + lane < n)
                key[q * 64 + lane] = ((uint32_t)((uint64_t)t[q] - (uint64_t)rmin) << 16) | (uint32_t)(q * 64 + lane);
            wave_sync();
            PdqWaveP<> pw{key, posl, posr, xs_b, xs_c};
            pw.select(n, (int)k);
            for (int r = lane; r < n; r += WAVE) inv[key[r] & 0xFFFFu] = (uint16_t)r;
          } else {
#pragma unroll
            for (int q = 0; q < Q; ++q)
              if (q < nq && q * 64 + lane < n) {
                key[q * 64 + lane] = (uint32_t)((uint64_t)t[q] - (uint64_t)rmin);
                pid[q * 64 + lane] = (uint16_t)(q * 64 + lane);
              }
            wave_sync();
            PdqWave<uint32_t> pw{key, pid, posl, posr, xs_b, xs_c};
            pw.select(n, (int)k);
            for (int r = lane; r < n; r += WAVE) inv[pid[r]] = (uint16_t)r;
          }
          wave_sync();
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (q < nq) {
              const int p = q * 64 + lane;
              sel[q] = ballot(p < n && inv[p] < k);
            }
        }
      }
    }
    KAD_PT(t3);
    KAD_PADD(2, t3 - t2);
    if (rflags) {
      KAD_PADD(4, 1);
      KAD_PADD(5, t3 - t2);
    }

    // ---------------- output, ascending cluster id (= ascending position)
    {
      LArgs ae = largs();
      const bool dup = fc & KAD_W_DUPLICATE;
      const bool replicas =
          !dup && ae->p.replicas_plugin == KAD_PL_CLUSTER_CAPACITY_WEIGHT && (fc & REC_DESIRED_POS) && k > 0;
      int base = 0;
      if (dup || replicas) {
        int32_t* oc = ae->o.cluster + ooff;
        int64_t* orp = ae->o.replicas + ooff;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          if ((sel[q] >> lane) & 1) {
            const uint32_t at = (uint32_t)(base + mbcnt(sel[q]));
            stg(oc, at, (int32_t)cid[q]);
            stg(orp, at, (int64_t)(dup ? -1 : 0));
          }
          base += popc64(sel[q]);
        }
      }
      if (lane == 0) {
        ae->o.status[w] = KAD_ST_OK;
        ae->o.count[w] = base;  // Divide without replicas plugin: empty map
        ae->o.flags[w] = rflags;
      }
    }
    wave_sync();
    KAD_PT(t4);
    KAD_PADD(3, t4 - t3);
  }
#ifdef KAD_PHASE_PROF
  {
    const int gwv = blockIdx.x * (int)(blockDim.x >> 6) + wv;
    if (lane == 0 && gwv < 8192) {
      g_wavetime[2 * gwv] = wt_start;
      g_wavetime[2 * gwv + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
#endif
  KAD_PFLUSH_LEAN;
}

// ================================================== wide schedule kernel
// schedule_wide_kernel<NCH> — 256 < C <= 64*NCH (C3: 1 000 clusters, 16
// chunks) on a clean snapshot. The lean kernel's register-resident positions
// do not scale to feasible lists of several hundred clusters (C3: 20 % of the
// units have n > 256), so here:
//   * one 1024-thread workgroup per CU (persistent grid = #CUs): ONE block-
//     shared LDS copy of the cluster attributes (C = 1000: ~56 KB) serves 16
//     waves, and each wave's region (positions, replay scratch: 6 KB at
//     P = 512) fits beside it in the 160 KB LDS;
//   * units are dequeued dynamically: 8 work heads (one per contiguous eighth
//     of the batch, a wave starts at head blockIdx % 8 — the round-robin XCD
//     of its block, for locality only) hand out WQ_BATCH units per returning
//     atomicAdd, one batch ahead of use; an exhausted head sends the wave to
//     the next one, so every wave runs until the whole batch is drained (no
//     static-share tail);
//   * each unit's 64-B record and static filter words arrive in ONE VGPR,
//     loaded one unit ahead (lanes 0-15: UnitRec, lanes 16..16+2*nch: sw);
//   * filter per 64-cluster chunk: two ds_read_b128 (available cpu/mem as
//     exact f64; NS|NE taint word + GVK word) → lane masks ANDed in SALU →
//     compaction into the wave's position list (u16 cluster ids);
//   * scores and totals for positions 64q + lane (q < WIDE_Q) in registers,
//     normalisation by DPP wave max; MaxCluster's k-th largest total by LDS
//     histogram (span < 128) or ballot bisection; the same tie rules as the
//     lean kernel (all ties / n <= 12 insertionSort / PdqWave replay).
// Units with more than WIDE_P feasible clusters, REC_FULL units and requests
// outside the exact-f64 range go to the defer list (schedule_kernel).
constexpr int WIDE_MAX_NCH = 16;
constexpr int WIDE_THREADS = 1024;
#ifndef KAD_DUMMY_STRIDE
#define KAD_DUMMY_STRIDE 1  // u16 dummy slots of the wide kernel's compaction: P + stride * lane (<= 2: inside idx / pid)
#endif
#ifndef KAD_WIDE_ZS
#define KAD_WIDE_ZS 1  // the wide kernel's per-cluster zero-request resource scores (c_zs)
#endif
#ifndef KAD_WIDE_C8
#define KAD_WIDE_C8 0  // compaction at exactly 8 chunks: 0 chunk loop, 1 8-cluster lane pieces, 2 16-cluster pieces
#endif
// the row path's body (defined with schedule_row_kernel below), run by the wide kernel's opening phase
template <int SM, int NT, class ArgsOf>
__device__ __forceinline__ void row_units(ArgsOf args, char* smem, int rexp);
// the wide kernel's row phase as a separate (not inlined) function: its register demand stays out of the
// unit loop's allocation
template <int SM>
__device__ __attribute__((noinline)) void wide_rows(char* smem, const __attribute__((address_space(4))) struct WideArgs* a);

struct WideLayout {
  size_t key, idx, pid, posl, posr, bytes;
};
__host__ __device__ inline WideLayout wide_layout() {
  WideLayout L;
  L.key = 0;                      // u32[P] replay keys / histogram
  L.idx = L.key + 4 * WIDE_P;     // u16[P] position -> cluster id
  L.posl = L.idx;                 // u16[P + 64] replay scratch, then ranks (idx is dead by then: the
                                  // cluster ids are in registers)
  L.pid = L.idx + 2 * WIDE_P + 128;  // u16[P] replay: original position
  L.posr = L.pid + 2 * WIDE_P;    // u16[P]
  L.bytes = L.posr + 2 * WIDE_P;
  return L;
}
// the compaction stores every feasible cluster's id at its position, even past P (up to 64*nch):
// those land in pid / posr of the same wave's region and the unit is deferred
static_assert(2 * 64 * WIDE_MAX_NCH <= 6 * WIDE_P, "idx overflow past P must stay in the wave's region");
// block-shared cluster cache: av (f64 x2), tg (u64 x2: NS|NE taints, GVK word),
// cap (f64 x2), iv (f32 x2), [ne u64], [pn u64]
__host__ __device__ inline size_t wide_cache_bytes(int C, int cache_ne, int cache_pn, int cache_zs = 0) {
  const size_t Cp = (size_t)((C + 63) & ~63);
  return Cp * (16 + 16 + 16 + 8 + 8 * cache_ne + 8 * cache_pn + 4 * cache_zs);
}

struct WideArgs {
  SnapDev s;
  BatchDev b;
  OutDev o;
  ProfDev p;
  int waves_per_block;
  int cache_ne, cache_pn;
  int cache_zs;     // the resource scores of a zero request per cluster (c_zs, below)
  int rows_inline;  // the units prep_kernel routed to rows run in this kernel's opening phase (row_units)
  int batch;        // units per work-queue batch (launch_schedule: by units per wave)
  int exp;  // measurement-only variants (KAD_WIDE_EXPERIMENT, never set by default; results differ from
            // the reference): bit 0 skips the pdqsort replay (ties taken by position), bit 1 ends each unit
            // after the filters, bit 2 after the scores (no selection), bit 3 skips the output pass
};
typedef const __attribute__((address_space(4))) WideArgs* WArgs;
__device__ __forceinline__ WArgs wargs() {
  return (WArgs)opq((uintptr_t)__builtin_amdgcn_kernarg_segment_ptr());
}
// experiment bits: compiled out of product builds
#if defined(KAD_PHASE_PROF) || defined(KAD_TUNING)
#define WIDE_EXP(bits) ((wargs()->exp & (bits)) != 0)
#else
#define WIDE_EXP(bits) false
#endif

__device__ __forceinline__ void wide_status(int w, int32_t st) {
  if (lane_id() == 0) {
    WArgs a = wargs();
    a->o.status[w] = st;
    a->o.count[w] = 0;
    a->o.flags[w] = 0;
  }
}
__device__ __forceinline__ void wide_defer(int w) {
  if (lane_id() == 0) {
    WArgs a = wargs();
    const int slot = atomicAdd(a->b.defer_n, 1);
    a->b.defer[slot] = w;
  }
}

__device__ __forceinline__ void wide_row_or_defer(int w) {
  if (lane_id() == 0) {
    WArgs a = wargs();
    if (a->b.use_rows && !a->b.early_rows) {  // (early_rows: the row kernel may already be done)
      const int slot = atomicAdd(a->b.rows_n, 1);
      a->b.rows[slot] = w;
    } else {
      const int slot = atomicAdd(a->b.defer_n, 1);
      a->b.defer[slot] = w;
    }
  }
}

// XN > 0: the kernel is specialised for exactly XN chunks; SM >= 0: for the score-plugin mask SM (the
// profile's plugins as compile-time constants: every runtime plugin test of the hot loops folds away, and
// with it the 64-bit condition masks the compiler otherwise keeps live — and spills — across the loop)
// ZR: every unit of the batch has a zero ResourceRequest (BatchDev::zero_req): the resource scores are the
// per-cluster column c_zs. (A per-unit test inside the one instantiation cost C3's units, which all carry
// requests, 31 us of 1.13 ms for the zero-request units' 24 us: profiles/r06/ab_c3_zero_request_kernel.txt)
template <int NCH, int XN, int SM, bool ZR = false>
__global__ __launch_bounds__(WIDE_THREADS, 4) void schedule_wide_kernel(WideArgs args) {
  (void)args;  // read through wargs()
  constexpr int Q = WIDE_Q;
  constexpr int P = WIDE_P;
  static_assert(XN <= NCH, "exact chunk count within the template bound");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the units prep_kernel routed to the row path (more than P feasible clusters, BatchDev::early_rows):
  // the first blocks take them, one unit per block at a time, before their own work queue — in the LDS
  // of the waves' regions (the cluster cache above is loaded afterwards); the queue's dynamic batches
  // absorb the delay of these blocks' static first batches. First in the kernel, so that nothing of the
  // unit loop is live across the row body (its register pressure does not spill the loop's values).
  if (wargs()->rows_inline) {
    const int rn = __hip_atomic_load(wargs()->b.rows_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int)blockIdx.x < rn) {
      wide_rows<SM>(smem, wargs());  // (a callee cannot read the kernarg segment pointer itself: pass it)
      __syncthreads();  // the row body's LDS reads are done before the waves' regions are reused
    }
  }
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int C, W, TWs;
  uint32_t fm, sm;
  {
    WArgs a = wargs();
    C = a->s.C;
    TWs = a->s.TW;
    W = a->b.W;
    fm = a->p.filter_mask;
    sm = SM >= 0 ? (uint32_t)SM : a->p.score_mask;
  }
  const int nch = XN > 0 ? XN : (C + 63) >> 6;
  const int Cp = nch * 64;
  const WideLayout L = wide_layout();
  const int nwaves = blockDim.x >> 6;
  char* region = smem + (size_t)wv * L.bytes;
  uint32_t* key = (uint32_t*)(region + L.key);
  uint16_t* idx = (uint16_t*)(region + L.idx);
  uint16_t* pid = (uint16_t*)(region + L.pid);
  uint16_t* posl = (uint16_t*)(region + L.posl);
  uint16_t* posr = (uint16_t*)(region + L.posr);
  uint16_t* inv = posl;
  char* cache = smem + (size_t)nwaves * L.bytes;
  double2* c_av = (double2*)cache;
  ulonglong2* c_tg = (ulonglong2*)(cache + (size_t)16 * Cp);
  double2* c_cap = (double2*)(cache + (size_t)32 * Cp);
  float2* c_iv = (float2*)(cache + (size_t)48 * Cp);
  uint64_t* c_ne = nullptr;
  uint64_t* c_pn = nullptr;
  // the sum of the profile's resource scores for a ZERO request per cluster: the live controller never sets
  // ResourceRequest (schedulingtriggers.go:188-191), so Least / Most / Balanced are per-cluster constants
  // there — one LDS read per position instead of the exact-f64 quotients
  int32_t* c_zs = nullptr;
  {
    WArgs a = wargs();
    size_t o = (size_t)56 * Cp;
    if (a->cache_ne) {
      c_ne = (uint64_t*)(cache + o);
      o += (size_t)8 * Cp;
    }
    if (a->cache_pn) {
      c_pn = (uint64_t*)(cache + o);
      o += (size_t)8 * Cp;
    }
    if (a->cache_zs) c_zs = (int32_t*)(cache + o);
  }
  const bool f_taint = fm & BIT(KAD_PL_TAINT_TOLERATION), f_api = fm & BIT(KAD_PL_API_RESOURCES);
  const bool fold = wargs()->s.fold;  // taint + API filters in the static words (prep_kernel)
  const bool fitf = wargs()->s.fitfold;  // and the cpu / memory fit test
  // the static words are always read: they also clear the last chunk's lanes past C (prep_kernel)
  const bool f_fit = fm & BIT(KAD_PL_CLUSTER_RESOURCES_FIT);
  const bool s_res =
      sm & (BIT(KAD_PL_LEAST_ALLOCATED) | BIT(KAD_PL_MOST_ALLOCATED) | BIT(KAD_PL_BALANCED_ALLOCATION));
  const bool s_tt = sm & BIT(KAD_PL_TAINT_TOLERATION);
  {
    WArgs a = wargs();
    for (int c = threadIdx.x; c < Cp; c += blockDim.x) {
      const bool in = c < C;
      const uint32_t cl = in ? (uint32_t)c : 0u;
      const int64_t ac = in ? ldg(a->s.alloc_cpu, cl) : 1, uc = in ? ldg(a->s.used_cpu, cl) : 0;
      const int64_t am = in ? ldg(a->s.alloc_mem, cl) : 1, um = in ? ldg(a->s.used_mem, cl) : 0;
      double capc, avc, capm, avm;
      score_res(ac, uc, capc, avc);
      score_res(am, um, capm, avm);
      c_av[c] = make_double2(avc, avm);
      c_cap[c] = make_double2(capc, capm);
      const float ivc = (float)(100.0 / capc), ivm = (float)(100.0 / capm);
      c_iv[c] = make_float2(ivc, ivm);
      c_tg[c] = make_ulonglong2(in ? ldg(a->s.nsne, cl) : 0ull, in ? ldg(a->s.gvk, cl) : 0ull);
      if (c_ne) c_ne[c] = in ? ldg(a->s.ne, cl) : 0;
      if (c_pn) c_pn[c] = in ? ldg(a->s.pns, cl) : 0;
      if (c_zs) {  // the score expressions below with request 0: x = available
        const double xcp = fmax(avc, 0.0), xmp = fmax(avm, 0.0);
        const int okc = -(int)(avc >= 0.0), okm = -(int)(avm >= 0.0);
        int x = 0;
        if (sm & BIT(KAD_PL_LEAST_ALLOCATED)) x += (quot100(xcp, capc, ivc) + quot100(xmp, capm, ivm)) >> 1;
        if (sm & BIT(KAD_PL_MOST_ALLOCATED))
          x += ((quot100(capc - xcp, capc, ivc) & okc) + (quot100(capm - xmp, capm, ivm) & okm)) >> 1;
        if (sm & BIT(KAD_PL_BALANCED_ALLOCATION)) x += (int)balanced_d((capc - avc) / capc, (capm - avm) / capm);
        c_zs[c] = x;
      }
    }
    __syncthreads();
  }

  uint32_t* heads;
  const UnitRec* recs;
  const uint64_t* sws;
  {
    WArgs a = wargs();
    heads = a->b.wq;
    recs = a->b.rec;
    sws = a->b.sw;
  }
  WorkTicket tk = wq_start(nwaves, wargs()->batch);
#ifdef KAD_PHASE_PROF
  const unsigned long long wt_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz, device-wide
  unsigned long long wx_units = 0, wx_max = 0, wx_deq = wt_start, wx_str = 0;
#endif
  // one VGPR per unit: lanes 0-15 its UnitRec dwords, lanes 16..16+2*nch its static filter words
  auto fetch = [&](int w) -> uint32_t {
    if (w < 0) return 0u;
    if (lane < 16) return ldg((const uint32_t*)(recs + w), (uint32_t)lane);
    if (lane < 16 + 2 * nch) return ldg((const uint32_t*)(sws + (size_t)w * nch), (uint32_t)(lane - 16));
    return 0u;  // chunks past nch: nothing feasible
  };
  int2 cb = wq_resolve(heads, W, tk);  // the static first batch
  if (cb.y > 0) wq_issue(heads, tk);   // the next batch's ticket, resolved when this batch ends
  int w = cb.y > 0 ? cb.x : -1;
  uint32_t cur = fetch(w);
  int bend = cb.x + cb.y;
  KAD_PACC;
  while (w >= 0) {
    // per unit, opaque copies of the loop invariants its conditions derive from: the conditions are then
    // evaluated inside the unit (a few scalar compares) instead of hoisted out of the unit loop and kept
    // live — and spilled — across it as 64-bit masks
    const int nch_o = XN > 0 ? nch : opq(nch);
#define nch nch_o
    // the next unit: within this batch, else the head of the next batch
    int wn = -1;
    if (w + 1 < bend) {
      wn = w + 1;
    } else {
      const int2 nb = wq_resolve(heads, W, tk);
      if (nb.y > 0) {
        wn = nb.x;
        bend = nb.x + nb.y;
        wq_issue(heads, tk);  // resolved one batch later
#ifdef KAD_PHASE_PROF
        wx_deq = __builtin_amdgcn_s_memrealtime();
#endif
      }
    }
    const uint32_t nxt = fetch(wn);
    KAD_PT(t0);
#ifdef KAD_PHASE_PROF
    const unsigned long long ut0 = __builtin_amdgcn_s_memrealtime();
    int ut_n = 0;
    uint32_t ut_fl = 0;
#endif

    auto fld = [&](int d) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)cur, d); };
    auto fld64 = [&](int d) -> int64_t { return (int64_t)(((uint64_t)fld(d + 1) << 32) | fld(d)); };
    const uint32_t fc = fld(0);
    const int gvc = (int)fld(1);
    const int tsc = (int)fld(2);
    const int64_t rqc = fld64(4), rqm = fld64(6);
    const uint64_t tolc = (uint64_t)fld64(12);
    do {  // one unit; `break` = done with it
      if (fc & REC_ROW) break;  // prep_kernel routed it to schedule_row_kernel
      if (fc & KAD_W_STICKY) {  // generic_scheduler.go:101-104
        wide_status(w, KAD_ST_STICKY);
        break;
      }
      if ((fc & REC_FULL) || (uint64_t)rqc >= (1ull << 46) || (uint64_t)rqm >= (1ull << 46) ||
          (fc & KAD_W_WIDE_SCORES)) {
        wide_defer(w);
        break;
      }
      const double rqcd = (double)rqc, rqmd = (double)rqm;  // exact: 0 <= request < 2^46
      const int spo = (int)fld(3);
      const int64_t mc = fld64(8), ooff = fld64(10);
      const uint64_t tolp0 = (uint64_t)fld64(14);
      const bool use_cur = f_taint && (fc & KAD_W_HAS_CURRENT);
      const bool fit_on = f_fit && (fc & KAD_W_FIT_NONZERO);
      const uint64_t o_taint = f_taint ? 0ull : ~0ull;
      const uint64_t o_api = f_api ? 0ull : ~0ull, a_api = gvc >= 0 ? ~0ull : 0ull;
      const double fcpu = fit_on ? rqcd : -1.0, fmem = fit_on ? rqmd : -1.0;  // fit off: compare against -1

      // ---------------- filters → compacted feasible list (findClustersThatFitWorkload, :152-169)
      int n = 0;
      // the chunk loop twice: FAST (one taint word, no CurrentClusters) has no branch inside a
      // 4-chunk group, so the 8 LDS reads of a group issue together; compaction stores are
      // exec-free (infeasible lanes and overflow positions write into pid[], rewritten before use)
      // MODE 2 (FOLD): taint + API already in the static words; 1 (FAST): one taint word, no
      // CurrentClusters; 0: general
      auto filter_chunks = [&](auto mode_t) {
        constexpr int MODE = decltype(mode_t)::value;
        constexpr bool FAST = MODE >= 1, FOLD = MODE >= 2, FITF = MODE == 3;
        // exactly 8 chunks (C4's instantiation): KAD_WIDE_C8 0 keeps the unrolled chunk loop below, 1 gives
        // each lane 8 clusters (all 64 lanes hold bits), 2 the 16-cluster pieces of the general case (half the
        // lanes idle at 512 clusters; 5a66d20 took C4's wide kernel 665 -> 688 us: profiles/r06/bisect_c4.txt)
        constexpr int C8 = KAD_WIDE_C8;
        constexpr bool PIECES = FITF && !(XN == 8 && C8 == 0);
        if constexpr (PIECES) {
          // the static words are the whole filter: compact them with each lane owning B = 16 (8) clusters
          // instead of a chunk loop (per chunk two readlanes, a 64-bit rank and a store — ~9 VALU + 4 SALU, 16
          // chunks at C3). Lane L takes clusters B·L .. B·L+B-1 (its B bits of the dword in lane 16 + L·B/32 of
          // `cur`), its first position is the wave's exclusive prefix of the piece popcounts (cluster order),
          // and the lanes write their set bits one per trip — as many trips as the densest piece holds
          // (C3: ~6); lanes out of bits write their dummy slot P + lane (no exec-mask branch)
          constexpr bool B8 = XN == 8 && C8 == 1;
          constexpr int B = B8 ? 8 : 16;
          const uint32_t dw = (uint32_t)__builtin_amdgcn_ds_bpermute((16 + (B8 ? lane >> 2 : lane >> 1)) << 2, (int)cur);
          uint32_t x = B8 ? (dw >> ((lane & 3) << 3)) & 0xFFu : (dw >> ((lane & 1) << 4)) & 0xFFFFu;
          const int c = __builtin_popcount(x);
          const int incl = wave_incl_sum_i32(c);
          n = __builtin_amdgcn_readlane(incl, 63);
          if (n > P) return;  // (positions past P are never written: the unit goes to rows / defer)
          int pos = incl - c;
          const int base = B * lane;
          while (ballot(x != 0)) {
            const bool on = x != 0;
            const int bit = __builtin_ctz(x | (1u << B));
            idx[on ? pos : P + KAD_DUMMY_STRIDE * lane] = (uint16_t)(base + bit);
            pos += on ? 1 : 0;
            x &= x - 1u;
          }
          return;
        }
        // FOLD: fully unrolled (constant readlane lanes for the static words); else one 4-chunk group per trip
#pragma unroll
        for (int g = 0; g < (FOLD ? NCH : nch); g += 4) {
          if (FOLD && g >= nch) break;
          uint64_t mk[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ch = g + j;
            const int c = ch * WAVE + lane;
            uint64_t m = ~0ull;  // lanes past C and chunks past nch: cleared in the static words
            const int cc = c < Cp ? c : 0;
            const double2 av = FITF ? make_double2(0.0, 0.0) : c_av[cc];
            const ulonglong2 tg = FOLD ? make_ulonglong2(0ull, 0ull) : c_tg[cc];
            const uint64_t sw0 = (((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)cur, 17 + 2 * ch)) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)cur, 16 + 2 * ch);
            bool tok;
            if constexpr (FAST) {
              tok = (tg.x & ~tolc) == 0;
            } else {
              WArgs a = wargs();
              const bool sch = use_cur && ch < nch && ((ldc(a->b.cw + (size_t)w * nch + ch) >> lane) & 1);
              tok = ((sch ? c_ne[cc] : tg.x) & ~tolc) == 0;
              for (int tw = 1; tw < TWs; ++tw) {  // more than 64 taint ids: words 1.. from global
                const uint32_t cl = c < C ? (uint32_t)c : 0u;
                const uint64_t xt = sch ? ldg(a->s.ne, (uint32_t)(tw * C) + cl) : ldg(a->s.nsne, (uint32_t)(tw * C) + cl);
                tok &= (xt & ~ldc(a->b.tol_all + (size_t)tsc * TWs + tw)) == 0;
              }
            }
            // fit.go:73-134 on exact f64: available - request >= 0 (FITF: in the static words)
            const uint64_t m_fit = FITF ? ~0ull : ballot(av.x >= fcpu) & ballot(av.y >= fmem);
            if constexpr (FOLD) {
              (void)tok;
              m &= sw0 & m_fit;
            } else {
              const uint64_t m_taint = ballot(tok);                    // taint_toleration.go:50-77
              const uint64_t m_api = ballot((tg.y >> (gvc & 63)) & 1);  // apiresources.go:25-43
              m &= sw0 & (m_taint | o_taint) & ((m_api & a_api) | o_api) & m_fit;
            }
            mk[j] = m;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            // positions past P (the unit is then deferred) stay inside the wave's region (pid, posl); the
            // rank is computed by every lane (pinned in a VGPR) so the address is one v_cndmask, not an
            // exec-mask branch
            int r = n + mbcnt(mk[j]);
            asm volatile("" : "+v"(r));
            idx[lane_on(mk[j]) ? r : P + lane] = (uint16_t)((g + j) * WAVE + lane);
            n += popc64(mk[j]);
          }
        }
      };
      // (the wide kernel runs on clean snapshots of C <= 1024: fold implies fitf; the general mode is
      // correct for any snapshot, re-testing what the static words hold)
      // (the LeastAllocated instantiation runs only on folded, fit-folded snapshots: the host checks; at C3
      // dropping the other modes takes its spilled SGPRs 27 -> 1, while the C4 instantiation ran 0.7 % slower
      // without them)
      if (SM == (1 << KAD_PL_LEAST_ALLOCATED) || (fold && fitf))
        filter_chunks(std::integral_constant<int, 3>{});
      else if (!fold && !use_cur && TWs == 1)
        filter_chunks(std::integral_constant<int, 1>{});
      else
        filter_chunks(std::integral_constant<int, 0>{});
      KAD_PT(t1);
      KAD_PADD(0, t1 - t0);
#ifdef KAD_PHASE_PROF
      ut_n = n;
#endif
      if (n == 0) {  // generic_scheduler.go:112-114
        wide_status(w, KAD_ST_NO_FEASIBLE);
        break;
      }
      if (n > P) {
        wide_row_or_defer(w);
        break;
      }
      if ((sm & BIT(KAD_PL_CLUSTER_AFFINITY)) && (fc & KAD_W_SCORE_ERROR)) {  // framework.go:149-159
        wide_status(w, KAD_ST_ERR_SCORE);
        break;
      }
      if (WIDE_EXP(2)) {
        wide_status(w, KAD_ST_OK);
        break;
      }
      wave_sync();

      // ---------------- scores of positions 64q + lane (RunScorePlugins, framework.go:139-181)
      const int nq = (n + 63) >> 6;
      int t[Q];
      uint32_t cid[Q];
      int ttv[Q];
      int ttmax = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        t[q] = 0;
        cid[q] = 0;
        ttv[q] = 0;
        if (q >= nq) continue;
        const int p = q * 64 + lane;
        const bool v = p < n;
        const uint32_t raw = idx[p];  // (p < 512 = P: inside the wave's region, no exec branch; past n discarded)
        cid[q] = v ? raw : 0u;
        const uint32_t cq = cid[q];
        if (ZR) {  // (s_res: ZR launches only with a resource score in the profile)
          t[q] = c_zs[cq];
        } else if (s_res) {
          // x = cap - req = available - request (exact); req > cap <=> x < 0 (score 0)
          const double2 cap = c_cap[cq], av = c_av[cq];
          const double xc = av.x - rqcd, xm = av.y - rqmd;
          const float2 iv = c_iv[cq];
          const double xcp = fmax(xc, 0.0), xmp = fmax(xm, 0.0);
          const int okc = -(int)(xc >= 0.0), okm = -(int)(xm >= 0.0);
          int x = 0;
          if (sm & BIT(KAD_PL_LEAST_ALLOCATED)) x += (quot100(xcp, cap.x, iv.x) + quot100(xmp, cap.y, iv.y)) >> 1;
          if (sm & BIT(KAD_PL_MOST_ALLOCATED))
            x += ((quot100(cap.x - xcp, cap.x, iv.x) & okc) + (quot100(cap.y - xmp, cap.y, iv.y) & okm)) >> 1;
          if (sm & BIT(KAD_PL_BALANCED_ALLOCATION)) x += (int)balanced_d((cap.x - xc) / cap.x, (cap.y - xm) / cap.y);
          t[q] = x;
        }
        if (s_tt) {  // taint_toleration.go:91-118: PreferNoSchedule taints not tolerated
          int tc = popc64(c_pn[cq] & ~tolp0);
          for (int tw = 1; tw < TWs; ++tw) {
            WArgs a = wargs();
            tc += popc64(ldg(a->s.pns, (uint32_t)(tw * C) + cq) & ~ldc(a->b.tol_pns + (size_t)tsc * TWs + tw));
          }
          ttv[q] = v ? tc : 0;
          ttmax = ttv[q] > ttmax ? ttv[q] : ttmax;
        }
      }
      if (s_tt) {  // DefaultNormalizeScore(100, reverse=true), framework/util.go:455-483
        ttmax = wave_max_u_i32(ttmax);
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (q < nq) t[q] += ttmax == 0 ? 100 : 100 - (int)small_quot(100 * ttv[q], ttmax);
      }
      // units without preferred terms (C4's) score 0 everywhere: one scalar load of the term count decides
      // before the 64-word window's vector load (2ef3455 loaded the window for every unit: C4's wide kernel
      // 688 -> 728 us, profiles/r06/bisect_c4.txt)
      if ((sm & BIT(KAD_PL_CLUSTER_AFFINITY)) && ldc(wargs()->b.sprog + spo) > 0) {  // cluster_affinity.go:96-140
        WArgs a = wargs();
        const int32_t* sp = a->b.sprog + spo;
        const uint32_t pv = ldg((const uint32_t*)sp, (uint32_t)lane);  // program words 0..63 (slack past the blob)
        {
          int afs[Q];  // |raw| <= sum |weight| <= 2^20 (wider units are deferred)
          int amax = 0;
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            afs[q] = 0;
            if (q < nq && q * 64 + lane < n) afs[q] = (int)affinity_score_pv(a->b.req_mask, pv, sp, nch, (int)cid[q]);
            amax = afs[q] > amax ? afs[q] : amax;
          }
          amax = wave_max_u_i32(amax);
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (q < nq) {
              const int num = 100 * afs[q];
              t[q] += amax == 0 ? afs[q] : (num >= 0 && num < (1 << 24) ? (int)small_quot(num, amax) : num / amax);
            }
        }
      }

      KAD_PT(t2);
      KAD_PADD(1, t2 - t1);
      // ---------------- select (framework.go:183-209, max_cluster.go:42-66)
      WArgs ad = wargs();
      int k = n;
      if (ad->p.select_plugin == KAD_PL_MAX_CLUSTER && !WIDE_EXP(4)) {
        const bool hm = fc & KAD_W_HAS_MAX_CLUSTERS;
        if (hm && mc < 0) {
          wide_status(w, KAD_ST_ERR_SELECT);
          break;
        }
        if (hm && mc < k) k = (int)mc;
      }
      // selection rule for the output pass: 0 all, 1 total >= T, 2 first ties (n <= 12), 3 replay ranks
      int mode = 0, T = 0, need = 0;
      uint32_t rflags = 0;
      if (k < n && k > 0) {
        int mn = INT32_MAX, mx = INT32_MIN;
#pragma unroll
        for (int q = 0; q < Q; ++q)
          if (q < nq) {
            const bool vq = q * 64 + lane < n;
            mn = (vq && t[q] < mn) ? t[q] : mn;
            mx = (vq && t[q] > mx) ? t[q] : mx;
          }
        int mn32, mx32;
        wave_minmax_u_i32(mn, mx, mn32, mx32);
        int lo32 = mn32, hi32 = mx32;
        int gcount = -1, e = 0;  // #(total > T), #(total == T); -1: count them below
        if ((uint32_t)mx32 - (uint32_t)mn32 < 128u) {
          // LDS histogram in descending bin order + one wave prefix sum: the k-th largest total, and the
          // counts above / at it from the same prefix (no per-position ballots)
          uint32_t* hist = key;
          *(uint2*)(hist + 2 * lane) = make_uint2(0u, 0u);
          wave_sync();
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (q < nq) {  // exec-free: lanes past n add 0 to bin `lane` (one shared bin: 26M of C3's 78M
              // LDS bank-conflict cycles, 0.5 % of the kernel; profiles/r06/ab_c3_lds_conflicts.txt)
              const bool vq = q * 64 + lane < n;
              atomicAdd(hist + (vq ? 127 - (t[q] - mn32) : lane), vq ? 1u : 0u);
            }
          wave_sync();
          const uint2 hh = *(const uint2*)(hist + 2 * lane);  // bins 127-2l, 126-2l
          const int pre = wave_incl_sum_i32((int)(hh.x + hh.y));
          const int l0 = (int)__builtin_ctzll(ballot(pre >= k));
          const int pl = __builtin_amdgcn_readlane(pre, l0);
          const int h0 = __builtin_amdgcn_readlane((int)hh.x, l0);
          const int h1 = __builtin_amdgcn_readlane((int)hh.y, l0);
          const bool first = pl - h1 >= k;  // T is the higher bin of lane l0's pair
          lo32 = mn32 + (first ? 127 - 2 * l0 : 126 - 2 * l0);
          e = first ? h0 : h1;
          gcount = first ? pl - h1 - h0 : pl - h1;
          wave_sync();
        } else {
          while (lo32 < hi32) {  // the largest T with #(total >= T) >= k
            const uint32_t d = (uint32_t)hi32 - (uint32_t)lo32;
            const int mid = (int)((uint32_t)lo32 + (d >> 1) + (d & 1));
            int cnt = 0;
#pragma unroll
            for (int q = 0; q < Q; ++q)
              if (q < nq) cnt += popc64(ballot(q * 64 + lane < n && t[q] >= mid));
            if (cnt >= k)
              lo32 = mid;
            else
              hi32 = mid - 1;
          }
        }
        T = lo32;
        if (gcount < 0) {
          gcount = 0;
#pragma unroll
          for (int q = 0; q < Q; ++q)
            if (q < nq) {
              const bool v = q * 64 + lane < n;
              gcount += popc64(ballot(v && t[q] > T));
              e += popc64(ballot(v && t[q] == T));
            }
        }
        need = k - gcount;
        if (need == e) {  // the cut takes every tie: no sort needed
          mode = 1;
        } else {
          rflags = KAD_RF_TIE_STRADDLE;
          if (n <= 12 || WIDE_EXP(1)) {  // pdqsort_func: a single (stable) insertionSort
            mode = 2;
          } else {
            // restricted pdqsort replay, wave-parallel, on u32 keys total - min (order-preserving)
            const int xs_b = (ad->p.flags & KAD_PROFILE_XORSHIFT_GO121) ? 7 : 17;
            const int xs_c = (ad->p.flags & KAD_PROFILE_XORSHIFT_GO121) ? 17 : 5;
            KAD_PT(r0);
            if ((uint32_t)mx32 - (uint32_t)mn32 < 65536u) {
              // packed replay: key << 16 | position (n <= 512), one LDS word per element
#pragma unroll
              for (int q = 0; q < Q; ++q)
                if (q < nq && q * 64 + lane < n)
                  key[q * 64 + lane] = ((uint32_t)(t[q] - mn32) << 16) | (uint32_t)(q * 64 + lane);
              wave_sync();
              PdqWaveP<> pw{key, posl, posr, xs_b, xs_c};
              KAD_PT(r1);
              pw.select(n, k);
              KAD_PT(r2);
              for (int r = lane; r < n; r += WAVE) inv[key[r] & 0xFFFFu] = (uint16_t)r;
              wave_sync();
              KAD_PT(r3);
              KAD_PADD(6, (r1 - r0) + (r3 - r2));
#ifdef KAD_PHASE_PROF
              KAD_PADD(7, pw.pr[0]);
              KAD_PADD(8, pw.pr[1]);
              KAD_PADD(9, pw.pr[2]);
              KAD_PADD(10, pw.pr[3]);
              KAD_PADD(11, n);
#endif
            } else {
#pragma unroll
              for (int q = 0; q < Q; ++q)
                if (q < nq && q * 64 + lane < n) {
                  key[q * 64 + lane] = (uint32_t)(t[q] - mn32);
                  pid[q * 64 + lane] = (uint16_t)(q * 64 + lane);
                }
              wave_sync();
              PdqWave<uint32_t> pw{key, pid, posl, posr, xs_b, xs_c};
              KAD_PT(r1);
              pw.select(n, k);
              KAD_PT(r2);
              for (int r = lane; r < n; r += WAVE) inv[pid[r]] = (uint16_t)r;
              wave_sync();
              KAD_PT(r3);
              KAD_PADD(6, (r1 - r0) + (r3 - r2));
            }
            mode = 3;
          }
        }
      } else if (k <= 0) {
        mode = -1;  // nothing selected
      }

      KAD_PT(t3);
      KAD_PADD(2, t3 - t2);
      if (rflags) {
        KAD_PADD(4, 1);
        KAD_PADD(5, t3 - t2);
      }
#ifdef KAD_PHASE_PROF
      ut_fl = rflags ? 1u : 0u;
#endif
      // ---------------- output, ascending cluster id (= ascending position)
      {
        WArgs ae = wargs();
        const bool dup = fc & KAD_W_DUPLICATE;
        const bool replicas =
            !dup && ae->p.replicas_plugin == KAD_PL_CLUSTER_CAPACITY_WEIGHT && (fc & REC_DESIRED_POS) && k > 0;
        int base = 0;
        if ((dup || replicas) && mode >= 0 && !WIDE_EXP(8)) {
          int32_t* oc = ae->o.cluster + ooff;
          int64_t* orp = ae->o.replicas + ooff;
          const int64_t rv = dup ? -1 : 0;
          // the selection mode is uniform: one branch per unit, then a branch-free predicate per position
          auto emit = [&](int q, bool s) {
            const uint64_t sel = ballot(s);
            const uint32_t at = (uint32_t)(base + mbcnt(sel));
            if (s) {
              stg(oc, at, (int32_t)cid[q]);
              stg(orp, at, rv);
            }
            base += popc64(sel);
          };
          if (mode == 3) {  // the replay's ranks
#pragma unroll
            for (int q = 0; q < Q; ++q)
              if (q < nq) {
                const int p = q * 64 + lane;
                const uint32_t rk = inv[p];  // (p < P + 64: inside the region, no exec branch; past n discarded)
                emit(q, p < n && rk < (uint32_t)k);
              }
          } else if (mode == 2) {  // every total > T, then the first `need` ties by position
            int eq_before = 0;
#pragma unroll
            for (int q = 0; q < Q; ++q)
              if (q < nq) {
                const bool v = q * 64 + lane < n;
                const uint64_t eqm = ballot(v && t[q] == T);
                emit(q, v && (t[q] > T || (t[q] == T && mbcnt(eqm) + eq_before < need)));
                eq_before += popc64(eqm);
              }
          } else {  // 0: every position; 1: total >= T
            const int Tlo = mode == 0 ? INT32_MIN : T;
#pragma unroll
            for (int q = 0; q < Q; ++q)
              if (q < nq) emit(q, q * 64 + lane < n && t[q] >= Tlo);
          }
        }
        if (lane == 0) {
          ae->o.status[w] = KAD_ST_OK;
          ae->o.count[w] = base;  // Divide without replicas plugin: empty map
          ae->o.flags[w] = rflags;
        }
      }
      wave_sync();
      KAD_PT(t4);
      KAD_PADD(3, t4 - t3);
    } while (false);
#ifdef KAD_PHASE_PROF
    {
      KAD_PT(tz);
      wx_units++;
      wx_max = (tz - t0) > wx_max ? (tz - t0) : wx_max;
      const unsigned long long ut1 = __builtin_amdgcn_s_memrealtime();
      if (lane == 0 && w < KAD_UTRACE_MAX) {
        const unsigned long long gw = (unsigned long long)(blockIdx.x * nwaves + wv) & 0xFFFFull;
        g_ustart[w] = ut0;
        g_uinfo[w] = (ut1 - ut0) | ((unsigned long long)(ut_n & 0x7FFF) << 32) | ((unsigned long long)ut_fl << 47) |
                     (gw << 48);
      }
    }
#endif
    cur = nxt;
    w = wn;
#undef nch
  }
#ifdef KAD_PHASE_PROF
  {
    const int gwv = blockIdx.x * nwaves + wv;
    if (lane == 0 && gwv < 8192) {
      g_wavetime[2 * gwv] = wt_start;
      g_wavetime[2 * gwv + 1] = __builtin_amdgcn_s_memrealtime();
      g_wavex[6 * gwv] = wx_units;
      g_wavex[6 * gwv + 1] = wx_max;
      g_wavex[6 * gwv + 2] = wx_deq;
      g_wavex[6 * gwv + 3] = pacc[4];
      g_wavex[6 * gwv + 4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      g_wavex[6 * gwv + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    }
  }
#endif
  KAD_PFLUSH_LEAN;
}


// ================================================== row schedule kernel
// schedule_row_kernel — the units whose feasible list is longer than the lean / wide kernels' register
// positions (C5: 16 % of the units, a few thousand feasible clusters of 10 000), on snapshots where
// every filter is in the static words (BatchDev::use_rows: clean, SnapDev::fold and ::fitfold,
// C <= ROW_MAX_C). One 512-thread workgroup per unit, two per CU (LDS: 6 B per cluster + the preferred-
// term words, which the replay scratch reuses), persistent (units dequeued from BatchDev::rows):
//   * compaction: the unit's static words → per-chunk popcounts → block prefix → cluster ids in LDS
//     (findClustersThatFitWorkload order, generic_scheduler.go:152-169);
//   * scores spread over the 8 waves (RunScorePlugins, framework.go:139-181), the clean-snapshot
//     arithmetic of the wide kernel (exact f64 quotients, 32-bit totals), block maxima for
//     DefaultNormalizeScore (framework/util.go:455-483);
//   * MaxCluster (max_cluster.go:42-66): the k-th largest total by a block-wide 8-bit radix histogram;
//     the cut takes every tie, or wave 0 replays Go's pdqsort restricted to k (PdqWave) on the LDS keys,
//     its position scratch in LDS up to ROW_NREP positions, else in the block's global slab;
//   * output in ascending cluster id by per-chunk ballots and a block prefix.
// Units outside the clean-f64 range (requests >= 2^46, wide affinity weights) or with more than
// ROW_MAX_TERMS preferred terms go on to the defer list.
constexpr int ROW_THREADS = 512;
constexpr int ROW_WAVES = ROW_THREADS / 64;
constexpr int ROW_MAX_WAVES = 16;  // the row body also runs on schedule_wide_kernel's 1024-thread blocks
constexpr int ROW_MAX_C = 12288;
constexpr int ROW_NREP = 2048;    // replays of up to this many positions keep their scratch in LDS
constexpr int ROW_BLOCK_PART = 256;  // replay partitions of longer ranges run on every wave of the block
#ifndef KAD_ROW_RU
#define KAD_ROW_RU 2
#endif
#ifndef KAD_ROW_MINW
#define KAD_ROW_MINW 2  // waves per SIMD the row kernel's VGPR budget is sized for (2 blocks of 8 waves / CU: 4)
#endif
// scoring: positions per thread trip, their gathers issued together. 3 cut the score phase's cycles per row
// by 29 % (profiling build, profiles/r03/q6_c5_ru*.json) but at 127 VGPRs the kernel ran 1.5 % longer (C5
// rows 1.28 -> 1.30 ms, two product builds on one box); 4 spills and drops to one block per CU
constexpr int ROW_RU = KAD_ROW_RU;
static_assert(ROW_MAX_BLOCKS >= 1, "row kernel slabs");
struct RowKLayout {
  size_t key, idx, x, pid, posl, posr, sw, cnt, hist, red, pre, bytes;
};
// a unit's staged record and score program (u32[2][ROW_PRE_DW], the next unit's prefetched into the other
// buffer): its UnitRec dwords, the program length, then its first ROW_PRE_PROG program words
constexpr int ROW_PRE_PROG = 64, ROW_PRE_DW = 16 + 1 + ROW_PRE_PROG + 15;
__host__ __device__ inline RowKLayout rowk_layout(int C) {
  const size_t Cp = (size_t)((C + 63) & ~63), nch = Cp / 64;
  RowKLayout L;
  L.key = 0;                              // u32[Cp]: fixed | TT raw << 16, then totals (sign-flipped), replay keys
  L.idx = L.key + 4 * Cp;                 // u16[Cp]: position → cluster id
  L.x = L.idx + 2 * Cp;                   // preferred-term words u64[8][nch] while scoring, then the replay
  L.pid = L.x;                            //   scratch: pid u16[NREP], posl u16[NREP + 64], posr u16[NREP]
  L.posl = L.pid + 2 * ROW_NREP;
  L.posr = L.posl + 2 * ROW_NREP + 128;
  const size_t xb = Cp > 6 * (size_t)ROW_NREP + 128 ? Cp : 6 * (size_t)ROW_NREP + 128;
  L.sw = (L.x + xb + 15) & ~(size_t)15;   // u64[2][nch]: the unit's static words (two buffers: the next
  L.cnt = L.sw + 16 * nch;                //   unit's are prefetched); i32[2][nch + 1]: chunk counts →
                                          //   exclusive prefix (+ total)
  L.hist = (L.cnt + 8 * (nch + 1) + 15) & ~(size_t)15;  // u32[256]
  L.red = L.hist + 4 * 256;               // i32[4][ROW_MAX_WAVES] per-wave partials, i32[24] broadcasts
  L.pre = L.red + 4 * (4 * ROW_MAX_WAVES + 24);  // u32[2][ROW_PRE_DW]: staged records + score programs
  L.bytes = L.pre + 4 * 2 * ROW_PRE_DW;
  return L;
}
size_t row_kernel_lds(int C) { return rowk_layout(C).bytes; }
bool row_kernel_fits(int C) { return C > 0 && C <= ROW_MAX_C; }
// per-block global slab for replays longer than ROW_NREP: pid u16[Cp], posl u16[Cp + 64], posr u16[Cp]
__host__ __device__ size_t row_slab_bytes(int C) { return ((size_t)6 * ((C + 63) & ~63) + 128 + 255) & ~(size_t)255; }

struct RowArgs {
  SnapDev s;
  BatchDev b;
  OutDev o;
  ProfDev p;
  char* slabs;  // [grid][row_slab_bytes(C)]
  int exp;      // measurement-only variants (profiling builds, KAD_ROW_EXPERIMENT; results differ): bit 0 no
                // resource scores, bit 1 no PreferNoSchedule counts, bit 2 no affinity scores
};
typedef const __attribute__((address_space(4))) RowArgs* RArgs;
__device__ __forceinline__ RArgs rargs() {
  return (RArgs)opq((uintptr_t)__builtin_amdgcn_kernarg_segment_ptr());
}

// block-wide reductions of one i32 per thread: wave partials in red[nw], every thread reads all (NW > 0: the
// wave count as a constant)
template <int NW>
__device__ __forceinline__ int row_block_max(int v, int* red, int nw) {
  const int r = wave_max_u_i32(v);
  if (lane_id() == 0) red[threadIdx.x >> 6] = r;
  __syncthreads();
  int m = red[0];
  if constexpr (NW > 0) {
#pragma unroll
    for (int i = 1; i < NW; ++i) m = red[i] > m ? red[i] : m;
  } else {
    for (int i = 1; i < nw; ++i) m = red[i] > m ? red[i] : m;
  }
  __syncthreads();
  return m;
}
template <int NW>
__device__ __forceinline__ int row_block_min(int v, int* red, int nw) { return -row_block_max<NW>(-v, red, nw); }
template <int NW>
__device__ __forceinline__ int row_block_sum(int v, int* red, int nw) {
  const int r = wave_sum_u_i32(v);
  if (lane_id() == 0) red[threadIdx.x >> 6] = r;
  __syncthreads();
  int m = 0;
  if constexpr (NW > 0) {
#pragma unroll
    for (int i = 0; i < NW; ++i) m += red[i];
  } else {
    for (int i = 0; i < nw; ++i) m += red[i];
  }
  __syncthreads();
  return m;
}
// exclusive prefix of cnt[0..m) in place by wave `by`, total in cnt[m]; callers sync before and after
__device__ __forceinline__ void row_exclusive_scan(int* cnt, int m, int by = 0) {
  if ((int)(threadIdx.x >> 6) != by) return;
  const int lane = lane_id();
  int carry = 0;
  for (int c0 = 0; c0 < m; c0 += WAVE) {
    const int i = c0 + lane;
    const int v = i < m ? cnt[i] : 0;
    const int inc = wave_incl_sum_i32(v);
    if (i < m) cnt[i] = carry + inc - v;
    carry += __builtin_amdgcn_readlane(inc, 63);
  }
  if (lane == 0) cnt[m] = carry;
}

// The row path over BatchDev::rows, for one workgroup: schedule_row_kernel's body (NT = ROW_THREADS) and
// schedule_wide_kernel's opening phase (NT = 0: the wide block's blockDim.x threads, up to ROW_MAX_WAVES
// waves) — the wide kernel's blocks take the units prep_kernel routed to rows before their own work
// queue, so no second stream, fork or join is needed. `args` returns the kernel's arguments (SnapDev s,
// BatchDev b, OutDev o, ProfDev p in the constant address space); smem: row_kernel_lds(C) bytes of LDS.
// SM >= 0: specialised for that score-plugin mask (as schedule_wide_kernel).
template <int SM, int NT, class ArgsOf>
__device__ __forceinline__ void row_units(ArgsOf rargs, char* smem, int rexp_arg) {
  constexpr int NW = NT / 64;
  const int NTH = NT > 0 ? NT : (int)blockDim.x;
  const int NWV = NT > 0 ? NW : NTH >> 6;
  const int tid = threadIdx.x, lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  int C, TW;
  uint32_t fm, sm;
  {
    auto a = rargs();
    C = a->s.C;
    TW = a->s.TW;
    fm = a->p.filter_mask;
    sm = SM >= 0 ? (uint32_t)SM : a->p.score_mask;
  }
  (void)fm;
  const int nch = (C + 63) >> 6;
  const RowKLayout L = rowk_layout(C);
  uint32_t* key = (uint32_t*)(smem + L.key);
  uint16_t* idx = (uint16_t*)(smem + L.idx);
  uint16_t* pid_l = (uint16_t*)(smem + L.pid);
  uint16_t* posl_l = (uint16_t*)(smem + L.posl);
  uint16_t* posr_l = (uint16_t*)(smem + L.posr);
  uint64_t* termw = (uint64_t*)(smem + L.x);  // preferred-term words (scoring and normalisation only)
  uint16_t* pid_g;  // the block's global slab (replays longer than ROW_NREP)
  pid_g = (uint16_t*)(rargs()->b.row_slabs + (size_t)blockIdx.x * row_slab_bytes(C));
  uint64_t* const swl0 = (uint64_t*)(smem + L.sw);
  int32_t* const cnt0 = (int32_t*)(smem + L.cnt);
  uint32_t* hist = (uint32_t*)(smem + L.hist);
  int32_t* red = (int32_t*)(smem + L.red);
  int32_t* bc = red + 4 * ROW_MAX_WAVES;  // broadcasts
#if defined(KAD_PHASE_PROF) || defined(KAD_TUNING)
  const int rexp = rexp_arg;
#else
  constexpr int rexp = 0;
  (void)rexp_arg;
#endif
  const bool s_res =
      (sm & (BIT(KAD_PL_LEAST_ALLOCATED) | BIT(KAD_PL_MOST_ALLOCATED) | BIT(KAD_PL_BALANCED_ALLOCATION))) && !(rexp & 1);
  const bool s_tt = (sm & BIT(KAD_PL_TAINT_TOLERATION)) && !(rexp & 2);

  KAD_PACC;
  // the next unit's list index is dequeued one unit ahead (thread 64, wave 1's lane 0), so the returning
  // atomic's latency overlaps the current unit. While wave 0 replays (or before the output pass) wave 1
  // also prefetches the next unit: its static words, chunk counts and their prefix into the other LDS
  // buffer (bc[20]: the prefetched unit, -1 the list is drained, -2 nothing prefetched); the list is
  // complete before this kernel starts (prep_kernel's early routing, or the lean kernel before it)
  // thread 64 holds the list length (complete before this kernel starts), its ticket and the unit the ticket
  // names, loaded one dequeue ahead: a dequeue returns a unit already in a register and only issues the next
  // ticket's atomic and list load (waited for at the next dequeue, a unit later)
  int ticket = 0, rn = 0, nxt_u = -1;
  if (tid == 64) {
    auto a = rargs();
    rn = __hip_atomic_load(a->b.rows_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = atomicAdd(a->b.rows_head, 1);
    nxt_u = ticket < rn ? a->b.rows[ticket] : -1;
  }
#ifdef KAD_PHASE_PROF
  const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long rt_units = 0;
#endif
  if (tid == 0) bc[20] = -2;
  int par = 0;  // the current unit's buffers
  uint32_t* const pre0 = (uint32_t*)(smem + L.pre);
  // one wave: unit u's UnitRec dwords (lanes 0-15), its score-program length and first ROW_PRE_PROG words into
  // pr — the unit's scalars are then LDS reads, not a chain of scalar loads (record → program → each term)
  auto stage_unit = [&](int u, uint32_t* pr) {
    auto a = rargs();
    const uint32_t rd = lane < 16 ? ldg((const uint32_t*)(a->b.rec + u), (uint32_t)lane) : 0u;
    const int so = ldg(a->b.sprog_off, (uint32_t)u), se = ldg(a->b.sprog_off, (uint32_t)u + 1u);
    const int len = se - so;
    const int32_t pw = lane < len ? ldg(a->b.sprog, (uint32_t)(so + lane)) : 0;
    if (lane < 16) pr[lane] = rd;
    if (lane == 0) pr[16] = (uint32_t)len;
    pr[17 + lane] = (uint32_t)pw;
  };
  auto next_unit = [&]() -> int {  // thread 64 only
    const int nx = nxt_u;
    if (nx >= 0) {
      auto a = rargs();
      ticket = atomicAdd(a->b.rows_head, 1);
      nxt_u = ticket < rn ? a->b.rows[ticket] : -1;
    }
    return nx;
  };
  auto prefetch = [&]() {  // wave 1
    if (lane == 0) bc[20] = next_unit();
    wave_sync();
    const int nx = __builtin_amdgcn_readfirstlane(bc[20]);
    if (nx < 0) return;
    stage_unit(nx, pre0 + (size_t)(par ^ 1) * ROW_PRE_DW);
    uint64_t* sw2 = swl0 + (size_t)(par ^ 1) * nch;
    int32_t* c2 = cnt0 + (size_t)(par ^ 1) * (nch + 1);
    const uint64_t* src = rargs()->b.sw + (size_t)nx * nch;
    for (int ch = lane; ch < nch; ch += WAVE) {
      const uint64_t m = ldg(src, (uint32_t)ch);
      sw2[ch] = m;
      c2[ch] = popc64(m);
    }
    wave_sync();
    row_exclusive_scan(c2, nch, 1);
  };
  for (;;) {
    __syncthreads();  // the previous unit's LDS reads (and wave 1's prefetch) are done
    KAD_PT(t0);
    if (tid == 64) {
      const int pf = bc[20];
      bc[21] = pf != -2 ? 1 : 0;
      bc[0] = pf != -2 ? pf : next_unit();
      bc[20] = -2;
    }
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(bc[0]);
    const bool pre = __builtin_amdgcn_readfirstlane(bc[21]) != 0;
    if (w < 0) break;
#ifdef KAD_PHASE_PROF
    rt_units++;
#endif
    if (pre) par ^= 1;
    uint64_t* const swl = swl0 + (size_t)par * nch;
    int32_t* const cnt = cnt0 + (size_t)par * (nch + 1);
    uint32_t* const pr = pre0 + (size_t)par * ROW_PRE_DW;
    bool did_pf = false;  // wave 1 prefetched the next unit during this one (uniform)
    auto a = rargs();
    if (!pre) {  // not prefetched: record, program and static words now (the chunk counts' prefix below)
      if (wv == 0) stage_unit(w, pr);
      for (int ch = tid; ch < nch; ch += NTH) {
        const uint64_t m = ldg(a->b.sw, (uint32_t)(w * nch + ch));
        swl[ch] = m;
        cnt[ch] = popc64(m);
      }
      __syncthreads();
      row_exclusive_scan(cnt, nch);
    }
    __syncthreads();
    auto prd = [&](int d) -> uint32_t { return (uint32_t)__builtin_amdgcn_readfirstlane((int)pr[d]); };
    auto prd64 = [&](int d) -> int64_t { return (int64_t)(((uint64_t)prd(d + 1) << 32) | prd(d)); };
    const uint32_t fc = prd(0);
    const int64_t rqc = prd64(4), rqm = prd64(6);
    const int spo = (int)prd(3);
    const int plen = (int)prd(16);
    // score program word i: staged in LDS (programs of up to ROW_PRE_PROG words, every bench unit's), else global
    auto spw = [&](int i) -> int32_t {
      return plen <= ROW_PRE_PROG ? (int32_t)prd(17 + i) : ldc(rargs()->b.sprog + spo + i);
    };
    const bool many_terms = (sm & BIT(KAD_PL_CLUSTER_AFFINITY)) && plen > 0 && spw(0) > ROW_MAX_TERMS;
    if ((uint64_t)rqc >= (1ull << 46) || (uint64_t)rqm >= (1ull << 46) || (fc & KAD_W_WIDE_SCORES) || many_terms) {
      if (tid == 0) {  // outside the exact clean-f64 range: the full kernel
        const int slot = atomicAdd(a->b.defer_n, 1);
        a->b.defer[slot] = w;
      }
      continue;
    }
    const int tsc = (int)prd(2);
    const int64_t mc = prd64(8), ooff = prd64(10);
    auto status = [&](int32_t st) {
      if (tid == 0) {
        auto ao = rargs();
        ao->o.status[w] = st;
        ao->o.count[w] = 0;
        ao->o.flags[w] = 0;
      }
    };

    // ---------------- compaction of the static words (every filter folded by prep_kernel)
    const int n = __builtin_amdgcn_readfirstlane(cnt[nch]);
    {
      // four chunks per trip, their words and offsets read together; every lane stores (infeasible lanes
      // into a dummy slot of the term-word region, unused until the term words below): no exec branch
      // between the LDS reads of consecutive chunks
      uint16_t* const dmy = (uint16_t*)(smem + L.x) + lane;
      for (int ch0 = wv; ch0 < nch; ch0 += 4 * NWV) {
        uint64_t mm[4];
        int co[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ch = ch0 + u * NWV;
          const int cl = ch < nch ? ch : nch - 1;
          const uint64_t m = swl[cl];
          mm[u] = ch < nch ? m : 0ull;
          co[u] = cnt[cl];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool on = lane_on(mm[u]);
          uint16_t* const dst = on ? idx + co[u] + mbcnt(mm[u]) : dmy;
          *dst = (uint16_t)((ch0 + u * NWV) * WAVE + lane);
        }
      }
    }
    KAD_PADD(0, 1);
    if (n == 0) {  // generic_scheduler.go:112-114
      status(KAD_ST_NO_FEASIBLE);
      continue;
    }
    if ((sm & BIT(KAD_PL_CLUSTER_AFFINITY)) && (fc & KAD_W_SCORE_ERROR)) {  // framework.go:149-159
      status(KAD_ST_ERR_SCORE);
      continue;
    }
    int k = n;
    if (a->p.select_plugin == KAD_PL_MAX_CLUSTER) {
      const bool hm = fc & KAD_W_HAS_MAX_CLUSTERS;
      if (hm && mc < 0) {
        status(KAD_ST_ERR_SELECT);
        continue;
      }
      if (hm && mc < k) k = (int)mc;
    }
    __syncthreads();
    KAD_PT(t1);
    KAD_PADD(1, t1 - t0);

    // ---------------- raw scores (RunScorePlugins, framework.go:139-181)
    const int32_t* sp = a->b.sprog + spo;
    const int n_terms = plen > 0 ? spw(0) : 0;
    const bool s_aff = (sm & BIT(KAD_PL_CLUSTER_AFFINITY)) && n_terms > 0 && !(rexp & 4);  // no terms: 0 everywhere
    // ClusterAffinity preferred terms (cluster_affinity.go:96-135) as per-chunk words in LDS (<= ROW_MAX_TERMS,
    // checked above): word (t, ch) = AND of the term's requirement rows — once per chunk instead of once per
    // feasible position; a position's raw score is then a sum of weights over LDS bit tests, recomputed
    // where it is needed (no per-position array)
    // the term list parsed once: weights in SGPRs (constant indices after unrolling), each term's
    // expression count and id offset in LDS for the (term, chunk) word pass
    int32_t wt[ROW_MAX_TERMS];
    int32_t* tdesc = bc + 4;  // [2][ROW_MAX_TERMS]: expression count, id offset (broadcast slots 4..19)
    {
      int pc = 1;
#pragma unroll
      for (int t = 0; t < ROW_MAX_TERMS; ++t) {
        wt[t] = 0;
        if (t < n_terms) {
          wt[t] = spw(pc);
          const int ne = spw(pc + 1);
          if (tid == 0) {
            tdesc[t] = ne;
            tdesc[ROW_MAX_TERMS + t] = pc + 2;
          }
          pc += 2 + ne;
        }
      }
    }
    int wabs = 0;  // sum of |weight|: bounds |raw affinity score|
#pragma unroll
    for (int t = 0; t < ROW_MAX_TERMS; ++t) wabs += t < n_terms ? (wt[t] < 0 ? -wt[t] : wt[t]) : 0;
    const bool apack = s_aff && wabs <= 4095;
    auto raw_aff = [&](uint32_t c) {
      int af = 0;
#pragma unroll
      for (int t = 0; t < ROW_MAX_TERMS; ++t)
        if (t < n_terms) af += ((termw[t * nch + (c >> 6)] >> (c & 63)) & 1) ? wt[t] : 0;
      return af;
    };
    if (s_aff) {
      __syncthreads();  // tdesc
      for (int x = tid; x < n_terms * nch; x += NTH) {
        const int t = x / nch, ch = x - t * nch;
        const int ne = tdesc[t], io = tdesc[ROW_MAX_TERMS + t];
        uint64_t m = ~0ull;
        if (plen <= ROW_PRE_PROG && ne >= 1 && ne <= 4) {  // the rows' loads together (ids repeat past ne: AND is idempotent)
          uint64_t r[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int id = (int)pr[17 + io + (i < ne ? i : ne - 1)];
            r[i] = ldg(a->b.req_mask, (uint32_t)id * (uint32_t)nch + (uint32_t)ch);
          }
          m = r[0] & r[1] & r[2] & r[3];
        } else {
          for (int i = 0; i < ne; ++i) {
            const int id = plen <= ROW_PRE_PROG ? (int)pr[17 + io + i] : ldg(sp, (uint32_t)(io + i));
            m &= ldg(a->b.req_mask, (uint32_t)id * (uint32_t)nch + (uint32_t)ch);
          }
        }
        termw[x] = m;
      }
      __syncthreads();
    }
    KAD_PT(t1a);
    KAD_PADD(6, t1a - t1);
    const double rqcd = (double)rqc, rqmd = (double)rqm;
    int ttmax = 0, amax = 0;
    // the unit's tolerated PreferNoSchedule words, once (scalar)
    uint64_t tpn[TFOLD_MAX_TW];
#pragma unroll
    for (int tw = 0; tw < TFOLD_MAX_TW; ++tw) tpn[tw] = (s_tt && tw < TW) ? ldc(a->b.tol_pns + (size_t)tsc * TW + tw) : 0ull;
    // ROW_RU positions per trip: every gather of all of them is issued before any is used (the phase is
    // latency-bound: its resource, taint and affinity parts cost cycles in proportion to their load chains)
    constexpr int RU = ROW_RU;
    for (int j0 = tid; j0 < n; j0 += RU * NTH) {
      auto as = rargs();
      double4 r4[RU];
      float2 iv[RU];
      uint64_t pn[RU][TFOLD_MAX_TW];
      uint32_t cs[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int j = j0 + u * NTH;
        cs[u] = idx[j < n ? j : j0];
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        r4[u] = make_double4(0.0, 0.0, 1.0, 1.0);
        iv[u] = make_float2(0.f, 0.f);
        if (s_res) {  // (available cpu, available mem, cap cpu, cap mem) as f64, f32 100 / cap
          r4[u] = as->s.res4[cs[u]];
          iv[u] = as->s.res_iv[cs[u]];
        }
        if (s_tt) {  // one 32-B gather (SnapDev::pns4: the row kernel runs on clean snapshots, TW <= 4)
          const ulonglong4 q = as->s.pns4[cs[u]];
          pn[u][0] = q.x;
          pn[u][1] = q.y;
          pn[u][2] = q.z;
          pn[u][3] = q.w;
        } else {
#pragma unroll
          for (int tw = 0; tw < TFOLD_MAX_TW; ++tw) pn[u][tw] = 0ull;
        }
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int j = j0 + u * NTH;
        if (j >= n) break;
        const uint32_t c = cs[u];
        int x = 0;
        if (s_res) {  // the wide kernel's clean path: x = available - request, exact in f64
          const double capc = r4[u].z, capm = r4[u].w;
          const double xc = r4[u].x - rqcd, xm = r4[u].y - rqmd;
          const float ivc = iv[u].x, ivm = iv[u].y;
          const double xcp = fmax(xc, 0.0), xmp = fmax(xm, 0.0);
          const int okc = -(int)(xc >= 0.0), okm = -(int)(xm >= 0.0);
          if (sm & BIT(KAD_PL_LEAST_ALLOCATED)) x += (quot100(xcp, capc, ivc) + quot100(xmp, capm, ivm)) >> 1;
          if (sm & BIT(KAD_PL_MOST_ALLOCATED))
            x += ((quot100(capc - xcp, capc, ivc) & okc) + (quot100(capm - xmp, capm, ivm) & okm)) >> 1;
          if (sm & BIT(KAD_PL_BALANCED_ALLOCATION)) x += (int)balanced_d((capc - xc) / capc, (capm - xm) / capm);
        }
        int tc = 0;
        if (s_tt)  // taint_toleration.go:91-118: PreferNoSchedule taints not tolerated
#pragma unroll
          for (int tw = 0; tw < TFOLD_MAX_TW; ++tw)
            if (tw < TW) tc += popc64(pn[u][tw] & ~tpn[tw]);
        int af = 0;
        if (s_aff) {  // |raw| <= 2^20 (wider units were deferred above)
          af = raw_aff(c);
          amax = af > amax ? af : amax;
        }
        // x <= 300 (three resource scores), tc <= 256 (TW <= 4); the raw affinity score rides along when the
        // unit's weights keep it within 13 signed bits, so the normalisation does not recompute it
        key[j] = (uint32_t)x | ((uint32_t)tc << 10) | (apack ? ((uint32_t)af & 0x1FFFu) << 19 : 0u);
        ttmax = tc > ttmax ? tc : ttmax;
      }
    }
    KAD_PT(t1b);
    KAD_PADD(7, t1b - t1a);
    if (s_tt) ttmax = row_block_max<NW>(ttmax, red, NWV);
    if (s_aff) amax = row_block_max<NW>(amax, red, NWV);
    __syncthreads();
    KAD_PT(t2);
    KAD_PADD(2, t2 - t1);

    // ---------------- DefaultNormalizeScore + totals, stored order-preserving as u32 (total ^ 2^31)
    int mn = INT32_MAX, mx = INT32_MIN;
    for (int j = tid; j < n; j += NTH) {
      const uint32_t x = key[j];
      int t = (int)(x & 0x3FFu);
      if (s_tt) t += ttmax == 0 ? 100 : 100 - (int)small_quot(100 * (int)((x >> 10) & 0x1FFu), ttmax);
      if (s_aff) {
        const int af = apack ? ((int32_t)x >> 19) : raw_aff(idx[j]);
        const int num = 100 * af;
        t += amax == 0 ? af : (num >= 0 && num < (1 << 24) ? (int)small_quot(num, amax) : num / amax);
      }
      key[j] = (uint32_t)t ^ 0x80000000u;
      mn = t < mn ? t : mn;
      mx = t > mx ? t : mx;
    }
    mn = row_block_min<NW>(mn, red, NWV);
    mx = row_block_max<NW>(mx, red, NWV);
    KAD_PT(t3);
    KAD_PADD(3, t3 - t2);

    // ---------------- select (framework.go:183-209, max_cluster.go:42-66)
    uint16_t* inv = nullptr;  // ranks after a replay (LDS or the block's slab)
    // mode: -1 nothing, 0 all, 1 total >= T, 3 replay ranks < k
    int mode = k >= n ? 0 : (k <= 0 ? -1 : 1);
    uint32_t rflags = 0;
    uint32_t Tk = 0;  // the k-th largest total, sign-flipped
    if (mode == 1) {
      const uint32_t base = (uint32_t)mn ^ 0x80000000u;
      const uint32_t span = (uint32_t)mx - (uint32_t)mn;
      uint32_t prefix = 0, pmask = 0;
      int kk = k;
      if (span != 0) {
        const int bits = 32 - __builtin_clz(span);
        // digits from the top: the first pass takes the span's top 8 bits (C5's totals span ~9 bits: 8-bit
        // digits aligned at bit 8 put every position into 2 bins, thousands of LDS atomics on two words)
        for (int hi = bits; hi > 0; hi -= 8) {
          const int shift = hi > 8 ? hi - 8 : 0;
          const uint32_t dmask = (1u << (hi - shift)) - 1u;
          for (int i = tid; i < 256; i += NTH) hist[i] = 0;  // (NTH >= 256 on every caller; any NTH is correct)
          __syncthreads();
          for (int j = tid; j < n; j += NTH) {
            const uint32_t d = key[j] - base;
            if ((d & pmask) == prefix) atomicAdd(&hist[(d >> shift) & dmask], 1u);
          }
          __syncthreads();
          if (wv == 0) {  // lane l owns digits 255-4l .. 252-4l (descending)
            int h[4], s4 = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              h[q] = (int)hist[255 - 4 * lane - q];
              s4 += h[q];
            }
            const int incl = wave_incl_sum_i32(s4);
            const int excl = incl - s4;
            if (excl < kk && kk <= incl) {
              int cum = excl;
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                if (cum + h[q] >= kk) {
                  bc[1] = 255 - 4 * lane - q;
                  bc[2] = cum;
                  break;
                }
                cum += h[q];
              }
            }
          }
          __syncthreads();
          const int digit = __builtin_amdgcn_readfirstlane(bc[1]), above = __builtin_amdgcn_readfirstlane(bc[2]);
          kk -= above;
          prefix |= (uint32_t)digit << shift;
          pmask |= dmask << shift;
        }
      }
      Tk = base + prefix;
      int g = 0, e = 0;
      for (int j = tid; j < n; j += NTH) {
        const uint32_t t = key[j];
        g += t > Tk;
        e += t == Tk;
      }
      g = row_block_sum<NW>(g, red, NWV);
      e = row_block_sum<NW>(e, red, NWV);
      KAD_PT(t4);
      KAD_PADD(4, t4 - t3);
      if (k - g != e) {  // ties straddle the cut: Go's pdqsort decides which tied clusters stay (n > 256)
        rflags = KAD_RF_TIE_STRADDLE;
        mode = 3;
        const bool in_lds = n <= ROW_NREP;
        const size_t Cp = (size_t)nch * 64;
        uint16_t* pid = in_lds ? pid_l : pid_g;
        uint16_t* posl = in_lds ? posl_l : pid_g + Cp;
        uint16_t* posr = in_lds ? posr_l : pid_g + 2 * Cp + 64;
        inv = posl;
        // packed replay (key - min << 16 | position: every C5 row, n <= C < 2^16) unless the totals span 2^16
        const bool packed = (uint32_t)mx - (uint32_t)mn < 65536u;
        for (int j = tid; j < n; j += NTH) {
          if (packed)
            key[j] = (((key[j] ^ 0x80000000u) - (uint32_t)mn) << 16) | (uint32_t)j;
          else
            pid[j] = (uint16_t)j;
        }
        __syncthreads();
        const int xs_b = (a->p.flags & KAD_PROFILE_XORSHIFT_GO121) ? 7 : 17;
        const int xs_c = (a->p.flags & KAD_PROFILE_XORSHIFT_GO121) ? 17 : 5;
        // packed: the partitions of ranges longer than ROW_BLOCK_PART run on all 8 waves, then wave 0 goes
        // on alone (red[] is free scratch here)
        did_pf = true;  // wave 1 prefetches the next unit while wave 0 finishes the replay alone
        if (packed && in_lds) {
          PdqWaveP<> pw{key, posl, posr, xs_b, xs_c};
          const auto st = pw.select_block(n, k, ROW_BLOCK_PART, NWV, wv, red);
          if (wv == 0) pw.select_from(st, k);
          else if (wv == 1) prefetch();
        } else if (packed) {  // elements stay in LDS; stopper scratch in the slab (workgroup fences order both)
          PdqWaveP<true> pw{key, posl, posr, xs_b, xs_c};
          const auto st = pw.select_block(n, k, ROW_BLOCK_PART, NWV, wv, red);
          if (wv == 0) pw.select_from(st, k);
          else if (wv == 1) prefetch();
        } else if (wv == 1) {
          prefetch();
        } else if (wv == 0) {
          if (in_lds) {
            PdqWave<uint32_t> pw{key, pid, posl, posr, xs_b, xs_c};
            pw.select(n, k);
          } else {  // keys stay in LDS; positions in the slab (workgroup-scope fences order both)
            PdqWave<uint32_t, true> pw{key, pid, posl, posr, xs_b, xs_c};
            pw.select(n, k);
          }
        }
        __syncthreads();
        for (int r = tid; r < n; r += NTH) inv[packed ? (key[r] & 0xFFFFu) : pid[r]] = (uint16_t)r;
        __syncthreads();
        KAD_PT(t5);
        KAD_PADD(5, t5 - t4);
      }
    }

    // ---------------- output, ascending cluster id (= ascending position)
    if (!did_pf && wv == 1) prefetch();  // (into the other buffers: the output pass uses this unit's cnt)
    const bool dup = fc & KAD_W_DUPLICATE;
    const bool replicas =
        !dup && a->p.replicas_plugin == KAD_PL_CLUSTER_CAPACITY_WEIGHT && (fc & REC_DESIRED_POS) && k > 0;
    int total = 0;
    if ((dup || replicas) && mode >= 0) {
      const int nq = (n + 63) >> 6;
      auto selected = [&](int p) -> bool {
        if (p >= n) return false;
        if (mode == 0) return true;
        if (mode == 1) return key[p] >= Tk;
        return inv[p] < k;
      };
      for (int q = wv; q < nq; q += NWV) {
        const uint64_t m = ballot(selected(q * WAVE + lane));
        if (lane == 0) cnt[q] = popc64(m);
      }
      __syncthreads();
      row_exclusive_scan(cnt, nq);
      __syncthreads();
      total = __builtin_amdgcn_readfirstlane(cnt[nq]);
      auto ao = rargs();
      int32_t* oc = ao->o.cluster + ooff;
      int64_t* orp = ao->o.replicas + ooff;
      for (int q = wv; q < nq; q += NWV) {
        const int p = q * WAVE + lane;
        const bool s = selected(p);
        const uint64_t m = ballot(s);
        if (s) {
          const uint32_t at = (uint32_t)(cnt[q] + mbcnt(m));
          stg(oc, at, (int32_t)idx[p]);
          stg(orp, at, (int64_t)(dup ? -1 : 0));
        }
      }
    }
    if (tid == 0) {
      auto ao = rargs();
      ao->o.status[w] = KAD_ST_OK;
      ao->o.count[w] = total;  // Divide without replicas plugin: empty map
      ao->o.flags[w] = rflags;
    }
  }
#ifdef KAD_PHASE_PROF
  // per-block (start, end, units) of the last launch in g_wavetime / g_wavex (the wide kernel's slots)
  if (tid == 0 && blockIdx.x < 8192) {
    g_wavetime[2 * blockIdx.x] = rt_start;
    g_wavetime[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    g_wavex[6 * blockIdx.x] = rt_units;
  }
#endif
  KAD_PFLUSH_ROW;
}

template <int SM>
__device__ __attribute__((noinline)) void wide_rows(char* smem, WArgs a) {
  row_units<SM, 0>([a] { return a; }, smem, 0);
}

template <int SM = -1>
__global__ __launch_bounds__(ROW_THREADS, KAD_ROW_MINW) void schedule_row_kernel(RowArgs args) {
  (void)args;  // read through rargs()
  extern __shared__ __attribute__((aligned(16))) char smem[];
#if defined(KAD_PHASE_PROF) || defined(KAD_TUNING)
  const int rexp = rargs()->exp;
#else
  constexpr int rexp = 0;
#endif
  row_units<SM, ROW_THREADS>([] { return rargs(); }, smem, rexp);
}

// ============================================================ plan kernel
struct PlanLayout {
  size_t cid, hash, w, mn, mx, cap, cur, fl, plan, over, ofl, w2, mx2, adj, plan2, over2, ofl2, ord, act, act2, bytes;
};
__host__ __device__ inline PlanLayout plan_layout(int K) {
  const size_t Kp = (size_t)((K + 63) & ~63);
  PlanLayout L;
  size_t o = 0;
  auto take = [&](size_t n) {
    size_t r = o;
    o += (n + 15) & ~(size_t)15;
    return r;
  };
  L.w = take(8 * Kp);
  L.mn = take(8 * Kp);
  L.mx = take(8 * Kp);
  L.cap = take(8 * Kp);
  L.cur = take(8 * Kp);
  L.plan = take(8 * Kp);
  L.over = take(8 * Kp);
  L.w2 = take(8 * Kp);
  L.mx2 = take(8 * Kp);
  L.adj = take(8 * Kp);
  L.plan2 = take(8 * Kp);
  L.over2 = take(8 * Kp);
  L.cid = take(4 * Kp);
  L.hash = take(4 * Kp);
  L.fl = take(4 * Kp);
  L.ofl = take(4 * Kp);
  L.ofl2 = take(4 * Kp);
  L.ord = take(4 * Kp);
  L.act = take(4 * Kp);
  L.act2 = take(4 * Kp);
  L.bytes = o;
  return L;
}
size_t plan_wave_bytes(int K) { return plan_layout(K).bytes; }

__device__ PlanWs plan_ws(char* region, int K) {
  const PlanLayout L = plan_layout(K);
  PlanWs ws;
  ws.cid = (int32_t*)(region + L.cid);
  ws.hash = (uint32_t*)(region + L.hash);
  ws.w = (int64_t*)(region + L.w);
  ws.mn = (int64_t*)(region + L.mn);
  ws.mx = (int64_t*)(region + L.mx);
  ws.cap = (int64_t*)(region + L.cap);
  ws.cur = (int64_t*)(region + L.cur);
  ws.fl = (uint32_t*)(region + L.fl);
  ws.plan = (int64_t*)(region + L.plan);
  ws.over = (int64_t*)(region + L.over);
  ws.ofl = (uint32_t*)(region + L.ofl);
  ws.w2 = (int64_t*)(region + L.w2);
  ws.mx2 = (int64_t*)(region + L.mx2);
  ws.adj = (int64_t*)(region + L.adj);
  ws.plan2 = (int64_t*)(region + L.plan2);
  ws.over2 = (int64_t*)(region + L.over2);
  ws.ofl2 = (uint32_t*)(region + L.ofl2);
  ws.ord = (int32_t*)(region + L.ord);
  ws.act = (int32_t*)(region + L.act);
  ws.act2 = (int32_t*)(region + L.act2);
  return ws;
}

// binary search of cluster id c in a sorted CSR slice [lo, hi)
__device__ __forceinline__ int find_sorted(const int32_t* a, int lo, int hi, int c) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const int v = a[mid];
    if (v == c) return mid;
    if (v < c)
      lo = mid + 1;
    else
      hi = mid;
  }
  return -1;
}

// LANES: rows of K <= 64 only, the planner in registers (8 waves / SIMD: <= 64 VGPRs); else rows of
// K > 64 only, with the LDS / global-scratch workspace (GSCR). launch_plan runs the first and, when
// some row may exceed 64 clusters, the second; each skips the other's rows.
// PlanRowHdr of every planner row (once per batch upload): one lane per row
__global__ __launch_bounds__(256) void plan_hdr_kernel(BatchDev b, const int32_t* rows, int n_rows, PlanRowHdr* out) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n_rows) return;
  const int w = rows[r];
  PlanRowHdr h;
  h.w = w;
  h.flags = b.flags[w];
  h.off = b.out_off[w];
  h.slots = (int32_t)(b.out_off[w + 1] - b.out_off[w]);
  h.p0 = b.pref_off[w];
  h.p1 = b.pref_off[w + 1];
  h.c0 = b.cur_off[w];
  h.c1 = b.cur_off[w + 1];
  h.k0 = b.key_off[w];
  h.k1 = b.key_off[w + 1];
  h.pad = 0;
  h.desired = b.desired[w];
  h.pad2 = 0;
  out[r] = h;
}

template <bool GSCR, bool LANES>
__global__ __launch_bounds__(64, LANES ? 8 : 1) void plan_kernel(SnapDev s, BatchDev b, OutDev o, const PlanRowHdr* rows,
                                                                 int n_rows, int kmax, char* gscratch, int wave_bytes,
                                                                 int r_stride, int tbl_cp, const int32_t* list = nullptr,
                                                                 const int32_t* list_n = nullptr) {
  // list (LANES only): the rows plan_pair_kernel left to the 64-lane planner (32 < K <= 64): row list[i] for
  // i < *list_n instead of row i
  if (list) n_rows = __hip_atomic_load(list_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = lane_id_h();
  const int gw = blockIdx.x;
  // LDS: the row workspace of rows with K > 64 (kmax > 64 only), then the lookup tables
  char* region = GSCR ? gscratch + (size_t)gw * wave_bytes : smem;
  const size_t ws_bytes = (GSCR || LANES || kmax <= WAVE) ? 0 : plan_layout(kmax).bytes;
  // cluster id → (row tag << 16 | preference / current-cluster index + 1) lookup tables in LDS
  // (tbl_cp > 0), written per row and never cleared: an entry counts only with the row's tag (the wave's
  // row counter; the tables are zeroed when it wraps). Replaces two binary searches in global memory per
  // selected cluster.
  uint32_t* tbl_p = (uint32_t*)(smem + ws_bytes);
  uint32_t* tbl_c = tbl_p + tbl_cp;
  uint64_t* kbuf = LANES ? (uint64_t*)(smem + ws_bytes + (size_t)tbl_cp * 8) : nullptr;  // sort keys (64)
  const bool use_tbl = !GSCR && tbl_cp > 0;
  uint32_t tag = 0;
  if (use_tbl) {  // LDS starts undefined: no entry may carry a tag before its row writes it
    for (int i = lane; i < 2 * tbl_cp; i += WAVE) tbl_p[i] = 0;
    wsync<GSCR>();
  }
  KAD_PACC;
  // XCD-aware row ranges (grid a multiple of 8; blocks go round-robin over the 8 XCDs): the blocks of XCD
  // x walk the x-th contiguous eighth of the rows, so neighbouring rows — which share the cache lines of
  // the per-unit columns (status, count, flags, headers, slot ids, preference columns) — are read through
  // one L2 instead of once by each XCD's L2 (C4: FETCH_SIZE per launch 1.09 -> 0.54 GB, time unchanged)
  int r_lo = gw, r_hi = n_rows, r_st = r_stride;
  if ((r_stride & 7) == 0 && r_stride >= 8) {
    const int x = gw & 7;
    r_lo = (int)((int64_t)n_rows * x / 8) + (gw >> 3);
    r_hi = (int)((int64_t)n_rows * (x + 1) / 8);
    r_st = r_stride >> 3;
  }
  // the row's PlanRowHdr in lanes 0..15 (one 64-B line), loaded one row ahead
  auto fetch_hdr = [&](int r) -> uint32_t {
    if (r >= r_hi) return 0u;
    const int rr = list ? ldc(list + r) : r;
    return lane < 16 ? ldg((const uint32_t*)(rows + rr), (uint32_t)lane) : 0u;
  };
  uint32_t hn = fetch_hdr(r_lo);
  for (int r = r_lo; r < r_hi; r += r_st) {
    KAD_PT(t0);
    const uint32_t hc = hn;
    hn = fetch_hdr(r + r_st);
    auto hf = [&](int d) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)hc, d); };
    const int w = (int)hf(0);
    const uint32_t f = hf(1);
    const int64_t off = (int64_t)(((uint64_t)hf(3) << 32) | hf(2));
    const int slots = (int)hf(4);
    const int p0 = (int)hf(5), p1 = (int)hf(6);
    const int c0 = (int)hf(7), c1 = (int)hf(8);
    const int ko0 = (int)hf(9), ko1 = (int)hf(10);
    const int64_t desired = (int64_t)(((uint64_t)hf(13) << 32) | hf(12));
    // everything this row reads next issues together (one memory round trip): the schedule stage's status,
    // count and flags, the unit's slot ids (within its bound, whatever the count), key bytes, and (K <= 64)
    // the preference / current-cluster ids for the lookup tables
    const int st = o.status[w];
    const int K = o.count[w];
    const uint32_t rflags0 = o.flags[w];
    const uint8_t* key = b.key + ko0;
    const int klen = ko1 - ko0;
    // su.Key() bytes in lanes (uniform): the FNV-1 continuation of every element
    // reads them with v_readlane instead of one dependent load per byte
    const uint32_t kb0 = lane < klen ? (uint32_t)key[lane] : 0u;
    int c_l = 0;
    if (LANES && slots > 0) c_l = o.cluster[off + (lane < slots ? lane : 0)];  // (no slot: nothing to read)
    // the lookup tables' first 64 preference / current-cluster ids (uniform guards, clamped lanes: no
    // exec branch), so that the name hashes and the preference columns below share the next round trip
    int pid_l = 0, cid_l = 0;
    if (use_tbl && p1 > p0) pid_l = b.pref_id[p0 + (p0 + lane < p1 ? lane : 0)];
    if (use_tbl && c1 > c0) cid_l = b.cur_id[c0 + (c0 + lane < c1 ? lane : 0)];
    if (st != KAD_ST_OK || K <= 0 || (K <= WAVE) != LANES) continue;
    const int64_t total = (f & KAD_W_HAS_DESIRED) ? desired : 0;
    // rows of K <= 64: element `lane`'s name hash (and cores) are loaded before the lookup tables are
    // filled, so those loads and the tables' index loads share one memory round trip
    uint32_t h_l = 0;
    int64_t ac_l = 0, av_l = 0;  // cores for dynamic weights (rsp.go:183-272)
    if constexpr (LANES) {
      const int first_c = __builtin_amdgcn_readfirstlane(c_l);  // (every lane active: lane 0 holds element 0)
      if (lane >= K) c_l = first_c;  // past K: element 0 (masked off later)
      h_l = s.name_fnv[c_l];
      if (f & KAD_W_DYNAMIC_WEIGHTS) {
        ac_l = s.alloc_cores[c_l];
        av_l = s.avail_cores[c_l];
      }
    }
    // preferences (rsp.go:99-126)
    if (use_tbl) {
      tag = (tag + 1) & 0xFFFFu;
      if (tag == 0) {  // wrapped: no stale entry may carry a live tag
        for (int i = lane; i < 2 * tbl_cp; i += WAVE) tbl_p[i] = 0;
        wsync<GSCR>();
        tag = 1;
      }
      if (p0 + lane < p1) tbl_p[pid_l] = (tag << 16) | (uint32_t)(lane + 1);
      if (c0 + lane < c1) tbl_c[cid_l] = (tag << 16) | (uint32_t)(lane + 1);
      for (int j = p0 + WAVE + lane; j < p1; j += WAVE) tbl_p[b.pref_id[j]] = (tag << 16) | (uint32_t)(j - p0 + 1);
      for (int j = c0 + WAVE + lane; j < c1; j += WAVE) tbl_c[b.cur_id[j]] = (tag << 16) | (uint32_t)(j - c0 + 1);
      wsync<GSCR>();
    }
    // element i: cluster id, hash, preference columns, current replicas
    auto gather = [&](int i, int& c, PlanLane& e) {
      uint32_t h;
      if constexpr (LANES) {
        c = c_l;  // i == lane (or 0 past K)
        h = h_l;
      } else {
        c = o.cluster[off + i];
        h = s.name_fnv[c];
      }
      int pi, ci;
      if (use_tbl) {
        const uint32_t tp = tbl_p[c], tc = tbl_c[c];
        pi = (tp >> 16) == tag ? p0 + (int)(tp & 0xFFFFu) - 1 : -1;
        ci = (tc >> 16) == tag ? c0 + (int)(tc & 0xFFFFu) - 1 : -1;
      } else {
        pi = find_sorted(b.pref_id, p0, p1, c);
        ci = find_sorted(b.cur_id, c0, c1, c);
      }
      e.fl = 0;
      e.w = e.mn = e.mx = e.cap = 0;
      if (pi >= 0) {
        // all five columns in one round trip (pi is in bounds), flags select after
        const uint32_t pf = b.pref_fl[pi];
        int64_t pw, pmx, pcp;
        if (b.pref_narrow) {  // i32 columns (KAD_BATCH_NARROW_PREFS)
          pw = b.pref_w32[pi];
          pmx = b.pref_max32[pi];
          pcp = b.pref_cap32[pi];
          e.mn = b.pref_min32[pi];
        } else {
          pw = b.pref_w[pi];
          pmx = b.pref_max[pi];
          pcp = b.pref_cap[pi];
          e.mn = b.pref_min[pi];
        }
        if (pf & KAD_PREF_HAS_WEIGHT) e.w = pw;
        if (pf & KAD_PREF_HAS_MAX) {
          e.fl |= EF_HAS_MAX;
          e.mx = pmx;
        }
        if (pf & KAD_PREF_HAS_CAP) {
          e.fl |= EF_HAS_CAP;
          e.cap = pcp;
        }
      }
      e.cur = ci >= 0 ? b.cur_rep[ci] : 0;
      // the FNV-1 continuation after the column loads are issued: the name hash's load and theirs share
      // one round trip
      for (int k0 = 0; k0 < klen; k0 += WAVE) {
        const uint32_t kb = k0 == 0 ? kb0 : (k0 + lane < klen ? (uint32_t)key[k0 + lane] : 0u);
        const int m = klen - k0 < WAVE ? klen - k0 : WAVE;
        for (int q = 0; q < m; ++q) {
          h *= 16777619u;
          h ^= (uint32_t)__builtin_amdgcn_readlane((int)kb, q);
        }
      }
      e.hash = h;
    };
    const bool avoid = f & KAD_W_AVOID_DISRUPTION;
    const bool keep = f & KAD_W_KEEP_UNSCHED;
    uint32_t rflags = rflags0;
    if constexpr (LANES) {
      // ---------------- one element per lane, the planner in registers (kad_plan.h plan_row_lanes)
      const bool v = lane < K;
      // every lane runs the gather (its FNV loop reads the key bytes of all lanes with v_readlane, so the
      // lanes that hold them must be live); lanes past K take element 0 and are masked off
      int c = 0;
      PlanLane e;
      gather(v ? lane : 0, c, e);
      if (!v) {
        e = PlanLane{0, 0, 0, 0, 0, 0u, 0u};
        c = 0;
      }
      wsync<GSCR>();  // the next row's table writes follow this row's reads
      KAD_PT(t1);
      KAD_PADD(0, t1 - t0);
      KAD_PADD(5, 1);
      if (f & KAD_W_DYNAMIC_WEIGHTS) {
        // CalcWeightLimit (rsp.go:183-213) + AvailableToPercentage (rsp.go:215-272)
        const int64_t ac = v ? ac_l : 0, av = v ? av_l : 0;
        const double sum = wave_sum_f64(v ? (double)ac : 0.0);
        const double suma = wave_sum_f64((v && av > 0) ? (double)av : 0.0);
        if (suma == 0) {
          e.w = v ? go_f2i(round(1000.0 / (double)K)) : 0;
        } else {
          const int64_t lim = sum == 0 ? go_f2i(round(1000.0 / (double)K))
                                       : go_f2i(round((double)ac / sum * 1000.0 * 1.4));
          const double avd = av < 0 ? 0.0 : (double)av;
          int64_t wt = go_f2i(round(avd / suma * 1000.0));
          if (wt > lim) wt = lim;
          const int64_t sumtmp = wave_sum_i64(v ? wt : 0);
          wt = go_f2i(round((double)wt / (double)sumtmp * 1000.0));
          const int64_t other = wave_sum_i64(v ? wt : 0);
          const int64_t maxw = wave_max_i64(v ? wt : 0);
          e.w = v ? wt : 0;
          if (maxw > 0) {  // remainder → first strict maximum (lowest cluster id among ties)
            const uint64_t tm = ballot(v && wt == maxw);
            const int first = (int)__builtin_ctzll(tm);
            if (popc64(tm) > 1) rflags |= KAD_RF_REMAINDER_TIE;
            if (lane == first) e.w = wadd(e.w, wsub(1000, other));
          }
        }
      }
      KAD_PT(t2);
      KAD_PADD(1, t2 - t1);
      PlanOut po;
      rflags |= plan_row_lanes(e, K, total, avoid, keep, po, kbuf);
      KAD_PT(t3);
      KAD_PADD(2, t3 - t2);
      // result = plan + overflow, zeros dropped (rsp.go:162-179), ascending cluster id
      const int64_t rr = v ? wadd(po.plan, (po.ofl & EF_HAS_OVER) ? po.over : 0) : 0;
      const bool nz = v && rr != 0;
      const uint64_t m = ballot(nz);
      if (nz) {
        const int64_t at = off + mbcnt(m);
        o.cluster[at] = c;
        o.replicas[at] = rr;
      }
      if (lane == 0) {
        o.count[w] = popc64(m);
        o.flags[w] = rflags;
      }
      KAD_PT(t4);
      KAD_PADD(3, t4 - t3);
      continue;
    } else {
    // ---------------- K > 64: the row state in the LDS / global-scratch workspace (kad_plan.h plan_row)
    PlanWs ws = plan_ws(region, K);
    for (int i0 = 0; i0 < K; i0 += WAVE) {
      const int i = i0 + lane;
      int c;
      PlanLane e;
      gather(i < K ? i : 0, c, e);  // every lane (see the K <= 64 path)
      if (i < K) {
        ws.cid[i] = c;
        ws.hash[i] = e.hash;
        ws.w[i] = e.w;
        ws.mn[i] = e.mn;
        ws.mx[i] = e.mx;
        ws.cap[i] = e.cap;
        ws.fl[i] = e.fl;
        ws.cur[i] = e.cur;
      }
    }
    wsync<GSCR>();
    KAD_PT(t1);
    KAD_PADD(0, t1 - t0);
    KAD_PADD(5, 1);
    if (f & KAD_W_DYNAMIC_WEIGHTS) {
      // CalcWeightLimit (rsp.go:183-213) + AvailableToPercentage (rsp.go:215-272)
      double sum = 0.0, suma = 0.0;
      for (int i = lane; i < K; i += WAVE) {
        const int c = ws.cid[i];
        sum += (double)s.alloc_cores[c];
        const int64_t av = s.avail_cores[c];
        if (av > 0) suma += (double)av;
      }
      sum = wave_sum_f64(sum);
      suma = wave_sum_f64(suma);
      if (suma == 0) {
        const int64_t even = go_f2i(round(1000.0 / (double)K));
        for (int i = lane; i < K; i += WAVE) ws.w[i] = even;
      } else {
        int64_t sumtmp = 0;
        for (int i = lane; i < K; i += WAVE) {
          const int c = ws.cid[i];
          const int64_t lim = sum == 0 ? go_f2i(round(1000.0 / (double)K))
                                       : go_f2i(round((double)s.alloc_cores[c] / sum * 1000.0 * 1.4));
          double v = (double)s.avail_cores[c];
          if (v < 0.0) v = 0.0;
          int64_t wt = go_f2i(round(v / suma * 1000.0));
          if (wt > lim) wt = lim;
          ws.w[i] = wt;
          sumtmp = wadd(sumtmp, wt);
        }
        sumtmp = wave_sum_i64(sumtmp);
        int64_t other = 0, maxw = 0;
        for (int i = lane; i < K; i += WAVE) {
          const int64_t wt = go_f2i(round((double)ws.w[i] / (double)sumtmp * 1000.0));
          ws.w[i] = wt;
          other = wadd(other, wt);
          maxw = wt > maxw ? wt : maxw;
        }
        other = wave_sum_i64(other);
        maxw = wave_max_i64(maxw);
        wsync<GSCR>();
        if (maxw > 0) {  // remainder → first strict maximum (lowest cluster id among ties)
          int first = K, ties = 0;
          for (int i = lane; i < K; i += WAVE) {
            if (ws.w[i] == maxw) {
              first = i < first ? i : first;
              ties++;
            }
          }
          for (int m = 32; m >= 1; m >>= 1) {
            const int of = __shfl_xor(first, m);
            first = of < first ? of : first;
          }
          ties = wave_sum_i32(ties);
          if (ties > 1) rflags |= KAD_RF_REMAINDER_TIE;
          if (lane == 0) ws.w[first] = wadd(ws.w[first], wsub(1000, other));
        }
      }
      wsync<GSCR>();
    }
    KAD_PT(t2);
    KAD_PADD(1, t2 - t1);
    rflags |= plan_row<GSCR>(ws, K, total, avoid, keep);
    KAD_PT(t3);
    KAD_PADD(2, t3 - t2);
    // result = plan + overflow, zeros dropped (rsp.go:162-179), ascending cluster id
    int base = 0;
    for (int i0 = 0; i0 < K; i0 += WAVE) {
      const int i = i0 + lane;
      int64_t r = 0;
      if (i < K) r = wadd(ws.plan[i], (ws.ofl[i] & EF_HAS_OVER) ? ws.over[i] : 0);
      const bool nz = i < K && r != 0;
      const uint64_t m = ballot(nz);
      if (nz) {
        const int64_t at = off + base + mbcnt(m);
        o.cluster[at] = ws.cid[i];
        o.replicas[at] = r;
      }
      base += popc64(m);
    }
    if (lane == 0) {
      o.count[w] = base;
      o.flags[w] = rflags;
    }
    wsync<GSCR>();
    KAD_PT(t4);
    KAD_PADD(3, t4 - t3);
    }
  }
  KAD_PFLUSH_PLAN;
}

// plan_pair_kernel — rows of K <= 32, two per wave (kad_plan.h plan_row_pair): row A (the wave's r-th row) in
// lanes 0-31, row B (the next row of its range) in lanes 32-63; C4's rows hold 15 selected clusters on
// average, so the 64-lane planner (one row per wave) left three quarters of its lanes idle. The same steps as
// plan_kernel<false, true> per segment: the row's header line, the schedule stage's status / count / flags,
// the slot ids, key bytes and preference / current-cluster ids in one round trip; name hashes and cores; the
// lookup tables (u16 per segment: (tag << 10) | (index + 1), rows of more than 1022 ids search the sorted
// lists instead); the preference columns; the FNV-1 continuation; dynamic weights; the plan. Rows with
// 32 < K <= 64 go to `big` (plan_kernel<false, true> runs them next); K > 64 rows are the workspace planner's.
#ifndef KAD_PAIR_MINW
#define KAD_PAIR_MINW 6  // waves per SIMD plan_pair_kernel's VGPR budget is sized for (6: 80 VGPRs; 8 spills, 5 / 7
                         // slower: profiles/r06/ab_c4_pair_planner.txt, ab_c4_planner_occupancy_classes.txt)
#endif
__global__ __launch_bounds__(64, KAD_PAIR_MINW) void plan_pair_kernel(SnapDev s, BatchDev b, OutDev o, const PlanRowHdr* rows,
                                                          int n_rows, int r_stride, int tbl_cp, int32_t* big,
                                                          int32_t* big_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = lane_id_h();
  const int sl = lane & 31;
  const bool hi = lane >= 32;
  const int gw = blockIdx.x;
  uint16_t* const tbl = (uint16_t*)smem;  // [kind: pref, cur][segment][tbl_cp]
  uint16_t* const tbl_p = tbl + (hi ? tbl_cp : 0);
  uint16_t* const tbl_c = tbl + 2 * (size_t)tbl_cp + (hi ? tbl_cp : 0);
  uint64_t* const kbuf = (uint64_t*)(smem + (size_t)tbl_cp * 8);
  const bool use_tbl = tbl_cp > 0;
  constexpr int TAG_MAX = 63, IDX_MAX = 1022;
  uint32_t tag = 0;
  auto clear_tables = [&]() {
    for (int i = lane; i < 2 * tbl_cp; i += WAVE) ((uint32_t*)tbl)[i] = 0u;  // 4 tables of tbl_cp u16
    wave_sync();
  };
  if (use_tbl) clear_tables();
  int r_lo = gw, r_hi = n_rows, r_st = r_stride;
  if ((r_stride & 7) == 0 && r_stride >= 8) {  // XCD-contiguous ranges (plan_kernel)
    const int x = gw & 7;
    r_lo = (int)((int64_t)n_rows * x / 8) + (gw >> 3);
    r_hi = (int)((int64_t)n_rows * (x + 1) / 8);
    r_st = r_stride >> 3;
  }
  for (int r = r_lo; r < r_hi; r += 2 * r_st) {
    const int rr = hi ? r + r_st : r;  // this segment's row
    const bool has = rr < r_hi;
    const uint32_t hc = (has && sl < 16) ? ldg((const uint32_t*)(rows + rr), (uint32_t)sl) : 0u;
    auto hf = [&](int d) -> uint32_t { return (uint32_t)seg_read32((int)hc, d); };
    const int w = has ? (int)hf(0) : 0;
    const uint32_t f = hf(1);
    const int64_t off = (int64_t)(((uint64_t)hf(3) << 32) | hf(2));
    const int p0 = (int)hf(5), p1 = (int)hf(6);
    const int c0 = (int)hf(7), c1 = (int)hf(8);
    const int ko0 = (int)hf(9), ko1 = (int)hf(10);
    const int64_t desired = (int64_t)(((uint64_t)hf(13) << 32) | hf(12));
    // the schedule stage's outputs, the slot ids, key bytes and the first 32 preference / current ids together
    const int st = has ? o.status[w] : -1;
    const int Kr = has ? o.count[w] : 0;
    const uint32_t rflags0 = has ? o.flags[w] : 0u;
    const int klen = ko1 - ko0;
    const bool ok = st == KAD_ST_OK && Kr > 0;
    const bool pok = ok && Kr <= 32;
    const int K = pok ? Kr : 0;
    const uint8_t* key = b.key + ko0;
    const uint32_t kb0 = (pok && sl < klen) ? (uint32_t)key[sl] : 0u;
    int c_l = pok ? o.cluster[off + (sl < K ? sl : 0)] : 0;
    const bool tbl_row = use_tbl && p1 - p0 <= IDX_MAX && c1 - c0 <= IDX_MAX;
    int pid_l = 0, cid_l = 0;
    if (pok && tbl_row && p1 > p0) pid_l = b.pref_id[p0 + (p0 + sl < p1 ? sl : 0)];
    if (pok && tbl_row && c1 > c0) cid_l = b.cur_id[c0 + (c0 + sl < c1 ? sl : 0)];
    if (ok && Kr > 32 && Kr <= WAVE && sl == 0) big[atomicAdd(big_n, 1)] = rr;  // the 64-lane planner's
    if (!ballot(pok)) continue;
    const int64_t total = (f & KAD_W_HAS_DESIRED) ? desired : 0;
    const bool dyn = f & KAD_W_DYNAMIC_WEIGHTS;
    const uint32_t h_l = s.name_fnv[c_l];
    int64_t ac_l = 0, av_l = 0;
    if (ballot(pok && dyn)) {
      ac_l = s.alloc_cores[c_l];
      av_l = s.avail_cores[c_l];
    }
    if (use_tbl) {
      if (++tag > TAG_MAX) {  // wrapped: no stale entry may carry a live tag
        clear_tables();
        tag = 1;
      }
      const uint16_t tg = (uint16_t)(tag << 10);
      if (pok && tbl_row) {
        if (p0 + sl < p1) tbl_p[pid_l] = (uint16_t)(tg | (sl + 1));
        if (c0 + sl < c1) tbl_c[cid_l] = (uint16_t)(tg | (sl + 1));
        for (int j = p0 + 32 + sl; j < p1; j += 32) tbl_p[b.pref_id[j]] = (uint16_t)(tg | (j - p0 + 1));
        for (int j = c0 + 32 + sl; j < c1; j += 32) tbl_c[b.cur_id[j]] = (uint16_t)(tg | (j - c0 + 1));
      }
      wave_sync();
    }
    // element sl of this segment's row (lanes past K: element 0, masked off below)
    const bool v = sl < K;
    const int c = c_l;
    PlanLane e;
    {
      int pi, ci;
      if (pok && tbl_row) {
        const uint32_t tp = tbl_p[c], tcc = tbl_c[c];
        pi = (tp >> 10) == tag ? p0 + (int)(tp & 1023u) - 1 : -1;
        ci = (tcc >> 10) == tag ? c0 + (int)(tcc & 1023u) - 1 : -1;
      } else if (pok) {
        pi = find_sorted(b.pref_id, p0, p1, c);
        ci = find_sorted(b.cur_id, c0, c1, c);
      } else {
        pi = ci = -1;
      }
      e.fl = 0;
      e.w = e.mn = e.mx = e.cap = 0;
      if (pi >= 0) {
        const uint32_t pf = b.pref_fl[pi];
        int64_t pw, pmx, pcp;
        if (b.pref_narrow) {
          pw = b.pref_w32[pi];
          pmx = b.pref_max32[pi];
          pcp = b.pref_cap32[pi];
          e.mn = b.pref_min32[pi];
        } else {
          pw = b.pref_w[pi];
          pmx = b.pref_max[pi];
          pcp = b.pref_cap[pi];
          e.mn = b.pref_min[pi];
        }
        if (pf & KAD_PREF_HAS_WEIGHT) e.w = pw;
        if (pf & KAD_PREF_HAS_MAX) {
          e.fl |= EF_HAS_MAX;
          e.mx = pmx;
        }
        if (pf & KAD_PREF_HAS_CAP) {
          e.fl |= EF_HAS_CAP;
          e.cap = pcp;
        }
      }
      e.cur = ci >= 0 ? b.cur_rep[ci] : 0;
      // FNV-1 continuation with su.Key() (planner.go:185-195): the segment's key bytes by readlane
      uint32_t h = h_l;
      const int kmax = wave_max_u_i32(pok ? klen : 0);
      for (int k0 = 0; k0 < kmax; k0 += 32) {
        const uint32_t kb = k0 == 0 ? kb0 : ((pok && k0 + sl < klen) ? (uint32_t)key[k0 + sl] : 0u);
        const int m = kmax - k0 < 32 ? kmax - k0 : 32;
        for (int q = 0; q < m; ++q) {
          const uint32_t byte = (uint32_t)seg_read32((int)kb, q);
          if (k0 + q < klen) h = (h * 16777619u) ^ byte;
        }
      }
      e.hash = h;
    }
    if (use_tbl) wave_sync();  // the next pair's table writes follow these reads
    if (!v) e = PlanLane{0, 0, 0, 0, 0, 0u, 0u};
    uint32_t rflags = rflags0;
    if (ballot(pok && dyn)) {
      // CalcWeightLimit (rsp.go:183-213) + AvailableToPercentage (rsp.go:215-272), per segment
      const int64_t ac = v ? ac_l : 0, av = v ? av_l : 0;
      const double sum = seg_sum_f64(v ? (double)ac : 0.0);
      const double suma = seg_sum_f64((v && av > 0) ? (double)av : 0.0);
      int64_t wdyn;
      uint32_t tf = 0;
      // (segment-uniform branches: a segment's reductions read only its own lanes, so the two segments may
      // take different ones)
      if (suma == 0) {
        wdyn = v ? go_f2i(round(1000.0 / (double)(K > 0 ? K : 1))) : 0;
      } else {
        const int64_t lim = sum == 0 ? go_f2i(round(1000.0 / (double)(K > 0 ? K : 1)))
                                     : go_f2i(round((double)ac / sum * 1000.0 * 1.4));
        const double avd = av < 0 ? 0.0 : (double)av;
        int64_t wt = go_f2i(round(avd / suma * 1000.0));
        if (wt > lim) wt = lim;
        const int64_t sumtmp = seg_sum_i64(v ? wt : 0);
        wt = go_f2i(round((double)wt / (double)sumtmp * 1000.0));
        const int64_t other = seg_sum_i64(v ? wt : 0);
        const int64_t maxw = seg_max_i64(v ? wt : 0);
        wdyn = v ? wt : 0;
        const uint32_t tm = seg_ballot(v && wt == maxw);
        if (maxw > 0) {  // remainder → first strict maximum (lowest cluster id among ties)
          const int first = (int)__builtin_ctz(tm | 0x80000000u);
          if (__builtin_popcount(tm) > 1) tf = KAD_RF_REMAINDER_TIE;
          if (sl == first) wdyn = wadd(wdyn, wsub(1000, other));
        }
      }
      if (dyn) {
        e.w = wdyn;
        rflags |= tf;
      }
    }
    PlanOut po;
    rflags |= plan_row_pair(e, K, total, (f & KAD_W_AVOID_DISRUPTION) != 0, (f & KAD_W_KEEP_UNSCHED) != 0, po, kbuf);
    // result = plan + overflow, zeros dropped (rsp.go:162-179), ascending cluster id
    const int64_t res = v ? wadd(po.plan, (po.ofl & EF_HAS_OVER) ? po.over : 0) : 0;
    const bool nz = v && res != 0;
    const uint32_t m = seg_ballot(nz);
    if (nz) {
      const int64_t at = off + seg_mbcnt(m);
      o.cluster[at] = c;
      o.replicas[at] = res;
    }
    if (pok && sl == 0) {
      o.count[w] = __builtin_popcount(m);
      o.flags[w] = rflags;
    }
  }
}

// ============================================= stand-alone stage entry points
template <bool GSCR>
__global__ __launch_bounds__(64) void select_rows_kernel(int n_rows, const int32_t* row_off, const int64_t* scores,
                                                         const int64_t* maxc, uint32_t pflags, int32_t* out_count,
                                                         int32_t* out_sel, int32_t* out_status, char* gscratch,
                                                         int wave_bytes, int kmax, int r_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = lane_id();
  char* region = GSCR ? gscratch + (size_t)blockIdx.x * wave_bytes : smem;
  const RowLayout L = row_layout(kmax);
  int64_t* tot = (int64_t*)(region + L.tot);
  uint16_t* perm = (uint16_t*)(region + L.perm);
  uint64_t* selb = (uint64_t*)(region + L.sel);
  uint32_t* hist = (uint32_t*)(region + L.hist);
  uint16_t* posl = (uint16_t*)(region + L.posl);
  uint16_t* posr = (uint16_t*)(region + L.posr);
  const int xs_b = (pflags & KAD_PROFILE_XORSHIFT_GO121) ? 7 : 17;
  const int xs_c = (pflags & KAD_PROFILE_XORSHIFT_GO121) ? 17 : 5;
  for (int r = blockIdx.x; r < n_rows; r += r_stride) {
    const int a = row_off[r], n = row_off[r + 1] - a;
    const int64_t mc = maxc[r];
    if (mc < 0) {
      if (lane == 0) {
        out_status[r] = KAD_ST_ERR_SELECT;
        out_count[r] = 0;
      }
      continue;
    }
    int64_t rmin = I64_MAX, rmax = I64_MIN;
    for (int j = lane; j < n; j += WAVE) {
      const int64_t t = scores[a + j];
      tot[j] = t;
      rmin = t < rmin ? t : rmin;
      rmax = t > rmax ? t : rmax;
    }
    rmin = wave_min_i64(rmin);
    rmax = wave_max_i64(rmax);
    wsync<GSCR>();
    const int64_t k = mc < n ? mc : n;
    SelWs ws{tot, selb, perm, hist, posl, posr};
    select_topk<GSCR>(ws, n, k, rmin, rmax, xs_b, xs_c);
    int base = 0;
    for (int jc = 0; jc < ((n + 63) >> 6); ++jc) {
      const uint64_t m = selb[jc];
      if ((m >> lane) & 1) out_sel[a + base + mbcnt(m)] = jc * WAVE + lane;
      base += popc64(m);
    }
    if (lane == 0) {
      out_status[r] = KAD_ST_OK;
      out_count[r] = base;
    }
    wsync<GSCR>();
  }
}

template <bool GSCR>
__global__ __launch_bounds__(64) void plan_rows_kernel(PlanRowsDev R, char* gscratch, int wave_bytes, int r_stride,
                                                       int force_ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = lane_id();
  char* region = GSCR ? gscratch + (size_t)blockIdx.x * wave_bytes : smem;
  // one row with the whole wave: the register planner for K <= 64 (plan_kernel's path), else (or with
  // force_ws == 1) the LDS-workspace planner
  auto one_row = [&](int r) {
    const int a = R.row_off[r], K = R.row_off[r + 1] - a;
    if (K <= 0) return;
    if (K <= WAVE && force_ws != 1) {
      const bool v = lane < K;
      PlanLane e{0, 0, 0, 0, 0, 0u, 0u};
      if (v) {
        e.hash = R.hash[a + lane];
        e.w = R.weight[a + lane];
        e.mn = R.min_r[a + lane];
        e.mx = R.max_r[a + lane];
        e.cap = R.cap[a + lane];
        e.cur = R.current[a + lane];
        e.fl = R.elem_flags[a + lane] & (EF_HAS_MAX | EF_HAS_CAP);
      }
      PlanOut po;
      plan_row_lanes(e, K, R.total[r], R.row_flags[r] & 1, (R.row_flags[r] >> 1) & 1, po);
      if (v) {
        R.out_plan[a + lane] = po.plan;
        R.out_overflow[a + lane] = (po.ofl & EF_HAS_OVER) ? po.over : -1;
      }
      return;
    }
    PlanWs ws = plan_ws(region, K);
    for (int i = lane; i < K; i += WAVE) {
      ws.cid[i] = i;
      ws.hash[i] = R.hash[a + i];
      ws.w[i] = R.weight[a + i];
      ws.mn[i] = R.min_r[a + i];
      ws.mx[i] = R.max_r[a + i];
      ws.cap[i] = R.cap[a + i];
      ws.cur[i] = R.current[a + i];
      ws.fl[i] = R.elem_flags[a + i] & (EF_HAS_MAX | EF_HAS_CAP);
    }
    wsync<GSCR>();
    plan_row<GSCR>(ws, K, R.total[r], R.row_flags[r] & 1, (R.row_flags[r] >> 1) & 1);
    for (int i = lane; i < K; i += WAVE) {
      R.out_plan[a + i] = ws.plan[i];
      R.out_overflow[a + i] = (ws.ofl[i] & EF_HAS_OVER) ? ws.over[i] : -1;
    }
    wsync<GSCR>();
  };
  if (force_ws == 2 && !GSCR) {  // rows r, r + 1 together in the two half-waves when both hold <= 32 elements (plan_row_pair)
    uint64_t* kbuf = (uint64_t*)region;
    const int sl = lane & 31;
    for (int r = 2 * (int)blockIdx.x; r < R.n_rows; r += 2 * r_stride) {
      const int KA = R.row_off[r + 1] - R.row_off[r];
      const int KB = r + 1 < R.n_rows ? R.row_off[r + 2] - R.row_off[r + 1] : 0;
      if (KA > 32 || KB > 32) {
        one_row(r);
        if (r + 1 < R.n_rows) one_row(r + 1);
        continue;
      }
      const int rr = lane >= 32 ? r + 1 : r;
      const int K = lane >= 32 ? KB : KA;
      const int a = rr < R.n_rows ? R.row_off[rr] : 0;
      const bool v = sl < K;
      PlanLane e{0, 0, 0, 0, 0, 0u, 0u};
      if (v) {
        e.hash = R.hash[a + sl];
        e.w = R.weight[a + sl];
        e.mn = R.min_r[a + sl];
        e.mx = R.max_r[a + sl];
        e.cap = R.cap[a + sl];
        e.cur = R.current[a + sl];
        e.fl = R.elem_flags[a + sl] & (EF_HAS_MAX | EF_HAS_CAP);
      }
      const uint32_t rf = K > 0 ? R.row_flags[rr] : 0u;
      PlanOut po;
      plan_row_pair(e, K, K > 0 ? R.total[rr] : 0, rf & 1, (rf >> 1) & 1, po, kbuf);
      if (v) {
        R.out_plan[a + sl] = po.plan;
        R.out_overflow[a + sl] = (po.ofl & EF_HAS_OVER) ? po.over : -1;
      }
    }
    return;
  }
  for (int r = blockIdx.x; r < R.n_rows; r += r_stride) one_row(r);
}

// ================================================================ launchers
int debug_phase_counters(uint64_t* out, int reset) {
#ifdef KAD_PHASE_PROF
  if (reset == -3 || reset == -4) {  // the wide kernel's per-unit trace: out holds 2^20 entries
    const hipError_t e = reset == -3 ? hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ustart), sizeof(unsigned long long) * KAD_UTRACE_MAX)
                                     : hipMemcpyFromSymbol(out, HIP_SYMBOL(g_uinfo), sizeof(unsigned long long) * KAD_UTRACE_MAX);
    return e == hipSuccess ? KAD_UTRACE_MAX : -1;
  }
  if (reset == -2) {  // the wide kernel's per-wave extras: out holds 8192 * 6 entries
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wavex), sizeof(unsigned long long) * 8192 * 6) != hipSuccess) return -1;
    return 8192;
  }
  if (reset < 0) {  // the lean kernel's per-wave (start, end) timestamps: out holds 8192 * 2 entries
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wavetime), sizeof(unsigned long long) * 8192 * 2) != hipSuccess) return -1;
    return 8192;
  }
  static unsigned long long h[256 * KAD_PSLOTS];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase), sizeof h) != hipSuccess) return -1;
  for (int i = 0; i < KAD_PSLOTS; ++i) {
    out[i] = 0;
    for (int s = 0; s < 256; ++s) out[i] += h[s * KAD_PSLOTS + i];
  }
  if (reset) {
    static const unsigned long long z[256 * KAD_PSLOTS] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z) != hipSuccess) return -1;
  }
  return KAD_PSLOTS;
#else
  (void)out;
  (void)reset;
  return 0;
#endif
}

static constexpr int MAX_RESIDENT_WAVES = 256 * 32;

hipError_t launch_req_masks(const SnapDev& s, const BatchDev& b, hipStream_t st, bool zero_rows, bool* zeroed) {
  (void)hipGetLastError();
  const int nch = (s.C + 63) >> 6;
  const long lanes = (long)b.n_rowreq * ((nch + REQ_RC - 1) / REQ_RC);
  *zeroed = zero_rows && lanes > 0;
  if (lanes > 0)
    hipLaunchKernelGGL(req_row_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, s, b, zero_rows ? 1 : 0);
  const int ngrp = (nch + REQ_G - 1) / REQ_G;
  const long waves = (long)b.n_seg * ngrp;
  if (waves > 0) hipLaunchKernelGGL(req_mask_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, s, b, ngrp);
  return hipGetLastError();
}

hipError_t launch_value_rows(const SnapDev& s, uint64_t* vrows, hipStream_t st) {
  (void)hipGetLastError();
  const long waves = (long)s.K * ((s.C + 63) >> 6);
  if (waves == 0) return hipSuccess;
  hipLaunchKernelGGL(value_rows_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, s, vrows);
  return hipGetLastError();
}

hipError_t launch_res_cols(const SnapDev& s, void* buf, hipStream_t st) {
  (void)hipGetLastError();
  if (s.C <= 0) return hipSuccess;
  double4* r4 = static_cast<double4*>(buf);
  ulonglong4* p4 = s.TW <= 4 ? reinterpret_cast<ulonglong4*>(static_cast<char*>(buf) + res_cols_pns4_offset(s.C)) : nullptr;
  hipLaunchKernelGGL(res_cols_kernel, dim3((unsigned)((s.C + 255) / 256)), dim3(256), 0, st, s, r4,
                     reinterpret_cast<float2*>(r4 + s.C), p4);
  return hipGetLastError();
}

hipError_t launch_slices(const SnapDev& s, uint64_t* slices, hipStream_t st) {
  (void)hipGetLastError();
  const int nch = (s.C + 63) >> 6;
  const long waves = (128L * s.TW + 64L * s.GW) * nch;
  if (waves == 0) return hipSuccess;
  hipLaunchKernelGGL(slice_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, s, slices);
  const long lanes = 2L * 8 * s.TW * 256 * nch;
  hipLaunchKernelGGL(taint_table_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, s,
                     slices + (128L * s.TW + 64L * s.GW) * nch);
  return hipGetLastError();
}

hipError_t launch_prep(const SnapDev& s, const BatchDev& b, const ProfDev& p, bool force_full, hipStream_t st) {
  (void)hipGetLastError();
  const int nch = (s.C + 63) >> 6;
  const long lanes = (long)b.W * (nch > 0 ? (nch + PREP_CPL - 1) / PREP_CPL : 1);
  const long grid = lanes > 0 ? (lanes + 255) / 256 : 1;  // one block at W = 0 still resets defer_n
  // wide snapshots (more than 64 chunks, up to 256): one unit per wave
  const int cw = (nch + 63) / 64;
  if (nch > 64 && cw <= 4 && tuning_env("KAD_PREP_WAVE", 1)) {
    // (not persistent: C5's one-unit-per-wave prep is L2-miss bound and took 587 -> 729 us with the resident
    // grid, profiles/r06/ab_c5_prep_persistent.txt)
    const long wgrid = b.W > 0 ? ((long)b.W + 3) / 4 : 1;
    const int ff = force_full ? 1 : 0;
    if (cw == 2) hipLaunchKernelGGL(prep_wave_kernel<2>, dim3((unsigned)wgrid), dim3(256), 0, st, s, b, p, ff);
    else if (cw == 3) hipLaunchKernelGGL(prep_wave_kernel<3>, dim3((unsigned)wgrid), dim3(256), 0, st, s, b, p, ff);
    else hipLaunchKernelGGL(prep_wave_kernel<4>, dim3((unsigned)wgrid), dim3(256), 0, st, s, b, p, ff);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(prep_kernel, dim3((unsigned)grid), dim3(256), 0, st, s, b, p, force_full ? 1 : 0);
  return hipGetLastError();
}

template <int NCH, bool CL, int SM = -1>
static void launch_lean(const LeanArgs& A, int grid, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((schedule_lean_kernel<NCH, CL, SM>), dim3(grid), dim3(64 * A.waves_per_block), lds, st, A);
}

static int n_cus() {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
  }
  return n_cu;
}

// the wide kernel takes clean snapshots with WIDE_MIN_NCH <= nch <= WIDE_MAX_NCH
// (KAD_WIDE_MIN_NCH overrides the lower bound, for A/B runs of C <= 256)
static bool use_wide(const SnapDev& s) {
  static int min_nch = -1;
  if (min_nch < 0) min_nch = tuning_env("KAD_WIDE_MIN_NCH", 5);
  const int nch = (s.C + 63) >> 6;
  return s.clean && nch >= min_nch && nch >= 1 && nch <= WIDE_MAX_NCH;
}
bool wide_path(const SnapDev& s) { return use_wide(s); }

static hipError_t launch_defer_pass(const SnapDev& s, const BatchDev& b, const OutDev& o, const ProfDev& p, void* gscr,
                                    size_t scr_bytes, hipStream_t st) {
  const size_t wb = row_layout(s.C).bytes;
  if (wb <= (size_t)LDS_BUDGET) {
    int wpb2 = (int)(LDS_BUDGET / wb);
    wpb2 = wpb2 > 4 ? 4 : (wpb2 < 1 ? 1 : wpb2);
    long waves2 = b.W < 256 * 16 ? b.W : 256 * 16;
    const int grid2 = (int)((waves2 + wpb2 - 1) / wpb2);
    const SchedArgs A2{s, b, o, p, nullptr, (int)wb, wpb2, grid2 * wpb2, b.defer, b.defer_n};
    hipLaunchKernelGGL(schedule_kernel<false>, dim3(grid2), dim3(64 * wpb2), wb * wpb2, st, A2);
  } else {  // rows too large for LDS: per-wave global scratch slabs
    size_t slots = scr_bytes / wb;
    if (slots < 1) return hipErrorInvalidValue;
    if (slots > (size_t)MAX_RESIDENT_WAVES) slots = MAX_RESIDENT_WAVES;
    if (slots > (size_t)b.W) slots = b.W;
    const SchedArgs A2{s, b, o, p, (char*)gscr, (int)wb, 1, (int)slots, b.defer, b.defer_n};
    hipLaunchKernelGGL(schedule_kernel<true>, dim3((int)slots), dim3(64), small_layout(s.C).bytes, st, A2);
  }
  return hipGetLastError();
}

// schedule_row_kernel over BatchDev::rows (its length is only known on the device: the persistent
// workgroups dequeue until the list is drained)
static hipError_t launch_rows(const SnapDev& s, const BatchDev& b, const OutDev& o, const ProfDev& p, hipStream_t st) {
  if (!b.use_rows) return hipSuccess;
  const size_t lds = row_kernel_lds(s.C);
  constexpr int SM_DEFAULT = (1 << KAD_PL_TAINT_TOLERATION) | (1 << KAD_PL_BALANCED_ALLOCATION) |
                             (1 << KAD_PL_LEAST_ALLOCATED) | (1 << KAD_PL_CLUSTER_AFFINITY);
  // the default plugin set's scores as constants (C5), else the generic kernel
  void (*fn)(RowArgs) = p.score_mask == (uint32_t)SM_DEFAULT ? schedule_row_kernel<SM_DEFAULT> : schedule_row_kernel<-1>;
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)schedule_row_kernel<SM_DEFAULT>, (const void*)schedule_row_kernel<-1>})
      if (hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)) return e;
    attr = true;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, ROW_THREADS, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  long grid = (long)n_cus() * per_cu;
  if (grid > ROW_MAX_BLOCKS) grid = ROW_MAX_BLOCKS;
  if (grid > b.W) grid = b.W;
  if (!b.row_slabs) return hipErrorInvalidValue;
  static const int exp = tuning_env("KAD_ROW_EXPERIMENT", 0);
  const RowArgs A{s, b, o, p, b.row_slabs, exp};
  hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(ROW_THREADS), lds, st, A);
  return hipGetLastError();
}

hipError_t launch_schedule(const SnapDev& s, const BatchDev& b, const OutDev& o, const ProfDev& p, void* gscr,
                           size_t scr_bytes, hipStream_t st, hipEvent_t after_main, hipEvent_t after_rows,
                           hipStream_t side, hipEvent_t fork, hipEvent_t join) {
  auto rec = [&](hipEvent_t ev) { return ev ? hipEventRecord(ev, st) : hipSuccess; };
  (void)hipGetLastError();  // clear any stale error so the check below is this launch's
  if (b.W == 0) return hipSuccess;
  const size_t wb = row_layout(s.C).bytes;
  if (use_wide(s)) {
    const int cache_ne = (p.filter_mask & (1u << KAD_PL_TAINT_TOLERATION)) && (b.flags_or & KAD_W_HAS_CURRENT);
    const int cache_pn = (p.score_mask >> KAD_PL_TAINT_TOLERATION) & 1;
    const size_t per_wave = wide_layout().bytes;
    const size_t lds_max = 160 * 1024;
    const bool s_res = p.score_mask & ((1u << KAD_PL_LEAST_ALLOCATED) | (1u << KAD_PL_MOST_ALLOCATED) |
                                       (1u << KAD_PL_BALANCED_ALLOCATION));
    // zero-request batches: the resource-score column, when it costs no wave (LDS beside the 16 wave regions)
    const int cache_zs = (KAD_WIDE_ZS && s_res && b.zero_req &&
                          wide_cache_bytes(s.C, cache_ne, cache_pn, 1) + (size_t)(WIDE_THREADS / 64) * per_wave <= lds_max)
                             ? 1
                             : 0;
    const size_t cache = wide_cache_bytes(s.C, cache_ne, cache_pn, cache_zs);
    int wpb = (int)((lds_max - cache) / per_wave);
    wpb = wpb > WIDE_THREADS / 64 ? WIDE_THREADS / 64 : wpb;
    if (wpb < 1) return hipErrorInvalidValue;
    const size_t lds = cache + (size_t)wpb * per_wave;
    // the instantiation: the score set of the bench profiles (C2/C3: LeastAllocated alone; C4: the default set,
    // also at its exact 8 chunks — 16 exact chunks unroll past the 128-VGPR budget and spill), else generic
    const int nch = (s.C + 63) >> 6;
    constexpr int SM_LEAST = 1 << KAD_PL_LEAST_ALLOCATED;
    constexpr int SM_DEFAULT = (1 << KAD_PL_TAINT_TOLERATION) | (1 << KAD_PL_BALANCED_ALLOCATION) |
                               (1 << KAD_PL_LEAST_ALLOCATED) | (1 << KAD_PL_CLUSTER_AFFINITY);
    const bool zr = cache_zs != 0;
    const void* fn = zr ? (const void*)schedule_wide_kernel<WIDE_MAX_NCH, 0, -1, true>
                        : (const void*)schedule_wide_kernel<WIDE_MAX_NCH, 0, -1>;
    const bool folded = s.fold && s.fitfold;  // the LeastAllocated specialisation compiles the folded filter only
    if (folded && nch == 16 && p.score_mask == (uint32_t)SM_LEAST)
      fn = zr ? (const void*)schedule_wide_kernel<WIDE_MAX_NCH, 0, SM_LEAST, true>
              : (const void*)schedule_wide_kernel<WIDE_MAX_NCH, 0, SM_LEAST>;
    else if (nch == 8 && p.score_mask == (uint32_t)SM_DEFAULT)
      fn = zr ? (const void*)schedule_wide_kernel<8, 8, SM_DEFAULT, true> : (const void*)schedule_wide_kernel<8, 8, SM_DEFAULT>;
    static bool attr = false;
    if (!attr) {
      for (const void* f : {(const void*)schedule_wide_kernel<WIDE_MAX_NCH, 0, -1>,
                            (const void*)schedule_wide_kernel<WIDE_MAX_NCH, 0, SM_LEAST>,
                            (const void*)schedule_wide_kernel<8, 8, SM_DEFAULT>,
                            (const void*)schedule_wide_kernel<WIDE_MAX_NCH, 0, -1, true>,
                            (const void*)schedule_wide_kernel<WIDE_MAX_NCH, 0, SM_LEAST, true>,
                            (const void*)schedule_wide_kernel<8, 8, SM_DEFAULT, true>})
        if (hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max)) return e;
      attr = true;
    }
    long grid = n_cus();
    const long need = ((long)b.W + wpb - 1) / wpb;
    if (grid > need) grid = need;
    static const int exp = tuning_env("KAD_WIDE_EXPERIMENT", 0);
    // the routed long units inside the wide kernel (its opening phase) when the row body's LDS fits below
    // the cluster cache; else the row kernel beside it on a second stream
    const int no_inline = tuning_env("KAD_ROWS_NO_INLINE", 0);  // (read per launch: tuning builds only)
    // (the row body needs >= 2 waves: wave 1 dequeues and prefetches while wave 0 replays)
    const bool inline_rows = b.early_rows && b.use_rows && !no_inline && wpb >= 2 &&
                             row_kernel_lds(s.C) <= (size_t)wpb * per_wave;
    // work-queue batch: 4 units, 3 when the waves take fewer than 64 units each (a 125k-unit shard: the last
    // batches are the tail; at 1M units 3-unit batches cost more in dequeue atomics than they save:
    // profiles/r05/ab_wide_batch_c3.txt)
    const long upw = ((long)b.W + grid * wpb - 1) / (grid * wpb);
    const int wbatch = upw < 64 ? 3 : WQ_BATCH;
    const WideArgs A{s, b, o, p, wpb, cache_ne, cache_pn, cache_zs, inline_rows ? 1 : 0, wbatch, exp};
    const bool beside = !inline_rows && b.early_rows && b.use_rows && side && fork && join;
    if (beside) {  // the row kernel on the side stream, from the end of prep_kernel, beside the wide kernel
      if (hipError_t e = hipEventRecord(fork, st)) return e;
      if (hipError_t e = hipStreamWaitEvent(side, fork, 0)) return e;
      if (hipError_t e = launch_rows(s, b, o, p, side)) return e;
      if (hipError_t e = hipEventRecord(join, side)) return e;
    }
    hipLaunchKernelGGL((void (*)(WideArgs))fn, dim3((unsigned)grid), dim3(64 * wpb), lds, st, A);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = rec(after_main);
    if (beside) {
      // joined even when the wide launch failed: the row kernel on the side stream must finish before
      // anything later on st (the next batch upload) can overwrite what it reads
      const hipError_t j = hipStreamWaitEvent(st, join, 0);
      if (e == hipSuccess) e = j;
    } else if (e == hipSuccess && !inline_rows) {
      e = launch_rows(s, b, o, p, st);
    }
    if (e != hipSuccess) return e;
    if (hipError_t e2 = rec(after_rows)) return e2;
    // the defer pass only when some unit can reach the defer list (BatchDev::may_defer, host-checked:
    // REC_FULL units, requests or affinity weights outside the exact path, rows with more preferred terms
    // than ROW_MAX_TERMS, or units past WIDE_P without early routing)
    if (!b.may_defer) return hipSuccess;
    return launch_defer_pass(s, b, o, p, gscr, scr_bytes, st);
  }
  if (fast_path(s.C)) {
    const int nch = (s.C + 63) >> 6;
    const size_t lb = lean_layout(s.C, lean_qmax(nch <= 4 ? nch : 0)).bytes;
    const int wpb = 4;
    // runs of consecutive units per wave: long enough to amortise the
    // register-resident cluster attributes, short enough that the grid is
    // many times the resident wave count
    const int cache_ne = (p.filter_mask & (1u << KAD_PL_TAINT_TOLERATION)) && (b.flags_or & KAD_W_HAS_CURRENT);
    const int cache_pn = (p.score_mask >> KAD_PL_TAINT_TOLERATION) & 1;
    const size_t lds = lb * wpb + (nch <= 4 ? lean_cache_bytes(s.C, 6 + cache_ne + cache_pn + ((s.clean && nch >= 1 && nch <= 4) ? 1 : 0)) : 0);
    // one wave per resident slot: contiguous equal shares, no tail of late blocks
    const int n_cu = n_cus();
    int per_cu = 0;
    hipError_t oe;
    const bool cl = s.clean && nch >= 1 && nch <= 4;
    // score-set specialisations of the bench profiles: C2 (4 clean chunks, LeastAllocated alone), C5 (long
    // lists, the default set)
    constexpr int SM_LEAST = 1 << KAD_PL_LEAST_ALLOCATED;
    constexpr int SM_DEFAULT = (1 << KAD_PL_TAINT_TOLERATION) | (1 << KAD_PL_BALANCED_ALLOCATION) |
                               (1 << KAD_PL_LEAST_ALLOCATED) | (1 << KAD_PL_CLUSTER_AFFINITY);
    const bool least4 = cl && nch == 4 && p.score_mask == (uint32_t)SM_LEAST;
    const bool def0 = nch > 4 && p.score_mask == (uint32_t)SM_DEFAULT;
#define KAD_OCC(N, B) hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, schedule_lean_kernel<N, B>, 64 * wpb, lds)
    switch (nch) {
      case 1: oe = cl ? KAD_OCC(1, true) : KAD_OCC(1, false); break;
      case 2: oe = cl ? KAD_OCC(2, true) : KAD_OCC(2, false); break;
      case 3: oe = cl ? KAD_OCC(3, true) : KAD_OCC(3, false); break;
      case 4:
        oe = least4 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, schedule_lean_kernel<4, true, SM_LEAST>,
                                                                    64 * wpb, lds)
                    : (cl ? KAD_OCC(4, true) : KAD_OCC(4, false));
        break;
      default:
        oe = def0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, schedule_lean_kernel<0, false, SM_DEFAULT>,
                                                                  64 * wpb, lds)
                  : KAD_OCC(0, false);
        break;
    }
#undef KAD_OCC
    if (oe != hipSuccess || per_cu < 1) per_cu = 1;
    per_cu = tuning_env("KAD_LEAN_BLOCKS_PER_CU", per_cu);
    long grid = (long)n_cu * per_cu;
    const long need = ((long)b.W + wpb - 1) / wpb;  // at least one unit per wave
    if (grid > need) grid = need;
    // units per work-queue batch: at most LEAN_BATCH (one VGPR of UnitRecs), small enough that every wave
    // takes >= 12 batches, so the waves run out of work together (C2: 16 units per wave → 1-unit batches)
    const long upw = ((long)b.W + grid * wpb - 1) / (grid * wpb);
    int bsz = (int)(upw / 6);
    bsz = bsz < 1 ? 1 : (bsz > LEAN_BATCH ? LEAN_BATCH : bsz);
    const LeanArgs A{s, b, o, p, (int)lb, wpb, bsz, cache_ne, cache_pn};
    switch (nch) {
      case 1: cl ? launch_lean<1, true>(A, (int)grid, lds, st) : launch_lean<1, false>(A, (int)grid, lds, st); break;
      case 2: cl ? launch_lean<2, true>(A, (int)grid, lds, st) : launch_lean<2, false>(A, (int)grid, lds, st); break;
      case 3: cl ? launch_lean<3, true>(A, (int)grid, lds, st) : launch_lean<3, false>(A, (int)grid, lds, st); break;
      case 4:
        if (least4)
          launch_lean<4, true, SM_LEAST>(A, (int)grid, lds, st);
        else
          cl ? launch_lean<4, true>(A, (int)grid, lds, st) : launch_lean<4, false>(A, (int)grid, lds, st);
        break;
      default: def0 ? launch_lean<0, false, SM_DEFAULT>(A, (int)grid, lds, st) : launch_lean<0, false>(A, (int)grid, lds, st); break;
    }
    if (hipError_t e = hipGetLastError()) return e;
    if (hipError_t e = rec(after_main)) return e;
    // nothing can be deferred (host-checked: every unit and cluster is in the
    // lean kernel's range and every feasible list fits its registers)
    if (nch <= 4 && !b.may_defer) return rec(after_rows);
    if (nch > 4)
      if (hipError_t e = launch_rows(s, b, o, p, st)) return e;
    if (hipError_t e = rec(after_rows)) return e;
    // the defer list: its length is only known on the device, so the grid
    // strides over it (waves past its end exit at once)
    return launch_defer_pass(s, b, o, p, gscr, scr_bytes, st);
  }
  if (wb <= (size_t)LDS_BUDGET) {
    int wpb = (int)(LDS_BUDGET / wb);
    wpb = wpb > 4 ? 4 : (wpb < 1 ? 1 : wpb);
    const int grid = (b.W + wpb - 1) / wpb;
    const SchedArgs A{s, b, o, p, nullptr, (int)wb, wpb, grid * wpb, nullptr, nullptr};
    hipLaunchKernelGGL(schedule_kernel<false>, dim3(grid), dim3(64 * wpb), wb * wpb, st, A);
  } else {
    size_t slots = scr_bytes / wb;
    if (slots < 1) return hipErrorInvalidValue;
    if (slots > (size_t)MAX_RESIDENT_WAVES) slots = MAX_RESIDENT_WAVES;
    if (slots > (size_t)b.W) slots = b.W;
    const int grid = (int)slots;
    const SchedArgs A{s, b, o, p, (char*)gscr, (int)wb, 1, grid, nullptr, nullptr};
    hipLaunchKernelGGL(schedule_kernel<true>, dim3(grid), dim3(64), small_layout(s.C).bytes, st, A);
  }
  return hipGetLastError();
}

hipError_t launch_plan_hdr(const BatchDev& b, const int32_t* rows, int n_rows, PlanRowHdr* out, hipStream_t st) {
  (void)hipGetLastError();
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(plan_hdr_kernel, dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, st, b, rows, n_rows, out);
  return hipGetLastError();
}

constexpr int PLAN_OVERSUB = 8;  // register planners' grid over the resident block count (launch_plan)
hipError_t launch_plan(const SnapDev& s, const BatchDev& b, const OutDev& o, const ProfDev& p, const PlanRowHdr* rows,
                       int n_rows, int kmax, void* gscr, size_t scr_bytes, hipStream_t st, int32_t* big, int32_t* big_n) {
  (void)hipGetLastError();  // clear any stale error so the check below is this launch's
  (void)p;
  if (n_rows == 0 || kmax <= 0) return hipSuccess;
  const int cp = (s.C + 63) & ~63;
  // grid: `over` times the resident block count, rows round-robin (r += grid). The pair planner takes up to
  // PLAN_OVERSUB = 8 (at least 16 rows per wave): each wave's rows are an eighth of a persistent wave's, and the
  // hardware starts the next waves as earlier ones finish — with a fixed stride per resident wave, the waves
  // whose rows held the most rounds set the kernel's end (C4: planner 1.463 -> 1.276 ms, step 2.29 -> 2.10 ms;
  // 16x equal, 32x / 64x slower: profiles/r06/ab_c4_plan_grid.txt). Small row sets (C5's) and the list kernel
  // (its rows are known on the device only) keep the resident grid: extra waves there only start and exit.
  auto persistent = [&](const void* fn, size_t lds, int over = 1) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, lds) != hipSuccess || per_cu < 1) per_cu = 8;
    const long res = (long)n_cus() * per_cu;
    long grid = res * over;
    if (over > 1 && grid > n_rows / 16) grid = n_rows / 16 > res ? n_rows / 16 : res;
    return (int)(grid > n_rows ? n_rows : grid);
  };
  static const int over = tuning_env("KAD_PLAN_GRID_MULT", PLAN_OVERSUB);
  // rows of K <= 64: the register planners, lookup tables only in LDS. Two rows per wave for K <= 32
  // (plan_pair_kernel: u16 tables, 8 B per cluster for the two segments), then the rows of 32 < K <= 64 it
  // listed, one per wave (plan_kernel<false, true>: u32 tables, 8 B per cluster)
  {
    const int tbl_cp = cp <= 1024 ? cp : 0;
    const size_t lds = (size_t)tbl_cp * 8 + 64 * 8;  // tables + sort keys
    static const int pairs = tuning_env("KAD_PLAN_PAIRS", 1);
    if (pairs && big) {
      if (hipError_t e = hipMemsetAsync(big_n, 0, sizeof(int32_t), st)) return e;
      const int grid = persistent((const void*)plan_pair_kernel, lds, over);
      hipLaunchKernelGGL(plan_pair_kernel, dim3((unsigned)grid), dim3(64), lds, st, s, b, o, rows, n_rows, grid, tbl_cp,
                         big, big_n);
      if (hipError_t e = hipGetLastError()) return e;
      const int grid2 = persistent((const void*)plan_kernel<false, true>, lds);
      hipLaunchKernelGGL((plan_kernel<false, true>), dim3((unsigned)grid2), dim3(64), lds, st, s, b, o, rows, n_rows,
                         kmax, (char*)nullptr, 0, grid2, tbl_cp, (const int32_t*)big, (const int32_t*)big_n);
    } else {
      const int grid = persistent((const void*)plan_kernel<false, true>, lds, over);
      hipLaunchKernelGGL((plan_kernel<false, true>), dim3((unsigned)grid), dim3(64), lds, st, s, b, o, rows, n_rows,
                         kmax, (char*)nullptr, 0, grid, tbl_cp, (const int32_t*)nullptr, (const int32_t*)nullptr);
    }
    if (hipError_t e = hipGetLastError()) return e;
  }
  if (kmax <= WAVE) return hipSuccess;
  // rows of K > 64: the workspace planner
  const size_t wb = plan_layout(kmax).bytes;
  // per-wave lookup tables (8 B per cluster) when they fit beside the row state
  const int tbl_cp = (cp <= 1024 && wb + (size_t)cp * 8 <= (size_t)LDS_BUDGET) ? cp : 0;
  const size_t wbt = wb + (size_t)tbl_cp * 8;
  if (wbt <= (size_t)LDS_BUDGET) {
    const int grid = persistent((const void*)plan_kernel<false, false>, wbt);
    hipLaunchKernelGGL((plan_kernel<false, false>), dim3((unsigned)grid), dim3(64), wbt, st, s, b, o, rows, n_rows,
                       kmax, (char*)nullptr, (int)wb, grid, tbl_cp);
  } else {
    size_t slots = scr_bytes / wb;
    if (slots < 1) return hipErrorInvalidValue;
    if (slots > (size_t)MAX_RESIDENT_WAVES) slots = MAX_RESIDENT_WAVES;
    if (slots > (size_t)n_rows) slots = n_rows;
    hipLaunchKernelGGL((plan_kernel<true, false>), dim3(slots), dim3(64), 0, st, s, b, o, rows, n_rows, kmax,
                       (char*)gscr, (int)wb, (int)slots, 0);
  }
  return hipGetLastError();
}

hipError_t launch_select_rows(int n_rows, const int32_t* row_off, const int64_t* scores, const int64_t* maxc,
                              uint32_t pflags, int kmax, int32_t* out_count, int32_t* out_sel, int32_t* out_status,
                              void* gscr, size_t scr_bytes, hipStream_t st) {
  (void)hipGetLastError();  // clear any stale error so the check below is this launch's
  if (n_rows == 0) return hipSuccess;
  const size_t wb = row_layout(kmax < 1 ? 1 : kmax).bytes;
  if (wb <= (size_t)LDS_BUDGET) {
    hipLaunchKernelGGL(select_rows_kernel<false>, dim3(n_rows), dim3(64), wb, st, n_rows, row_off, scores, maxc,
                       pflags, out_count, out_sel, out_status, (char*)nullptr, (int)wb, kmax < 1 ? 1 : kmax, n_rows);
  } else {
    size_t slots = scr_bytes / wb;
    if (slots < 1) return hipErrorInvalidValue;
    if (slots > (size_t)n_rows) slots = n_rows;
    hipLaunchKernelGGL(select_rows_kernel<true>, dim3(slots), dim3(64), 0, st, n_rows, row_off, scores, maxc, pflags,
                       out_count, out_sel, out_status, (char*)gscr, (int)wb, kmax, (int)slots);
  }
  return hipGetLastError();
}

hipError_t launch_plan_rows(const PlanRowsDev& r, int kmax, int force_ws, void* gscr, size_t scr_bytes,
                            hipStream_t st) {
  (void)hipGetLastError();  // clear any stale error so the check below is this launch's
  if (r.n_rows == 0 || kmax <= 0) return hipSuccess;
  const size_t wb = plan_layout(kmax).bytes;
  // force_ws (kad_debug_plan_force_workspace, tests): rows of K <= 64 through the LDS-workspace planner too
  if (wb <= (size_t)LDS_BUDGET) {
    hipLaunchKernelGGL(plan_rows_kernel<false>, dim3(r.n_rows), dim3(64), wb, st, r, (char*)nullptr, (int)wb,
                       r.n_rows, force_ws);
  } else {
    size_t slots = scr_bytes / wb;
    if (slots < 1) return hipErrorInvalidValue;
    if (slots > (size_t)r.n_rows) slots = r.n_rows;
    hipLaunchKernelGGL(plan_rows_kernel<true>, dim3(slots), dim3(64), 0, st, r, (char*)gscr, (int)wb, (int)slots,
                       force_ws);
  }
  return hipGetLastError();
}

}  // namespace kad

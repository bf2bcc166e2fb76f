// Divide-mode replica planning on one wavefront:
//   ClusterCapacityWeight.ReplicaScheduling (plugins/rsp/rsp.go:65-181) and
//   planner.Plan (pkg/controllers/util/planner/planner.go:83-366).
//
// The planner's loops are sequential in `remainingReplicas`, but every step is
// R ← R − min(min(e_i, R), V_i), i.e. R ← max(R − s_i, t_i) with
// (s, t) = (min(e_i, V_i), 0) or (min(e_i, V_i), −∞). These clamp functions
// compose associatively, (s1,t1)∘(s2,t2) = (s1+s2, max(t1−s2, t2)), so each
// pass over the sorted preferences is a wavefront prefix scan instead of a
// serial loop (SURVEY.md §7 hard part 5).
#pragma once
#include "kad_wave.h"

namespace kad {

constexpr uint32_t EF_HAS_MAX = 2u;
constexpr uint32_t EF_HAS_CAP = 4u;
constexpr uint32_t EF_HAS_OVER = 8u;   // overflow entry present
constexpr uint32_t EF_HAS_PLAN = 16u;  // plan entry present

struct Clamp {
  int64_t s, t;
};
__device__ __forceinline__ Clamp clamp_compose(Clamp a, Clamp b) {  // a then b
  Clamp r;
  r.s = wadd(a.s, b.s);
  int64_t at = a.t == NEG_INF ? NEG_INF : wsub(a.t, b.s);
  r.t = at > b.t ? at : b.t;
  return r;
}
__device__ __forceinline__ int64_t clamp_apply(Clamp f, int64_t R) {
  int64_t x = wsub(R, f.s);
  return x > f.t ? x : f.t;
}
// inclusive scan of clamp functions across the wave: DPP Hillis-Steele within
// 16-lane rows (row_shr 1/2/4/8), then row_bcast 15/31 across rows; lanes
// without a source combine with the identity (0, -inf). Every lane active.
template <int CTRL, int RM>
__device__ __forceinline__ Clamp dpp_clamp(Clamp v) {
  Clamp o;
  o.s = dpp64<CTRL, RM>(0, v.s);
  o.t = dpp64<CTRL, RM>(NEG_INF, v.t);
  return o;
}
__device__ __forceinline__ Clamp wave_scan_clamp(Clamp v) {
  v = clamp_compose(dpp_clamp<0x111, 0xf>(v), v);
  v = clamp_compose(dpp_clamp<0x112, 0xf>(v), v);
  v = clamp_compose(dpp_clamp<0x114, 0xf>(v), v);
  v = clamp_compose(dpp_clamp<0x118, 0xf>(v), v);
  v = clamp_compose(dpp_clamp<0x142, 0xa>(v), v);
  v = clamp_compose(dpp_clamp<0x143, 0xc>(v), v);
  return v;
}
// The same scan in 32 bits when the row is narrow (clamp_narrow: R and every
// |s| < 2^24, t in {0, -inf} — partial sums stay within 2^30 over 64 lanes, so
// no value wraps in either width and the results are identical): half the DPP
// moves and 32-bit compose. -inf is INT32_MIN in the narrow form.
constexpr int NEG32 = INT32_MIN;
constexpr int NEG30 = -(1 << 30);  // -inf of desired_plan_lanes32 (see there)
__device__ __forceinline__ bool clamp_narrow(Clamp f, int64_t R) {
  return R >= 0 && R < (1ll << 24) && !ballot(f.s <= -(1ll << 24) || f.s >= (1ll << 24));
}
#define KAD_CLAMP32_STEP(CTRL, RM)                                        \
  {                                                                       \
    const int ps = dpp32<CTRL, RM>(0, s), pt = dpp32<CTRL, RM>(NEG32, t); \
    const int at = pt == NEG32 ? NEG32 : pt - s;                          \
    t = at > t ? at : t;                                                  \
    s = ps + s;                                                           \
  }
__device__ __forceinline__ Clamp wave_scan_clamp_n(Clamp v, bool narrow) {
  if (!narrow) return wave_scan_clamp(v);
  int s = (int)v.s, t = v.t == NEG_INF ? NEG32 : (int)v.t;
  KAD_CLAMP32_STEP(0x111, 0xf)
  KAD_CLAMP32_STEP(0x112, 0xf)
  KAD_CLAMP32_STEP(0x114, 0xf)
  KAD_CLAMP32_STEP(0x118, 0xf)
  KAD_CLAMP32_STEP(0x142, 0xa)
  KAD_CLAMP32_STEP(0x143, 0xc)
  return Clamp{(int64_t)s, t == NEG32 ? NEG_INF : (int64_t)t};
}
#undef KAD_CLAMP32_STEP
// exclusive value: the inclusive scan shifted one lane up (wave_shr:1); lane 0 gets the identity
__device__ __forceinline__ Clamp wave_shr1_clamp(Clamp v) {
  Clamp o;
  o.s = dpp64<0x138, 0xf>(0, v.s);
  o.t = dpp64<0x138, 0xf>(NEG_INF, v.t);
  return o;
}
__device__ __forceinline__ Clamp readlane_clamp(Clamp v, int l) {
  Clamp o;
  o.s = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v.s >> 32), l) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v.s, l));
  o.t = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v.t >> 32), l) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v.t, l));
  return o;
}

// planner.go:249: extra = (remainingReplicas*weight + weightSum - 1) / weightSum
// (Go int64, truncating). For 0 <= the numerator < 2^52 and 0 < weightSum < 2^52
// an f64 quotient corrected twice with exact f64 products is the exact integer
// quotient (no 64-bit division sequence); otherwise the wrapping int64 path.
__device__ __forceinline__ int64_t ceil_extra(int64_t D, int64_t w, int64_t wsum) {
  const int64_t num = wsub(wadd(wmul(D, w), wsum), 1);
  const bool small = D >= 0 && D < (1ll << 26) && w >= 0 && w < (1ll << 26) && wsum > 0 && wsum < (1ll << 52);
  if (small && num >= 0 && num < (1ll << 52)) {
    const double nd = (double)num, sd = (double)wsum;
    int64_t q = (int64_t)(nd / sd);
    double r = nd - (double)q * sd;  // exact: q * sd <= nd + sd < 2^53
    q += (r >= sd) - (r < 0.0);
    r = nd - (double)q * sd;
    q += (r >= sd) - (r < 0.0);
    return q;
  }
  return go_div(num, wsum);
}

// ceil_extra with 1/weightSum precomputed (inv = 1.0 / wsum, wave-uniform): the f64 quotient estimate is
// within one of the truncated quotient, and the two exact corrections make it the integer quotient
__device__ __forceinline__ int64_t ceil_extra_inv(int64_t D, int64_t w, int64_t wsum, double inv) {
  const int64_t num = wsub(wadd(wmul(D, w), wsum), 1);
  const bool small = D >= 0 && D < (1ll << 26) && w >= 0 && w < (1ll << 26) && wsum > 0 && wsum < (1ll << 52);
  if (small && num >= 0 && num < (1ll << 52)) {
    const double nd = (double)num, sd = (double)wsum;
    int64_t q = (int64_t)(nd * inv);
    double r = nd - (double)q * sd;  // exact: q * sd <= nd + 2 sd < 2^53
    q += (r >= sd) - (r < 0.0);
    r = nd - (double)q * sd;
    q += (r >= sd) - (r < 0.0);
    return q;
  }
  return go_div(num, wsum);
}

// Per-wave planner workspace: arrays indexed by element (K elements).
struct PlanWs {
  int32_t* cid;    // snapshot cluster id (ascending) — or row position in kad_plan_rows
  uint32_t* hash;  // FNV-1 of name ‖ key
  int64_t* w;      // weight
  int64_t* mn;     // MinReplicas
  int64_t* mx;     // MaxReplicas (EF_HAS_MAX)
  int64_t* cap;    // estimated capacity (EF_HAS_CAP)
  int64_t* cur;    // current replicas
  uint32_t* fl;    // EF_* flags
  int64_t* plan;   // desired plan / result plan
  int64_t* over;   // overflow
  uint32_t* ofl;   // EF_HAS_OVER / EF_HAS_PLAN for the plan being built
  int64_t* w2;     // scale up/down weights
  int64_t* mx2;    // scale up/down max (I64_MAX = none)
  int64_t* adj;    // currentPlan
  int64_t* plan2;  // scale up/down plan
  int64_t* over2;  // scale up/down overflow (discarded by the reference)
  uint32_t* ofl2;
  int32_t* ord;    // sorted order
  int32_t* act;    // active list / compaction buffer
  int32_t* act2;
};

// sort elements in list[0..m) (element ids) by (weight desc, hash asc, id asc) into ord;
// returns true if two elements tie on (weight, hash) (Go order would be map-order dependent).
template <bool GSCR>
__device__ bool sort_by_weight_hash(const PlanWs& ws, const int64_t* wt, const int32_t* list, int m) {
  const int lane = lane_id_h();
  if (m <= WAVE) {  // one element per lane: compare against the others with v_readlane, no memory
    const int e = lane < m ? list[lane] : 0;
    const int64_t we = lane < m ? wt[e] : 0;
    const uint32_t he = lane < m ? ws.hash[e] : 0u;
    int rank = 0;
    bool tie = false;
    if (!ballot(lane < m && (we < 0 || we > 0x7FFFFFFF))) {
      // every weight in [0, 2^31): (weight desc, hash asc) as one ascending u64
      // key, so each step is two readlanes and one 64-bit compare per order
      const uint64_t ke = ((uint64_t)(uint32_t)(0x7FFFFFFF - (int)we) << 32) | he;
      for (int j = 0; j < m; j++) {
        const int f = __builtin_amdgcn_readlane(e, j);
        const uint64_t kf = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ke >> 32), j) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ke, j);
        rank += kf < ke || (kf == ke && f < e);
        tie |= (j != lane && kf == ke);
      }
      wsync<GSCR>();
      if (lane < m) ws.ord[rank] = e;
      wsync<GSCR>();
      return ballot(lane < m && tie) != 0;
    }
    for (int j = 0; j < m; j++) {
      const int f = __builtin_amdgcn_readlane(e, j);
      const int64_t wf = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)we >> 32), j)
                                    << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)we, j));
      const uint32_t hf = (uint32_t)__builtin_amdgcn_readlane((int)he, j);
      rank += wf > we || (wf == we && (hf < he || (hf == he && f < e)));
      tie |= (j != lane && wf == we && hf == he);
    }
    wsync<GSCR>();
    if (lane < m) ws.ord[rank] = e;
    wsync<GSCR>();
    return ballot(lane < m && tie) != 0;
  }
  bool tie = false;
  for (int i = lane; i < m; i += WAVE) {
    int e = list[i];
    int64_t we = wt[e];
    uint32_t he = ws.hash[e];
    int rank = 0;
    for (int j = 0; j < m; j++) {
      int f = list[j];
      int64_t wf = wt[f];
      uint32_t hf = ws.hash[f];
      bool before = wf > we || (wf == we && (hf < he || (hf == he && f < e)));
      rank += before;
      tie |= (f != e && wf == we && hf == he);
    }
    ws.act2[rank] = e;
  }
  wsync<GSCR>();
  for (int i = lane; i < m; i += WAVE) ws.ord[i] = ws.act2[i];
  wsync<GSCR>();
  return ballot(tie) != 0;
}

// getDesiredPlan (planner.go:211-304) over the sorted list ord[0..m).
// wt/mxv: weights and max (I64_MAX = none) per element; minimums from ws.mn
// when use_min; capacities from ws.cap/EF_HAS_CAP when use_cap.
// Writes plan[e], over[e], ofl[e] (EF_HAS_PLAN/EF_HAS_OVER) for listed e.
template <bool GSCR>
__device__ int64_t desired_plan(const PlanWs& ws, const int64_t* wt, const int64_t* mxv, bool use_min, bool use_cap,
                                int m, int64_t total, bool keep, int64_t* plan, int64_t* over, uint32_t* ofl) {
  const int lane = lane_id_h();
  // ---- minimum pass
  int64_t R = total;
  for (int base = 0; base < m; base += WAVE) {
    int i = base + lane;
    bool v = i < m;
    int e = v ? ws.ord[i] : 0;
    int64_t Mn = (v && use_min) ? ws.mn[e] : 0;
    bool hc = v && use_cap && (ws.fl[e] & EF_HAS_CAP);
    int64_t U = hc ? ws.cap[e] : I64_MAX;
    Clamp f;
    if (!v) {
      f = {0, NEG_INF};
    } else if (Mn >= 0) {
      f = {Mn < U ? Mn : U, 0};
    } else {
      f = {Mn, NEG_INF};
    }
    Clamp inc = wave_scan_clamp_n(f, clamp_narrow(f, R));
    Clamp exc = wave_shr1_clamp(inc);
    int64_t Ri = clamp_apply(exc, R);
    if (v) {
      int64_t mt = Mn < Ri ? Mn : Ri;
      uint32_t of = EF_HAS_PLAN;
      if (hc && ws.cap[e] < mt) {
        over[e] = mt - ws.cap[e];
        of |= EF_HAS_OVER;
        mt = ws.cap[e];
      } else {
        over[e] = 0;
      }
      plan[e] = mt;
      ofl[e] = of;
    }
    int last = (m - base) < WAVE ? (m - base - 1) : (WAVE - 1);
    R = clamp_apply(readlane_clamp(inc, last), R);
  }
  wsync<GSCR>();
  // ---- weighted rounds
  for (int i = lane; i < m; i += WAVE) ws.act[i] = ws.ord[i];
  wsync<GSCR>();
  int na = m;
  bool modified = true;
  // The reference loop ends after at most m+1 rounds for non-negative weights
  // (planner.go:216-220); the bound only guards the GPU against a hang on
  // adversarial (negative-weight) input, where Go itself would not terminate.
  int rounds = 0;
  while (modified && R > 0 && rounds++ < 4 * m + 64) {
    modified = false;
    int64_t wsum = 0;
    for (int i = lane; i < na; i += WAVE) wsum = wadd(wsum, wt[ws.act[i]]);
    wsum = wave_sum_i64(wsum);
    if (wsum <= 0) break;
    const int64_t D = R;
    int keepn = 0;
    bool mod = false;
    for (int base = 0; base < na; base += WAVE) {
      int i = base + lane;
      bool v = i < na;
      int e = v ? ws.act[i] : 0;
      int64_t start = v ? plan[e] : 0;
      int64_t ee = v ? ceil_extra(D, wt[e], wsum) : 0;
      bool hm = v && mxv[e] != I64_MAX;
      bool hc = v && use_cap && (ws.fl[e] & EF_HAS_CAP);
      int64_t U = I64_MAX;
      if (hm) U = mxv[e];
      if (hc && ws.cap[e] < U) U = ws.cap[e];
      int64_t V = U == I64_MAX ? I64_MAX : wsub(U, start);
      int64_t mm = ee < V ? ee : V;
      Clamp f = !v ? Clamp{0, NEG_INF} : (mm >= 0 ? Clamp{mm, 0} : Clamp{mm, NEG_INF});
      Clamp inc = wave_scan_clamp_n(f, clamp_narrow(f, R));
      Clamp exc = wave_shr1_clamp(inc);
      int64_t Ri = clamp_apply(exc, R);
      bool full = false;
      if (v) {
        int64_t extra = ee < Ri ? ee : Ri;
        int64_t t = wadd(start, extra);
        if (hm && t > mxv[e]) {
          t = mxv[e];
          full = true;
        }
        if (hc && t > ws.cap[e]) {
          over[e] = wadd((ofl[e] & EF_HAS_OVER) ? over[e] : 0, wsub(t, ws.cap[e]));
          ofl[e] |= EF_HAS_OVER;
          t = ws.cap[e];
          full = true;
        }
        plan[e] = t;
        if (t > start) mod = true;
      }
      uint64_t km = ballot(v && !full);
      if (v && !full) ws.act2[keepn + mbcnt(km)] = e;
      keepn += popc64(km);
      int last = (na - base) < WAVE ? (na - base - 1) : (WAVE - 1);
      R = clamp_apply(readlane_clamp(inc, last), R);
    }
    modified = ballot(mod) != 0;
    wsync<GSCR>();
    for (int i = lane; i < keepn; i += WAVE) ws.act[i] = ws.act2[i];
    na = keepn;
    wsync<GSCR>();
  }
  if (!keep) {
    for (int i = lane; i < m; i += WAVE) {
      int e = ws.ord[i];
      if (ofl[e] & EF_HAS_OVER) {
        int64_t v = over[e] < R ? over[e] : R;
        if (v > 0) {
          over[e] = v;
        } else {
          over[e] = 0;
          ofl[e] &= ~EF_HAS_OVER;
        }
      }
    }
  }
  wsync<GSCR>();
  return R;
}

// planner.Plan (planner.go:83-177) for K elements 0..K-1, all with preferences.
// Leaves the final plan in ws.plan, the overflow in ws.over/EF_HAS_OVER.
template <bool GSCR>
__device__ uint32_t plan_row(const PlanWs& ws, int K, int64_t total, bool avoid, bool keep) {
  const int lane = lane_id_h();
  uint32_t rflags = 0;
  for (int i = lane; i < K; i += WAVE) {
    ws.act[i] = i;
    ws.mx2[i] = (ws.fl[i] & EF_HAS_MAX) ? ws.mx[i] : I64_MAX;
  }
  wsync<GSCR>();
  if (sort_by_weight_hash<GSCR>(ws, ws.w, ws.act, K)) rflags |= KAD_RF_HASH_TIE;
  if (!avoid) keep = true;
  desired_plan<GSCR>(ws, ws.w, ws.mx2, true, true, K, total, keep, ws.plan, ws.over, ws.ofl);
  if (!avoid) return rflags;
  // currentPlan, capped by capacity (planner.go:134-146)
  int64_t cur_total = 0, des_total = 0;
  for (int i = lane; i < K; i += WAVE) {
    int64_t r = ws.cur[i];
    if ((ws.fl[i] & EF_HAS_CAP) && ws.cap[i] < r) r = ws.cap[i];
    cur_total = wadd(cur_total, r);
    des_total = wadd(des_total, ws.plan[i]);
    ws.adj[i] = r;  // adj := currentPlan
  }
  cur_total = wave_sum_i64(cur_total);
  des_total = wave_sum_i64(des_total);
  wsync<GSCR>();
  if (cur_total != des_total) {
    const bool up = cur_total < des_total;
    const int64_t count = up ? des_total - cur_total : cur_total - des_total;
    // preferences of the clusters to scale (planner.go:306-366)
    int m = 0;
    for (int base = 0; base < K; base += WAVE) {
      int i = base + lane;
      bool sel = false;
      if (i < K) {
        int64_t d = ws.plan[i], c = ws.adj[i];
        sel = up ? d > c : d < c;
        if (sel) {
          ws.w2[i] = up ? d - c : c - d;
          ws.mx2[i] = up ? ((ws.fl[i] & EF_HAS_MAX) ? ws.mx[i] - c : I64_MAX) : c;
        }
      }
      uint64_t bm = ballot(sel);
      if (sel) ws.act[m + mbcnt(bm)] = i;
      m += popc64(bm);
    }
    wsync<GSCR>();
    if (m > 0 && sort_by_weight_hash<GSCR>(ws, ws.w2, ws.act, m)) rflags |= KAD_RF_HASH_TIE;
    // scale plan: no capacity, no minimums, keepUnschedulable = false (its overflow is discarded)
    for (int i = lane; i < K; i += WAVE) ws.ofl2[i] = 0;
    wsync<GSCR>();
    if (m > 0) desired_plan<GSCR>(ws, ws.w2, ws.mx2, false, false, m, count, false, ws.plan2, ws.over2, ws.ofl2);
    for (int i = lane; i < K; i += WAVE) {
      int64_t a = ws.adj[i];
      if (ws.ofl2[i] & EF_HAS_PLAN) a = up ? wadd(a, ws.plan2[i]) : wsub(a, ws.plan2[i]);
      ws.plan[i] = a;
    }
  } else {
    for (int i = lane; i < K; i += WAVE) ws.plan[i] = ws.adj[i];
  }
  wsync<GSCR>();
  return rflags;
}

// ------------------------------------------------ rows of K <= 64 elements
// The same planner with one element per lane and every per-element array in
// registers: no LDS workspace, no wave syncs. Element i (ascending cluster id)
// lives in lane i; the sorted passes permute the operands into sorted lanes
// (ds_permute by rank), scan there with inactive lanes as the identity clamp
// (0, -inf) — which is what compacting the active list does — and send the
// results back (ds_bpermute by rank).
struct PlanLane {
  int64_t w, mn, mx, cap, cur;  // weight, MinReplicas, MaxReplicas (EF_HAS_MAX), capacity (EF_HAS_CAP), current
  uint32_t fl, hash;            // EF_HAS_MAX | EF_HAS_CAP; FNV-1 of name ‖ key
};
struct PlanOut {
  int64_t plan, over;  // final plan, overflow (EF_HAS_OVER in ofl)
  uint32_t ofl;
};

__device__ __forceinline__ int lane_perm32(int dst, int v) { return __builtin_amdgcn_ds_permute(dst << 2, v); }
__device__ __forceinline__ int lane_bperm32(int src, int v) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
__device__ __forceinline__ int64_t lane_perm64(int dst, int64_t v) {
  const uint32_t lo = (uint32_t)lane_perm32(dst, (int)(uint32_t)v);
  const uint32_t hi = (uint32_t)lane_perm32(dst, (int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t lane_bperm64(int src, int64_t v) {
  const uint32_t lo = (uint32_t)lane_bperm32(src, (int)(uint32_t)v);
  const uint32_t hi = (uint32_t)lane_bperm32(src, (int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l));
}

// rank of each listed lane (in = true) by (weight desc, hash asc, element asc) among the listed
// lanes (sort_by_weight_hash); unlisted lanes get m + their order among the unlisted, so the ranks are a
// permutation of 0..63. *tie: two listed elements equal on (weight, hash).
// kbuf (optional): 64 u64 of the wave's LDS; the listed keys are compacted there and read back as
// broadcasts (LDS reads instead of two v_readlane per compare)
__device__ __forceinline__ int lane_sort_rank(bool in, int64_t we, uint32_t he, bool* tie, uint64_t* kbuf = nullptr) {
  const int lane = lane_id_h();
  const uint64_t lm = ballot(in);
  const int m = popc64(lm);
  int rank = 0;
  bool t = false;
  if (!ballot(in && (we < 0 || we >= (1 << 25)))) {
    // every listed weight in [0, 2^25): (weight desc, hash asc, lane asc) as one unique ascending u64 key
    // — one compare per listed element; a (weight, hash) tie = equal keys but for the lane bits
    const uint64_t ke = ((uint64_t)(uint32_t)((1 << 25) - 1 - (int)(in ? we : 0)) << 38) | ((uint64_t)he << 6) | (uint64_t)lane;
    if (kbuf) {
      if (in) kbuf[mbcnt(lm)] = ke;
      wave_sync();
#pragma unroll 4
      for (int i = 0; i < m; ++i) rank += kbuf[i] < ke;
      wave_sync();  // the buffer is reused by the next sort
    } else {
      const uint32_t khi = (uint32_t)(ke >> 32), klo = (uint32_t)ke;
      for (uint64_t r = lm; r; r &= r - 1) {
        const int j = __builtin_ctzll(r);
        const uint64_t kf = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)khi, j) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)klo, j);
        rank += kf < ke;
      }
    }
    // ties: neighbours in sorted order with equal (weight, hash)
    const int rk = in ? rank : m + mbcnt(~lm);
    const int64_t sk = lane_perm64(rk, (int64_t)(ke >> 6));
    const int64_t pk = dpp64<0x138, 0xf>(-1, sk);  // wave_shr:1: the previous sorted lane's key
    *tie = ballot(lane > 0 && lane < m && sk == pk) != 0;
    return rk;
  } else {
    for (uint64_t r = lm; r; r &= r - 1) {
      const int j = __builtin_ctzll(r);
      const int64_t wf = readlane64(we, j);
      const uint32_t hf = (uint32_t)__builtin_amdgcn_readlane((int)he, j);
      rank += wf > we || (wf == we && (hf < he || (hf == he && j < lane)));
      t |= (j != lane && wf == we && hf == he);
    }
  }
  *tie = ballot(in && t) != 0;
  return in ? rank : m + mbcnt(~lm);
}

// getDesiredPlan (planner.go:211-304) on sorted lanes: lane s < m holds the s-th element of the
// sorted list (wt, mxv = I64_MAX for none, mn when use_min, cap when hc). Returns R; plan / over /
// ofl per sorted lane.
__device__ __forceinline__ int64_t desired_plan_lanes(int m, int64_t wt, int64_t mxv, int64_t Mn, bool hc, int64_t cap,
                                                      int64_t total, bool keep, int64_t& plan, int64_t& over,
                                                      uint32_t& ofl) {
  const int lane = lane_id_h();
  const bool v = lane < m;
  // ---- minimum pass
  int64_t R = total;
  {
    const int64_t U = hc ? cap : I64_MAX;
    Clamp f;
    if (!v)
      f = {0, NEG_INF};
    else if (Mn >= 0)
      f = {Mn < U ? Mn : U, 0};
    else
      f = {Mn, NEG_INF};
    const Clamp inc = wave_scan_clamp_n(f, clamp_narrow(f, R));
    const int64_t Ri = clamp_apply(wave_shr1_clamp(inc), R);
    int64_t mt = Mn < Ri ? Mn : Ri;
    ofl = v ? EF_HAS_PLAN : 0u;
    over = 0;
    if (v && hc && cap < mt) {
      over = mt - cap;
      ofl |= EF_HAS_OVER;
      mt = cap;
    }
    plan = v ? mt : 0;
    R = clamp_apply(readlane_clamp(inc, WAVE - 1), R);
  }
  // ---- weighted rounds over the active lanes (the reference's compacted list)
  bool active = v;
  bool modified = true;
  int rounds = 0;  // see desired_plan: guards only adversarial negative weights
  while (modified && R > 0 && rounds++ < 4 * m + 64) {
    const int64_t wsum = wave_sum_i64(active ? wt : 0);
    if (wsum <= 0) break;
    const int64_t D = R;
    const int64_t start = plan;
    const double inv = 1.0 / (double)wsum;  // wave-uniform
    const int64_t ee = active ? ceil_extra_inv(D, wt, wsum, inv) : 0;
    const bool hm = active && mxv != I64_MAX;
    const bool hcap = active && hc;
    int64_t U = I64_MAX;
    if (hm) U = mxv;
    if (hcap && cap < U) U = cap;
    const int64_t V = U == I64_MAX ? I64_MAX : wsub(U, start);
    const int64_t mm = ee < V ? ee : V;
    const Clamp f = !active ? Clamp{0, NEG_INF} : (mm >= 0 ? Clamp{mm, 0} : Clamp{mm, NEG_INF});
    const Clamp inc = wave_scan_clamp_n(f, clamp_narrow(f, R));
    const int64_t Ri = clamp_apply(wave_shr1_clamp(inc), R);
    bool full = false, mod = false;
    if (active) {
      const int64_t extra = ee < Ri ? ee : Ri;
      int64_t t = wadd(start, extra);
      if (hm && t > mxv) {
        t = mxv;
        full = true;
      }
      if (hcap && t > cap) {
        over = wadd((ofl & EF_HAS_OVER) ? over : 0, wsub(t, cap));
        ofl |= EF_HAS_OVER;
        t = cap;
        full = true;
      }
      plan = t;
      mod = t > start;
    }
    active = active && !full;
    R = clamp_apply(readlane_clamp(inc, WAVE - 1), R);
    modified = ballot(mod) != 0;
  }
  if (!keep && v && (ofl & EF_HAS_OVER)) {
    const int64_t x = over < R ? over : R;
    if (x > 0) {
      over = x;
    } else {
      over = 0;
      ofl &= ~EF_HAS_OVER;
    }
  }
  return R;
}

// The same getDesiredPlan in int32 for narrow rows (desired_narrow: total < 2^24; every listed weight in
// [0, 2^20); minimums in [0, 2^18); maximums and capacities in [0, 2^24); minimum <= maximum). Then no
// element starts a round above its bound (V >= 0), remainingReplicas only falls (R <= total), every
// clamp step is >= 0 and the steps of one scan sum below 2^25 (minimums: 64 · 2^18; rounds: Σ ceil ≤
// R + 64), so every value fits int32 and the results equal the int64 path's. -inf is NEG30 = -2^30:
// a genuine floor is >= -2^25, and -2^30 minus any scan's steps stays above INT32_MIN, so the clamp
// composition needs no -inf test (max(t_a − s_b, t_b) keeps both orders). weightSum < 2^26 and
// D·w + weightSum < 2^53 make the f64 quotient of ceil_extra exact after the two corrections.
__device__ __forceinline__ bool desired_narrow(bool v, int64_t total, int64_t wt, int64_t mxv, int64_t Mn, bool hc,
                                               int64_t cap) {
  return total >= 0 && total < (1 << 24) &&
         !ballot(v && (wt < 0 || wt >= (1 << 20) || Mn < 0 || Mn >= (1 << 18) ||
                       (mxv != I64_MAX && (mxv < 0 || mxv >= (1 << 24) || Mn > mxv)) ||
                       (hc && (cap < 0 || cap >= (1 << 24)))));
}
__device__ __forceinline__ int64_t desired_plan_lanes32(int m, int wt, int mxv, int Mn, bool hc, int cap, int total,
                                                        bool keep, int64_t& plan64, int64_t& over64, uint32_t& ofl) {
  constexpr int NONE = INT32_MAX;  // no maximum / capacity
  const int lane = lane_id_h();
  const bool v = lane < m;
  auto scan = [](int s, int t) {  // inclusive clamp scan; lanes without a source combine with (0, NEG30)
#define KAD_C32(CTRL, RM)                                                                  \
  {                                                                                        \
    const int pt = __builtin_amdgcn_update_dpp(NEG30, t, CTRL, RM, 0xf, false);           \
    const int at = pt - s;                                                                 \
    t = at > t ? at : t;                                                                   \
    s += __builtin_amdgcn_update_dpp(0, s, CTRL, RM, 0xf, true);                           \
  }
    KAD_C32(0x111, 0xf)
    KAD_C32(0x112, 0xf)
    KAD_C32(0x114, 0xf)
    KAD_C32(0x118, 0xf)
    KAD_C32(0x142, 0xa)
    KAD_C32(0x143, 0xc)
#undef KAD_C32
    return make_int2(s, t);
  };
  auto apply = [](int s, int t, int R) { const int x = R - s; return x > t ? x : t; };
  // ---- minimum pass
  int R = total;
  int plan, over = 0;
  {
    const int U = hc ? cap : NONE;
    const int fs = v ? (Mn < U ? Mn : U) : 0, ft = v ? 0 : NEG30;
    const int2 inc = scan(fs, ft);
    const int es = dpp32<0x138, 0xf>(0, inc.x), et = dpp32<0x138, 0xf>(NEG30, inc.y);  // exclusive
    const int Ri = apply(es, et, R);
    int mt = Mn < Ri ? Mn : Ri;
    ofl = v ? EF_HAS_PLAN : 0u;
    if (v && hc && cap < mt) {
      over = mt - cap;
      ofl |= EF_HAS_OVER;
      mt = cap;
    }
    plan = v ? mt : 0;
    R = apply(__builtin_amdgcn_readlane(inc.x, WAVE - 1), __builtin_amdgcn_readlane(inc.y, WAVE - 1), R);
  }
  bool active = v;
  bool modified = true;
  int rounds = 0;
  while (modified && R > 0 && rounds++ < 4 * m + 64) {
    const int wsum = wave_sum_i32(active ? wt : 0);
    if (wsum <= 0) break;
    const int D = R;
    const int start = plan;
    const double sd = (double)wsum, inv = 1.0 / sd;  // wave-uniform
    int ee = 0;
    if (active) {  // ceil((D·w + wsum − 1) / wsum), exact
      const double nd = (double)D * (double)wt + (double)(wsum - 1);
      int q = (int)(nd * inv);
      double r = nd - (double)q * sd;
      q += (r >= sd) - (r < 0.0);
      r = nd - (double)q * sd;
      q += (r >= sd) - (r < 0.0);
      ee = q;
    }
    const bool hm = active && mxv != NONE;
    const bool hcap = active && hc;
    int U = NONE;
    if (hm) U = mxv;
    if (hcap && cap < U) U = cap;
    const int V = U == NONE ? NONE : U - start;
    const int mm = ee < V ? ee : V;
    const int fs = active ? mm : 0, ft = (active && mm >= 0) ? 0 : NEG30;
    const int2 inc = scan(fs, ft);
    const int es = dpp32<0x138, 0xf>(0, inc.x), et = dpp32<0x138, 0xf>(NEG30, inc.y);
    const int Ri = apply(es, et, R);
    bool full = false, mod = false;
    if (active) {
      const int extra = ee < Ri ? ee : Ri;
      int t = start + extra;
      if (hm && t > mxv) {
        t = mxv;
        full = true;
      }
      if (hcap && t > cap) {
        over = ((ofl & EF_HAS_OVER) ? over : 0) + (t - cap);
        ofl |= EF_HAS_OVER;
        t = cap;
        full = true;
      }
      plan = t;
      mod = t > start;
    }
    active = active && !full;
    R = apply(__builtin_amdgcn_readlane(inc.x, WAVE - 1), __builtin_amdgcn_readlane(inc.y, WAVE - 1), R);
    modified = ballot(mod) != 0;
  }
  if (!keep && v && (ofl & EF_HAS_OVER)) {
    const int x = over < R ? over : R;
    if (x > 0) {
      over = x;
    } else {
      over = 0;
      ofl &= ~EF_HAS_OVER;
    }
  }
  plan64 = plan;
  over64 = over;
  return R;
}
// getDesiredPlan on sorted lanes, narrow rows in int32
__device__ __forceinline__ int64_t desired_plan_any(int m, int64_t wt, int64_t mxv, int64_t Mn, bool hc, int64_t cap,
                                                    int64_t total, bool keep, int64_t& plan, int64_t& over,
                                                    uint32_t& ofl) {
  if (desired_narrow(lane_id_h() < m, total, wt, mxv, Mn, hc, cap))
    return desired_plan_lanes32(m, (int)wt, mxv == I64_MAX ? INT32_MAX : (int)mxv, (int)Mn, hc, (int)cap, (int)total,
                                keep, plan, over, ofl);
  return desired_plan_lanes(m, wt, mxv, Mn, hc, cap, total, keep, plan, over, ofl);
}

// planner.Plan (planner.go:83-177) for K <= 64 elements, element i in lane i. Returns KAD_RF_HASH_TIE
// when a sort met a (weight, hash) tie.
__device__ __forceinline__ uint32_t plan_row_lanes(const PlanLane& e, int K, int64_t total, bool avoid, bool keep,
                                                   PlanOut& out, uint64_t* kbuf = nullptr) {
  const int lane = lane_id_h();
  const bool v = lane < K;
  uint32_t rflags = 0;
  const bool hmax = v && (e.fl & EF_HAS_MAX), hcap = v && (e.fl & EF_HAS_CAP);
  const int64_t mx2 = hmax ? e.mx : I64_MAX;
  bool tie;
  const int rank = lane_sort_rank(v, e.w, e.hash, &tie, kbuf);
  if (tie) rflags |= KAD_RF_HASH_TIE;
  if (!avoid) keep = true;
  // element lanes → sorted lanes
  const int64_t s_w = lane_perm64(rank, e.w), s_mx = lane_perm64(rank, mx2), s_mn = lane_perm64(rank, e.mn);
  const int64_t s_cap = lane_perm64(rank, e.cap);
  const bool s_hc = lane_perm32(rank, hcap ? 1 : 0) != 0;
  int64_t p_s, o_s;
  uint32_t f_s;
  desired_plan_any(K, s_w, s_mx, s_mn, s_hc, s_cap, total, keep, p_s, o_s, f_s);
  // sorted lanes → element lanes
  int64_t plan = lane_bperm64(rank, p_s);
  out.over = lane_bperm64(rank, o_s);
  out.ofl = (uint32_t)lane_bperm32(rank, (int)f_s);
  if (avoid) {
    // currentPlan, capped by capacity (planner.go:134-146)
    int64_t adj = v ? e.cur : 0;
    if (hcap && e.cap < adj) adj = e.cap;
    const int64_t cur_total = wave_sum_i64(adj), des_total = wave_sum_i64(v ? plan : 0);
    if (cur_total != des_total) {
      const bool up = cur_total < des_total;
      const int64_t count = up ? des_total - cur_total : cur_total - des_total;
      // preferences of the clusters to scale (planner.go:306-366)
      const bool sel = v && (up ? plan > adj : plan < adj);
      const int64_t w2 = up ? plan - adj : adj - plan;
      const int64_t m2 = up ? (hmax ? e.mx - adj : I64_MAX) : adj;
      const int m = popc64(ballot(sel));
      int64_t plan2 = 0;
      uint32_t ofl2 = 0;
      if (m > 0) {
        bool tie2;
        const int r2 = lane_sort_rank(sel, w2, e.hash, &tie2, kbuf);
        if (tie2) rflags |= KAD_RF_HASH_TIE;
        int64_t p2s, o2s;
        uint32_t f2s;
        // scale plan: no capacity, no minimums, keepUnschedulable = false (its overflow is discarded)
        desired_plan_any(m, lane_perm64(r2, w2), lane_perm64(r2, m2), 0, false, 0, count, false, p2s, o2s, f2s);
        plan2 = lane_bperm64(r2, p2s);
        // every lane takes part in the bpermute (a disabled source lane reads as 0), then the select
        const uint32_t f2 = (uint32_t)lane_bperm32(r2, (int)f2s);
        ofl2 = sel ? f2 : 0u;
      }
      plan = adj;
      if (ofl2 & EF_HAS_PLAN) plan = up ? wadd(adj, plan2) : wsub(adj, plan2);
    } else {
      plan = adj;
    }
  }
  out.plan = plan;
  return rflags;
}

// ------------------------------------------------ two rows per wave (rows of K <= 32)
// C4's rows hold 15 selected clusters on average (97 % at most 32), so the 64-lane planner leaves three
// quarters of each wave idle. plan_pair_kernel runs two rows per wave: row A in lanes 0-31, row B in lanes
// 32-63 (a "segment" each). What is row-uniform in the 64-lane planner is segment-uniform here (a VGPR
// holding one value per segment); scans and reductions stop at the segment boundary (no row_bcast31 step);
// the loops run until both segments are done, a finished segment's lanes frozen; the narrow / wide choice
// is made for the two rows together (both paths give identical results). Element i of a row is in
// segment lane i.
__device__ __forceinline__ int seg_lane() { return lane_id_h() & 31; }
__device__ __forceinline__ bool seg_hi() { return lane_id_h() >= 32; }
// lane l of this lane's segment
__device__ __forceinline__ int seg_read32(int v, int l) {
  const int a = __builtin_amdgcn_readlane(v, l), b = __builtin_amdgcn_readlane(v, 32 + l);
  return seg_hi() ? b : a;
}
__device__ __forceinline__ int64_t seg_read64(int64_t v, int l) {
  const uint32_t lo = (uint32_t)seg_read32((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)seg_read32((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// this segment's 32 bits of a wave ballot
__device__ __forceinline__ uint32_t seg_bits(uint64_t b) { return seg_hi() ? (uint32_t)(b >> 32) : (uint32_t)b; }
__device__ __forceinline__ uint32_t seg_ballot(bool p) { return seg_bits(ballot(p)); }
__device__ __forceinline__ int seg_mbcnt(uint32_t sb) { return __builtin_popcount(sb & ((1u << seg_lane()) - 1u)); }
// segment reductions: row_shr 1/2/4/8 within 16-lane rows, then row_bcast15 into rows 1 and 3 (row mask 0xa)
// — lanes 31 and 63 hold their segment's result; every lane active
#define KAD_SEG_STEPS(OP, ID)          \
  v = OP(v, dpp32<0x111, 0xf>(ID, v)); \
  v = OP(v, dpp32<0x112, 0xf>(ID, v)); \
  v = OP(v, dpp32<0x114, 0xf>(ID, v)); \
  v = OP(v, dpp32<0x118, 0xf>(ID, v)); \
  v = OP(v, dpp32<0x142, 0xa>(ID, v)); \
  return seg_read32(v, 31)
__device__ __forceinline__ int seg_sum_i32(int v) { KAD_SEG_STEPS(iadd_, 0); }
__device__ __forceinline__ int seg_max_i32(int v) { KAD_SEG_STEPS(imax_, INT32_MIN); }
#undef KAD_SEG_STEPS
__device__ __forceinline__ int64_t seg_sum_i64(int64_t v) {  // wrapping (Go int64)
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x111, 0xf>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x112, 0xf>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x114, 0xf>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x118, 0xf>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x142, 0xa>(0, v));
  return seg_read64(v, 31);
}
__device__ __forceinline__ int64_t seg_max_i64(int64_t v) {  // signed: high words, then the low words under them
  const int hi = (int)(v >> 32);
  const int mh = seg_max_i32(hi);
  const uint32_t lo = hi == mh ? (uint32_t)v : 0u;
  const uint32_t ml = (uint32_t)seg_max_i32((int)(lo ^ 0x80000000u)) ^ 0x80000000u;
  return (int64_t)(((uint64_t)(uint32_t)mh << 32) | ml);
}
__device__ __forceinline__ double seg_sum_f64(double v) {  // exact for integer-valued sums < 2^53
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
// inclusive clamp scan within each segment; lanes without a source combine with the identity (0, -inf)
__device__ __forceinline__ Clamp seg_scan_clamp(Clamp v) {
  v = clamp_compose(dpp_clamp<0x111, 0xf>(v), v);
  v = clamp_compose(dpp_clamp<0x112, 0xf>(v), v);
  v = clamp_compose(dpp_clamp<0x114, 0xf>(v), v);
  v = clamp_compose(dpp_clamp<0x118, 0xf>(v), v);
  v = clamp_compose(dpp_clamp<0x142, 0xa>(v), v);
  return v;
}
// exclusive value: the inclusive scan one lane up; each segment's lane 0 gets the identity
__device__ __forceinline__ Clamp seg_shr1_clamp(Clamp v) {
  Clamp o = wave_shr1_clamp(v);
  if (seg_lane() == 0) o = Clamp{0, NEG_INF};
  return o;
}
__device__ __forceinline__ Clamp seg_last_clamp(Clamp v) { return Clamp{seg_read64(v.s, 31), seg_read64(v.t, 31)}; }
// the 32-bit scan of desired_plan_lanes32 per segment (both rows narrow: see desired_narrow)
__device__ __forceinline__ bool pair_clamp_narrow(Clamp f, int64_t R) {
  return !ballot(R < 0 || R >= (1ll << 24) || f.s <= -(1ll << 24) || f.s >= (1ll << 24));
}
#define KAD_CLAMP32_STEP(CTRL, RM)                                        \
  {                                                                       \
    const int ps = dpp32<CTRL, RM>(0, s), pt = dpp32<CTRL, RM>(NEG32, t); \
    const int at = pt == NEG32 ? NEG32 : pt - s;                          \
    t = at > t ? at : t;                                                  \
    s = ps + s;                                                           \
  }
__device__ __forceinline__ Clamp seg_scan_clamp_n(Clamp v, bool narrow) {
  if (!narrow) return seg_scan_clamp(v);
  int s = (int)v.s, t = v.t == NEG_INF ? NEG32 : (int)v.t;
  KAD_CLAMP32_STEP(0x111, 0xf)
  KAD_CLAMP32_STEP(0x112, 0xf)
  KAD_CLAMP32_STEP(0x114, 0xf)
  KAD_CLAMP32_STEP(0x118, 0xf)
  KAD_CLAMP32_STEP(0x142, 0xa)
  return Clamp{(int64_t)s, t == NEG32 ? NEG_INF : (int64_t)t};
}
#undef KAD_CLAMP32_STEP

// lane_sort_rank per segment: the rank among the segment's listed lanes by (weight desc, hash asc, element
// asc); unlisted lanes get m + their order among the segment's unlisted lanes. kbuf: 64 u64 of the wave's
// LDS, segment s compacts its keys into kbuf[32 s ..]. *tie: per segment.
__device__ __forceinline__ int pair_sort_rank(bool in, int64_t we, uint32_t he, bool* tie, uint64_t* kbuf) {
  const int lane = lane_id_h(), sl = seg_lane();
  const uint64_t lmw = ballot(in);
  const uint32_t lm = seg_bits(lmw);
  const int m = __builtin_popcount(lm);
  const int mmax = __builtin_popcount((uint32_t)lmw) > __builtin_popcount((uint32_t)(lmw >> 32))
                       ? __builtin_popcount((uint32_t)lmw) : __builtin_popcount((uint32_t)(lmw >> 32));
  int rank = 0;
  bool t = false;
  if (!ballot(in && (we < 0 || we >= (1 << 25)))) {
    const uint64_t ke = ((uint64_t)(uint32_t)((1 << 25) - 1 - (int)(in ? we : 0)) << 38) | ((uint64_t)he << 6) | (uint64_t)lane;
    uint64_t* kb = kbuf + (lane & 32);
    if (in) kb[seg_mbcnt(lm)] = ke;
    wave_sync();
#pragma unroll 4
    for (int i = 0; i < mmax; ++i) rank += (i < m && kb[i] < ke) ? 1 : 0;
    wave_sync();  // the buffer is reused by the next sort
    const int rk = in ? rank : m + seg_mbcnt(~lm);
    const int64_t sk = lane_perm64((lane & 32) + rk, (int64_t)(ke >> 6));
    const int64_t pk = dpp64<0x138, 0xf>(-1, sk);  // the previous sorted lane's key (wave_shr:1)
    *tie = seg_ballot(sl > 0 && sl < m && sk == pk) != 0;
    return rk;
  }
  for (uint64_t r = lmw; r; r &= r - 1) {
    const int j = __builtin_ctzll(r);
    const int64_t wf = readlane64(we, j);
    const uint32_t hf = (uint32_t)__builtin_amdgcn_readlane((int)he, j);
    if ((j & 32) == (lane & 32)) {
      rank += wf > we || (wf == we && (hf < he || (hf == he && j < lane)));
      t |= (j != lane && wf == we && hf == he);
    }
  }
  *tie = seg_ballot(in && t) != 0;
  return in ? rank : m + seg_mbcnt(~lm);
}

// getDesiredPlan (planner.go:211-304) of two rows on sorted segment lanes (desired_plan_lanes per segment):
// m, total, keep segment-uniform. Returns each segment's R.
__device__ __forceinline__ int64_t desired_plan_pair(int m, int64_t wt, int64_t mxv, int64_t Mn, bool hc, int64_t cap,
                                                     int64_t total, bool keep, int64_t& plan, int64_t& over,
                                                     uint32_t& ofl) {
  const bool v = seg_lane() < m;
  int64_t R = total;
  {
    const int64_t U = hc ? cap : I64_MAX;
    Clamp f;
    if (!v)
      f = {0, NEG_INF};
    else if (Mn >= 0)
      f = {Mn < U ? Mn : U, 0};
    else
      f = {Mn, NEG_INF};
    const Clamp inc = seg_scan_clamp_n(f, pair_clamp_narrow(f, R));
    const int64_t Ri = clamp_apply(seg_shr1_clamp(inc), R);
    int64_t mt = Mn < Ri ? Mn : Ri;
    ofl = v ? EF_HAS_PLAN : 0u;
    over = 0;
    if (v && hc && cap < mt) {
      over = mt - cap;
      ofl |= EF_HAS_OVER;
      mt = cap;
    }
    plan = v ? mt : 0;
    R = clamp_apply(seg_last_clamp(inc), R);
  }
  bool active = v;
  bool modified = true;
  bool go = true;  // this segment still iterates (segment-uniform)
  int rounds = 0;
  for (;;) {
    go = go && modified && R > 0 && rounds < 4 * m + 64;
    if (!ballot(go)) break;
    rounds++;
    const int64_t wsum = seg_sum_i64((go && active) ? wt : 0);
    go = go && wsum > 0;
    if (!ballot(go)) break;
    const bool act = go && active;
    const int64_t D = R;
    const int64_t start = plan;
    const double inv = 1.0 / (double)(wsum > 0 ? wsum : 1);
    const int64_t ee = act ? ceil_extra_inv(D, wt, wsum, inv) : 0;
    const bool hm = act && mxv != I64_MAX;
    const bool hcap = act && hc;
    int64_t U = I64_MAX;
    if (hm) U = mxv;
    if (hcap && cap < U) U = cap;
    const int64_t V = U == I64_MAX ? I64_MAX : wsub(U, start);
    const int64_t mm = ee < V ? ee : V;
    const Clamp f = !act ? Clamp{0, NEG_INF} : (mm >= 0 ? Clamp{mm, 0} : Clamp{mm, NEG_INF});
    const Clamp inc = seg_scan_clamp_n(f, pair_clamp_narrow(f, go ? R : 0));
    const int64_t Ri = clamp_apply(seg_shr1_clamp(inc), R);
    bool full = false, mod = false;
    if (act) {
      const int64_t extra = ee < Ri ? ee : Ri;
      int64_t t = wadd(start, extra);
      if (hm && t > mxv) {
        t = mxv;
        full = true;
      }
      if (hcap && t > cap) {
        over = wadd((ofl & EF_HAS_OVER) ? over : 0, wsub(t, cap));
        ofl |= EF_HAS_OVER;
        t = cap;
        full = true;
      }
      plan = t;
      mod = t > start;
    }
    if (go) {
      active = active && !full;
      R = clamp_apply(seg_last_clamp(inc), R);
    }
    modified = seg_ballot(mod) != 0;
  }
  if (!keep && v && (ofl & EF_HAS_OVER)) {
    const int64_t x = over < R ? over : R;
    if (x > 0) {
      over = x;
    } else {
      over = 0;
      ofl &= ~EF_HAS_OVER;
    }
  }
  return R;
}

// desired_plan_lanes32 per segment (both rows narrow, desired_narrow's bounds)
__device__ __forceinline__ int64_t desired_plan_pair32(int m, int wt, int mxv, int Mn, bool hc, int cap, int total,
                                                       bool keep, int64_t& plan64, int64_t& over64, uint32_t& ofl) {
  constexpr int NONE = INT32_MAX;
  const bool v = seg_lane() < m;
  auto scan = [](int s, int t) {
#define KAD_C32(CTRL, RM)                                                        \
  {                                                                              \
    const int pt = __builtin_amdgcn_update_dpp(NEG30, t, CTRL, RM, 0xf, false); \
    const int at = pt - s;                                                       \
    t = at > t ? at : t;                                                         \
    s += __builtin_amdgcn_update_dpp(0, s, CTRL, RM, 0xf, true);                 \
  }
    KAD_C32(0x111, 0xf)
    KAD_C32(0x112, 0xf)
    KAD_C32(0x114, 0xf)
    KAD_C32(0x118, 0xf)
    KAD_C32(0x142, 0xa)
#undef KAD_C32
    return make_int2(s, t);
  };
  auto apply = [](int s, int t, int R) { const int x = R - s; return x > t ? x : t; };
  auto excl = [](int2 inc) {  // one lane up; each segment's lane 0 gets the identity
    int es = dpp32<0x138, 0xf>(0, inc.x), et = dpp32<0x138, 0xf>(NEG30, inc.y);
    if (seg_lane() == 0) {
      es = 0;
      et = NEG30;
    }
    return make_int2(es, et);
  };
  int R = total;
  int plan, over = 0;
  {
    const int U = hc ? cap : NONE;
    const int fs = v ? (Mn < U ? Mn : U) : 0, ft = v ? 0 : NEG30;
    const int2 inc = scan(fs, ft);
    const int2 ex = excl(inc);
    const int Ri = apply(ex.x, ex.y, R);
    int mt = Mn < Ri ? Mn : Ri;
    ofl = v ? EF_HAS_PLAN : 0u;
    if (v && hc && cap < mt) {
      over = mt - cap;
      ofl |= EF_HAS_OVER;
      mt = cap;
    }
    plan = v ? mt : 0;
    R = apply(seg_read32(inc.x, 31), seg_read32(inc.y, 31), R);
  }
  bool active = v;
  bool modified = true;
  bool go = true;
  int rounds = 0;
  for (;;) {
    go = go && modified && R > 0 && rounds < 4 * m + 64;
    if (!ballot(go)) break;
    rounds++;
    const int wsum = seg_sum_i32((go && active) ? wt : 0);
    go = go && wsum > 0;
    if (!ballot(go)) break;
    const bool act = go && active;
    const int D = R;
    const int start = plan;
    const double sd = (double)(wsum > 0 ? wsum : 1), inv = 1.0 / sd;
    int ee = 0;
    if (act) {  // ceil((D·w + wsum − 1) / wsum), exact
      const double nd = (double)D * (double)wt + (double)(wsum - 1);
      int q = (int)(nd * inv);
      double r = nd - (double)q * sd;
      q += (r >= sd) - (r < 0.0);
      r = nd - (double)q * sd;
      q += (r >= sd) - (r < 0.0);
      ee = q;
    }
    const bool hm = act && mxv != NONE;
    const bool hcap = act && hc;
    int U = NONE;
    if (hm) U = mxv;
    if (hcap && cap < U) U = cap;
    const int V = U == NONE ? NONE : U - start;
    const int mm = ee < V ? ee : V;
    const int fs = act ? mm : 0, ft = (act && mm >= 0) ? 0 : NEG30;
    const int2 inc = scan(fs, ft);
    const int2 ex = excl(inc);
    const int Ri = apply(ex.x, ex.y, R);
    bool full = false, mod = false;
    if (act) {
      const int extra = ee < Ri ? ee : Ri;
      int t = start + extra;
      if (hm && t > mxv) {
        t = mxv;
        full = true;
      }
      if (hcap && t > cap) {
        over = ((ofl & EF_HAS_OVER) ? over : 0) + (t - cap);
        ofl |= EF_HAS_OVER;
        t = cap;
        full = true;
      }
      plan = t;
      mod = t > start;
    }
    if (go) {
      active = active && !full;
      R = apply(seg_read32(inc.x, 31), seg_read32(inc.y, 31), R);
    }
    modified = seg_ballot(mod) != 0;
  }
  if (!keep && v && (ofl & EF_HAS_OVER)) {
    const int x = over < R ? over : R;
    if (x > 0) {
      over = x;
    } else {
      over = 0;
      ofl &= ~EF_HAS_OVER;
    }
  }
  plan64 = plan;
  over64 = over;
  return R;
}
__device__ __forceinline__ int64_t desired_plan_pair_any(int m, int64_t wt, int64_t mxv, int64_t Mn, bool hc,
                                                         int64_t cap, int64_t total, bool keep, int64_t& plan,
                                                         int64_t& over, uint32_t& ofl) {
  // desired_narrow's bounds for both rows together (one path for the wave; both give the same results)
  const bool v = seg_lane() < m;
  if (!ballot(total < 0 || total >= (1 << 24) ||
              (v && (wt < 0 || wt >= (1 << 20) || Mn < 0 || Mn >= (1 << 18) ||
                     (mxv != I64_MAX && (mxv < 0 || mxv >= (1 << 24) || Mn > mxv)) ||
                     (hc && (cap < 0 || cap >= (1 << 24)))))))
    return desired_plan_pair32(m, (int)wt, mxv == I64_MAX ? INT32_MAX : (int)mxv, (int)Mn, hc, (int)cap, (int)total,
                               keep, plan, over, ofl);
  return desired_plan_pair(m, wt, mxv, Mn, hc, cap, total, keep, plan, over, ofl);
}

// planner.Plan (planner.go:83-177) of two rows of K <= 32 (segment-uniform K, total, avoid, keep): element i
// of each row in its segment lane i. Returns each segment's KAD_RF_HASH_TIE.
__device__ __forceinline__ uint32_t plan_row_pair(const PlanLane& e, int K, int64_t total, bool avoid, bool keep,
                                                  PlanOut& out, uint64_t* kbuf) {
  const int base = lane_id_h() & 32;
  const bool v = seg_lane() < K;
  uint32_t rflags = 0;
  const bool hmax = v && (e.fl & EF_HAS_MAX), hcap = v && (e.fl & EF_HAS_CAP);
  const int64_t mx2 = hmax ? e.mx : I64_MAX;
  bool tie;
  const int rank = base + pair_sort_rank(v, e.w, e.hash, &tie, kbuf);
  if (tie) rflags |= KAD_RF_HASH_TIE;
  if (!avoid) keep = true;
  const int64_t s_w = lane_perm64(rank, e.w), s_mx = lane_perm64(rank, mx2), s_mn = lane_perm64(rank, e.mn);
  const int64_t s_cap = lane_perm64(rank, e.cap);
  const bool s_hc = lane_perm32(rank, hcap ? 1 : 0) != 0;
  int64_t p_s, o_s;
  uint32_t f_s;
  desired_plan_pair_any(K, s_w, s_mx, s_mn, s_hc, s_cap, total, keep, p_s, o_s, f_s);
  int64_t plan = lane_bperm64(rank, p_s);
  out.over = lane_bperm64(rank, o_s);
  out.ofl = (uint32_t)lane_bperm32(rank, (int)f_s);
  if (ballot(avoid)) {
    // currentPlan, capped by capacity (planner.go:134-146), per segment that avoids disruption
    int64_t adj = v ? e.cur : 0;
    if (hcap && e.cap < adj) adj = e.cap;
    const int64_t cur_total = seg_sum_i64(adj), des_total = seg_sum_i64(v ? plan : 0);
    const bool scale = avoid && cur_total != des_total;
    const bool up = cur_total < des_total;
    const int64_t count = up ? des_total - cur_total : cur_total - des_total;
    const bool sel = scale && v && (up ? plan > adj : plan < adj);
    const int64_t w2 = up ? plan - adj : adj - plan;
    const int64_t m2 = up ? (hmax ? e.mx - adj : I64_MAX) : adj;
    const int m = __builtin_popcount(seg_ballot(sel));
    int64_t plan2 = 0;
    uint32_t ofl2 = 0;
    if (ballot(m > 0)) {
      bool tie2;
      const int r2 = base + pair_sort_rank(sel, w2, e.hash, &tie2, kbuf);
      if (tie2) rflags |= KAD_RF_HASH_TIE;
      int64_t p2s, o2s;
      uint32_t f2s;
      // scale plan: no capacity, no minimums, keepUnschedulable = false (its overflow is discarded)
      desired_plan_pair_any(m, lane_perm64(r2, w2), lane_perm64(r2, m2), 0, false, 0, count, false, p2s, o2s, f2s);
      plan2 = lane_bperm64(r2, p2s);
      const uint32_t f2 = (uint32_t)lane_bperm32(r2, (int)f2s);
      ofl2 = sel ? f2 : 0u;
    }
    if (avoid) {
      int64_t pa = adj;
      if (ofl2 & EF_HAS_PLAN) pa = up ? wadd(adj, plan2) : wsub(adj, plan2);
      plan = pa;
    }
  }
  out.plan = plan;
  return rflags;
}

}  // namespace kad

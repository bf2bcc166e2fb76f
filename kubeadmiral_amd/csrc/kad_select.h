// MaxCluster selection on one wavefront (plugins/maxcluster/max_cluster.go:42-66).
//
// The reference sorts the feasible clusters by total score with Go 1.19
// sort.Slice (pdqsort, unstable) and keeps the first k. Only the SET of the
// first k matters downstream (Duplicate results are a map; rsp/planner order
// by weight+FNV). The wave therefore:
//   1. finds the k-th largest score T by an 8-bit-digit radix select over an
//      LDS histogram (one pass when scores span < 256 values);
//   2. counts g = #(> T), e = #(== T); if the cut takes every tied element
//      (k - g == e), the selection is {score >= T} and no sort is needed;
//   3. otherwise ("straddle") replays Go's pdqsort restricted to the
//      sub-ranges that contain position k (tests/test_pdq_select.py proves the
//      restriction exact) on the compacted index list in LDS.
#pragma once
#include "kad_wave.h"

namespace kad {

// ------------------------------------------------ restricted pdqsort replay
// The algorithm is written once over a storage policy S providing
//   gt(i, j)  : key at position i > key at position j  (Go less(i, j))
//   swap(i, j): exchange positions i and j.
// LdsStore: positions index v[] (LDS), keys int64 by original position.
// RegStore: one position per lane of two VGPRs (u32 key offset, original
//   position); the whole wave runs the scalar control flow and reads / writes
//   single lanes with v_readlane / v_writelane — no memory round trip per
//   comparison (rows of <= 64 entries whose key range fits 32 bits).
struct LdsStore {
  uint16_t* v;
  const int64_t* key;
  __device__ __forceinline__ bool gt(int i, int j) const { return key[v[i]] > key[v[j]]; }
  __device__ __forceinline__ void swap(int i, int j) const {
    uint16_t t = v[i];
    v[i] = v[j];
    v[j] = t;
  }
};
// v_writelane_b32 (no clang builtin on this toolchain: bind the LLVM intrinsic)
extern "C" __device__ int kad_writelane_i32(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

struct RegStore {
  uint32_t kv, iv;
  __device__ __forceinline__ uint32_t rl(uint32_t x, int l) const {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
  }
  __device__ __forceinline__ bool gt(int i, int j) const { return rl(kv, i) > rl(kv, j); }
  __device__ __forceinline__ void swap(int i, int j) {
    const uint32_t ki = rl(kv, i), kj = rl(kv, j), ii = rl(iv, i), ij = rl(iv, j);
    kv = (uint32_t)kad_writelane_i32((int)kj, i, (int)kv);
    kv = (uint32_t)kad_writelane_i32((int)ki, j, (int)kv);
    iv = (uint32_t)kad_writelane_i32((int)ij, i, (int)iv);
    iv = (uint32_t)kad_writelane_i32((int)ii, j, (int)iv);
  }
};

template <class S>
struct PdqT {
  S& st;
  int xs_b, xs_c;
  __device__ __forceinline__ bool less(int i, int j) const { return st.gt(i, j); }
  __device__ __forceinline__ void swap(int i, int j) const { st.swap(i, j); }
  __device__ __forceinline__ void insertion_sort(int a, int b) const {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && less(j, j - 1); j--) swap(j, j - 1);
  }
  __device__ __forceinline__ void sift_down(int lo, int hi, int first) const {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && less(first + child, first + child + 1)) child++;
      if (!less(first + root, first + child)) return;
      swap(first + root, first + child);
      root = child;
    }
  }
  __device__ __forceinline__ void heap_sort(int a, int b) const {
    int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
      swap(first, first + i);
      sift_down(lo, i, first);
    }
  }
  __device__ __forceinline__ bool partial_insertion_sort(int a, int b) const {
    int i = a + 1;
    for (int j = 0; j < 5; j++) {
      while (i < b && !less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < 50) return false;
      swap(i, i - 1);
      if (i - a >= 2) {
        for (int k = i - 1; k >= 1; k--) {  // sic: Go's lower bound is 1
          if (!less(k, k - 1)) break;
          swap(k, k - 1);
        }
      }
      if (b - i >= 2) {
        for (int k = i + 1; k < b; k++) {
          if (!less(k, k - 1)) break;
          swap(k, k - 1);
        }
      }
    }
    return false;
  }
  __device__ __forceinline__ void break_patterns(int a, int b) const {
    int length = b - a;
    if (length >= 8) {
      uint64_t r = (uint64_t)length;
      uint64_t modulus = 1ull << (64 - __clzll((unsigned long long)length));
      int idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; i++) {
        r ^= r << 13;
        r ^= r >> xs_b;
        r ^= r << xs_c;
        int other = (int)(r & (modulus - 1));
        if (other >= length) other -= length;
        swap(idx - 1 + i, a + other);
      }
    }
  }
  __device__ __forceinline__ void order2(int& a, int& b, int& swaps) const {
    if (less(b, a)) {
      int t = a;
      a = b;
      b = t;
      swaps++;
    }
  }
  __device__ __forceinline__ int median(int a, int b, int c, int& swaps) const {
    order2(a, b, swaps);
    order2(b, c, swaps);
    order2(a, b, swaps);
    return b;
  }
  __device__ __forceinline__ int choose_pivot(int a, int b, int& hint) const {
    int l = b - a, swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= 50) {
        i = median(i - 1, i, i + 1, swaps);
        j = median(j - 1, j, j + 1, swaps);
        k = median(k - 1, k, k + 1, swaps);
      }
      j = median(i, j, k, swaps);
    }
    hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
    return j;
  }
  __device__ __forceinline__ void reverse_range(int a, int b) const {
    for (int i = a, j = b - 1; i < j; i++, j--) swap(i, j);
  }
  __device__ __forceinline__ int partition_equal(int a, int b, int pivot) const {
    swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !less(a, i)) i++;
      while (i <= j && less(a, j)) j--;
      if (i > j) break;
      swap(i, j);
      i++;
      j--;
    }
    return i;
  }
  __device__ __forceinline__ int partition(int a, int b, int pivot, bool& already) const {
    swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && less(i, a)) i++;
    while (i <= j && !less(j, a)) j--;
    if (i > j) {
      swap(j, a);
      already = true;
      return j;
    }
    swap(i, j);
    i++;
    j--;
    for (;;) {
      while (i <= j && less(i, a)) i++;
      while (i <= j && !less(j, a)) j--;
      if (i > j) break;
      swap(i, j);
      i++;
      j--;
    }
    swap(j, a);
    already = false;
    return j;
  }
  // pdqsort_func(data, 0, n, bits.Len(n)) restricted to ranges straddling k.
  __device__ __forceinline__ void select(int n, int k) const {
    int a = 0, b = n;
    int limit = 32 - __clz(n);
    bool wasBalanced = true, wasPartitioned = true;
    while (a < k && k < b) {
      int length = b - a;
      if (length <= 12) {
        insertion_sort(a, b);
        return;
      }
      if (limit == 0) {
        heap_sort(a, b);
        return;
      }
      if (!wasBalanced) {
        break_patterns(a, b);
        limit--;
      }
      int hint;
      int pivot = choose_pivot(a, b, hint);
      if (hint == 2) {
        reverse_range(a, b);
        pivot = (b - 1) - (pivot - a);
        hint = 1;
      }
      if (wasBalanced && wasPartitioned && hint == 1) {
        if (partial_insertion_sort(a, b)) return;
      }
      if (a > 0 && !less(a - 1, pivot)) {
        a = partition_equal(a, b, pivot);
        continue;
      }
      bool already;
      int mid = partition(a, b, pivot, already);
      wasPartitioned = already;
      int leftLen = mid - a, rightLen = b - mid, thr = length / 8;
      if (leftLen < rightLen) {
        if (k < mid) {  // recursion into the smaller left side
          b = mid;
          wasBalanced = wasPartitioned = true;
        } else if (k > mid + 1) {
          wasBalanced = leftLen >= thr;
          a = mid + 1;
        } else {
          return;
        }
      } else {
        if (k > mid + 1) {  // recursion into the smaller right side
          a = mid + 1;
          wasBalanced = wasPartitioned = true;
        } else if (k < mid) {
          wasBalanced = rightLen >= thr;
          b = mid;
        } else {
          return;
        }
      }
    }
  }
};

// storage: LDS keys swapped in place with their original positions
template <class KeyT>
struct KeyLdsStoreT {
  KeyT* key;
  uint16_t* id;
  __device__ __forceinline__ bool gt(int i, int j) const { return key[i] > key[j]; }
  __device__ __forceinline__ void swap(int i, int j) const {
    const KeyT a = key[i], b = key[j];
    const uint16_t x = id[i], y = id[j];
    key[i] = b;
    key[j] = a;
    id[i] = y;
    id[j] = x;
  }
};

// storage: packed key << 16 | id words (PdqWaveP's heapsort fallback)
struct PackedLdsStore {
  uint32_t* e;
  __device__ __forceinline__ bool gt(int i, int j) const { return (e[i] >> 16) > (e[j] >> 16); }
  __device__ __forceinline__ void swap(int i, int j) const {
    const uint32_t a = e[i], b = e[j];
    e[i] = b;
    e[j] = a;
  }
};

// ------------------------------------------- wave-parallel restricted replay
// PdqWave runs the same control flow as PdqT::select — Go 1.19 pdqsort_func
// restricted to the ranges that straddle k — with the whole wave. The scalar
// decisions (pivot choice, branch structure, limit/balance bookkeeping) are
// uniform; the data-parallel steps are computed with ballots and prefix
// counts and applied as disjoint moves in LDS:
//   * partition / partitionEqual: Hoare's scans swap the t-th left stopper
//     with the t-th right stopper for every t with l_t < r_t (l_t rises, r_t
//     falls, so those t form a prefix); the split point is a + #(right
//     stoppers), so the result is exactly the serial one;
//   * insertionSort (<= 12 elements): stable rank = #greater + #equal before;
//   * reverseRange: disjoint pair swaps;
//   * partialInsertionSort: first descent by ballot, then each shift is a
//     rotation whose stop position is found by ballot.
// heapSort (only after log2(n) unbalanced partitions) falls back to lane 0.
// key/id: the n positions' keys (swapped in place) and original positions;
// posL: u16 scratch of n + 64 entries (lanes past the range write into the
// tail, so the stopper scatter needs no exec mask); posR: n entries.
#ifdef KAD_PHASE_PROF
// replay sub-phase counters (profiling build): cycles in partitions, pivot choice + breakPatterns,
// insertion sorts (partial and final), and the number of partitions
#define PQ_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define PQ_ADD(i, x) pr[i] += (uint32_t)(x)
#else
#define PQ_T(v)
#define PQ_ADD(i, x)
#endif
template <class KeyT, bool GS = false>
struct PdqWave {  // GS: key/id/posL/posR live in a global scratch slab
  KeyT* key;
  uint16_t* id;
  uint16_t* posL;
  uint16_t* posR;
  int xs_b, xs_c;
#ifdef KAD_PHASE_PROF
  mutable uint32_t pr[4] = {0, 0, 0, 0};
#endif

  __device__ __forceinline__ KeyT K(int p) const {
    const KeyT v = key[p];
    if constexpr (sizeof(KeyT) == 8) {
      const uint32_t lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
      return (KeyT)(((uint64_t)hi << 32) | lo);
    } else {
      return (KeyT)__builtin_amdgcn_readfirstlane((int)v);
    }
  }
  __device__ __forceinline__ bool less(int i, int j) const { return K(i) > K(j); }
  __device__ __forceinline__ void swap1(int i, int j) const {
    const KeyT ki = key[i], kj = key[j];
    const uint16_t ii = id[i], ij = id[j];
    wsync<GS>();
    if (lane_id() == 0) {
      key[i] = kj;
      key[j] = ki;
      id[i] = ij;
      id[j] = ii;
    }
    wsync<GS>();
  }
  __device__ __forceinline__ KeyT rl(KeyT v, int l) const {
    if constexpr (sizeof(KeyT) == 8) {
      const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
      const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
      return (KeyT)(((uint64_t)hi << 32) | lo);
    } else {
      return (KeyT)__builtin_amdgcn_readlane((int)v, l);
    }
  }
  // m = b - a <= 12: lane x takes rank #greater + #equal before (stable); the
  // keys come from the lanes by readlane, fully unrolled (no loop, no LDS reads)
  __device__ void insertion_sort(int a, int b) const {
    const int m = b - a, lane = lane_id();
    const bool in = lane < m;
    const KeyT kp = key[in ? a + lane : a];
    const uint16_t ip = id[in ? a + lane : a];
    int r = 0;
#pragma unroll
    for (int q = 0; q < 12; ++q) {
      const KeyT kq = rl(kp, q);
      r += (q < m) & ((int)(kq > kp) | (int)((kq == kp) & (q < lane)));
    }
    wsync<GS>();
    if (in) {
      key[a + r] = kp;
      id[a + r] = ip;
    }
    wsync<GS>();
  }
  __device__ void reverse_range(int a, int b) const {
    const int h = (b - a) / 2;
    for (int x0 = 0; x0 < h; x0 += WAVE) {
      const int x = x0 + lane_id();
      if (x < h) {
        const int i = a + x, j = b - 1 - x;
        const KeyT ki = key[i], kj = key[j];
        const uint16_t ii = id[i], ij = id[j];
        key[i] = kj;
        key[j] = ki;
        id[i] = ij;
        id[j] = ii;
      }
    }
    wsync<GS>();
  }
  __device__ __forceinline__ void order2(int& a, int& b, int& swaps) const {
    if (less(b, a)) {
      int t = a;
      a = b;
      b = t;
      swaps++;
    }
  }
  __device__ __forceinline__ int median(int a, int b, int c, int& swaps) const {
    order2(a, b, swaps);
    order2(b, c, swaps);
    order2(a, b, swaps);
    return b;
  }
  // choosePivot: lanes 0-2 each take one candidate triple (i-1, i, i+1 / j.. / k.. for l >= 50) with
  // three LDS reads and order it in VALU (Go's medianAdjacent: order2(a,b), order2(b,c), order2(a,b),
  // counting swaps); the median of the three medians on scalars. Returns the pivot position, *pkey its key.
  __device__ int choose_pivot(int a, int b, int& hint, KeyT& pkey) const {
    const int lane = lane_id();
    const int l = b - a;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    int swaps = 0;
    if (l >= 8) {
      const bool adj = l >= 50;
      const int g = lane < 3 ? lane : 0;
      const int base = g == 0 ? i : (g == 1 ? j : k);
      int pa = adj ? base - 1 : base, pb = base, pc = adj ? base + 1 : base;
      KeyT ka = key[pa], kb = key[pb], kc = key[pc];
      int sw = 0;
      if (adj) {
        auto o2 = [&](int& p0, KeyT& k0, int& p1, KeyT& k1) {  // order2: less(p1, p0) = k1 > k0
          const bool x = k1 > k0;
          const int tp = x ? p1 : p0, tq = x ? p0 : p1;
          const KeyT tk = x ? k1 : k0, tl = x ? k0 : k1;
          p0 = tp;
          p1 = tq;
          k0 = tk;
          k1 = tl;
          sw += x;
        };
        o2(pa, ka, pb, kb);
        o2(pb, kb, pc, kc);
        o2(pa, ka, pb, kb);
      }
      // lane g: the median (pb, kb) of its triple and its swap count
      i = __builtin_amdgcn_readlane(pb, 0);
      j = __builtin_amdgcn_readlane(pb, 1);
      k = __builtin_amdgcn_readlane(pb, 2);
      KeyT ki = rl(kb, 0), kj = rl(kb, 1), kk = rl(kb, 2);
      if (adj) swaps = __builtin_amdgcn_readlane(sw, 0) + __builtin_amdgcn_readlane(sw, 1) + __builtin_amdgcn_readlane(sw, 2);
      // median(i, j, k) with Go's order2 sequence
      if (kj > ki) { int tp = i; i = j; j = tp; KeyT tk = ki; ki = kj; kj = tk; swaps++; }
      if (kk > kj) { int tp = j; j = k; k = tp; KeyT tk = kj; kj = kk; kk = tk; swaps++; }
      if (kj > ki) { int tp = i; i = j; j = tp; KeyT tk = ki; ki = kj; kj = tk; swaps++; }
      pkey = kj;
    } else {
      pkey = K(j);
    }
    hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
    return j;
  }
  __device__ void break_patterns(int a, int b) const {
    int length = b - a;
    if (length >= 8) {
      uint64_t r = (uint64_t)length;
      uint64_t modulus = 1ull << (64 - __clzll((unsigned long long)length));
      int idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; i++) {
        r ^= r << 13;
        r ^= r >> xs_b;
        r ^= r << xs_c;
        int other = (int)(r & (modulus - 1));
        if (other >= length) other -= length;
        swap1(idx - 1 + i, a + other);
      }
    }
  }
  // first p in [i, b) with less(p, p-1), else b
  __device__ int first_descent(int i, int b) const {
    for (int p0 = i; p0 < b; p0 += WAVE) {
      const int p = p0 + lane_id();
      const uint64_t m = ballot(p < b && key[p] > key[p - 1]);
      if (m) return p0 + __ffsll((unsigned long long)m) - 1;
    }
    return b;
  }
  // the element at j0 moves left while it is less than its left neighbour
  // (Go's loop runs down to position 1, i.e. the element may reach 0)
  __device__ void shift_left(int j0) const {
    const int lane = lane_id();
    const KeyT X = K(j0);
    const uint16_t XI = (uint16_t)__builtin_amdgcn_readfirstlane((int)id[j0]);
    int m = 0;
    for (int q1 = j0; q1 > 0; q1 -= WAVE) {
      const int q = q1 - 1 - lane;
      const uint64_t mm = ballot(q >= 0 && key[q] >= X);
      if (mm) {
        m = q1 - 1 - (__ffsll((unsigned long long)mm) - 1) + 1;
        break;
      }
    }
    for (int p1 = j0; p1 > m; p1 -= WAVE) {  // [m, j0) → +1, high chunks first
      const int p = p1 - 1 - lane;
      const bool in = p >= m;
      KeyT kk = 0;
      uint16_t ii = 0;
      if (in) {
        kk = key[p];
        ii = id[p];
      }
      wsync<GS>();
      if (in) {
        key[p + 1] = kk;
        id[p + 1] = ii;
      }
      wsync<GS>();
    }
    if (lane == 0) {
      key[m] = X;
      id[m] = XI;
    }
    wsync<GS>();
  }
  // the element at j0-1 moves right while its right neighbour is less than it
  __device__ void shift_right(int j0, int b) const {
    const int lane = lane_id();
    const KeyT Y = K(j0 - 1);
    const uint16_t YI = (uint16_t)__builtin_amdgcn_readfirstlane((int)id[j0 - 1]);
    int mp = b - 1;
    for (int q0 = j0; q0 < b; q0 += WAVE) {
      const int q = q0 + lane;
      const uint64_t mm = ballot(q < b && key[q] <= Y);
      if (mm) {
        mp = q0 + __ffsll((unsigned long long)mm) - 2;
        break;
      }
    }
    for (int p0 = j0; p0 <= mp; p0 += WAVE) {  // (j0-1, mp] → -1, low chunks first
      const int p = p0 + lane;
      const bool in = p <= mp;
      KeyT kk = 0;
      uint16_t ii = 0;
      if (in) {
        kk = key[p];
        ii = id[p];
      }
      wsync<GS>();
      if (in) {
        key[p - 1] = kk;
        id[p - 1] = ii;
      }
      wsync<GS>();
    }
    if (lane == 0) {
      key[mp] = Y;
      id[mp] = YI;
    }
    wsync<GS>();
  }
  __device__ bool partial_insertion_sort(int a, int b) const {
    int i = a + 1;
    for (int step = 0; step < 5; step++) {
      i = first_descent(i, b);
      if (i == b) return true;
      if (b - a < 50) return false;
      swap1(i, i - 1);
      if (i - a >= 2) shift_left(i - 1);
      if (b - i >= 2) shift_right(i + 1, b);
    }
    return false;
  }
  // Hoare pairing over [lo, hi): right stoppers R (strict ? key > P : key >= P)
  // end on the left; swaps l_t <-> r_t for the prefix of t with l_t < r_t.
  // One pass ranks and scatters both stopper kinds (L from the left, R from
  // the left too: r_t = posR[#R - 1 - t]); a second swaps every valid pair.
  // Returns #R; *T = number of swaps.
  __device__ int pair_partition(int lo, int hi, KeyT P, bool strict, int* T) const {
    const int lane = lane_id();
    int cL = 0, cR = 0;
    for (int c0 = lo; c0 < hi; c0 += WAVE) {
      // exec-free: lanes past hi read position hi-1 and write their (unused) position into posL's
      // tail, at cL + lane - #R >= the final #L (posL has 64 spare entries)
      const int p = c0 + lane;
      const bool in = p < hi;
      const KeyT kk = key[in ? p : hi - 1];
      const bool isR = in && (strict ? kk > P : kk >= P);
      const uint64_t mR = ballot(isR);
      const int rR = mbcnt(mR);
      uint16_t* dst = isR ? posR + (cR + rR) : posL + (cL + lane - rR);
      *dst = (uint16_t)p;
      const int nin = hi - c0 < WAVE ? hi - c0 : WAVE;
      const int nr = popc64(mR);
      cR += nr;
      cL += nin - nr;
    }
    wsync<GS>();
    const int np = cL < cR ? cL : cR;
    int t_n = 0;
    for (int t0 = 0; t0 < np; t0 += WAVE) {
      const int t = t0 + lane;  // t < np + 64 <= n + 64: inside posL; posR index clamped
      const int l = posL[t];
      const int ri = cR - 1 - t;
      const int r = posR[ri > 0 ? ri : 0];
      const bool sw = t < np && l < r;
      const uint64_t m = ballot(sw);
      t_n += popc64(m);
      if (sw) {  // pairs are disjoint: every valid pair swaps at once
        const KeyT kl = key[l], kr = key[r];
        const uint16_t il = id[l], ir = id[r];
        key[l] = kr;
        key[r] = kl;
        id[l] = ir;
        id[r] = il;
      }
      if (~m) break;  // a prefix: once a t fails, every later t fails
    }
    wsync<GS>();
    *T = t_n;
    return cR;
  }
  // P: the pivot's key (choose_pivot)
  __device__ int partition(int a, int b, int pivot, KeyT P, bool& already) const {
    swap1(a, pivot);
    int T;
    const int j = a + pair_partition(a + 1, b, P, true, &T);
    swap1(j, a);
    already = T == 0;
    return j;
  }
  __device__ int partition_equal(int a, int b, int pivot, KeyT P) const {
    swap1(a, pivot);
    int T;
    return a + 1 + pair_partition(a + 1, b, P, false, &T);
  }
  __device__ void select(int n, int k) const {
    int a = 0, b = n;
    int limit = 32 - __clz(n);
    bool wasBalanced = true, wasPartitioned = true;
    while (a < k && k < b) {
      const int length = b - a;
      if (length <= 12) {
        PQ_T(i0);
        insertion_sort(a, b);
        PQ_T(i1);
        PQ_ADD(2, i1 - i0);
        return;
      }
      if (limit == 0) {
        if (lane_id() == 0) {
          KeyLdsStoreT<KeyT> st{key, id};
          PdqT<KeyLdsStoreT<KeyT>> s{st, xs_b, xs_c};
          s.heap_sort(a, b);
        }
        wsync<GS>();
        return;
      }
      PQ_T(c0);
      if (!wasBalanced) {
        break_patterns(a, b);
        limit--;
      }
      int hint;
      KeyT pk;
      int pivot = choose_pivot(a, b, hint, pk);
      if (hint == 2) {
        reverse_range(a, b);
        pivot = (b - 1) - (pivot - a);
        hint = 1;
      }
      PQ_T(c1);
      PQ_ADD(1, c1 - c0);
      if (wasBalanced && wasPartitioned && hint == 1) {
        const bool done = partial_insertion_sort(a, b);
        PQ_T(c2);
        PQ_ADD(2, c2 - c1);
        if (done) return;
        pk = K(pivot);  // the shifts may have moved another element to the pivot's position
      }
      PQ_T(c3);
      PQ_ADD(3, 1);
      if (a > 0 && !(K(a - 1) > pk)) {  // !less(a-1, pivot)
        a = partition_equal(a, b, pivot, pk);
        PQ_T(c4);
        PQ_ADD(0, c4 - c3);
        continue;
      }
      bool already;
      const int mid = partition(a, b, pivot, pk, already);
      PQ_T(c5);
      PQ_ADD(0, c5 - c3);
      wasPartitioned = already;
      const int leftLen = mid - a, rightLen = b - mid, thr = length / 8;
      if (leftLen < rightLen) {
        if (k < mid) {  // recursion into the smaller left side
          b = mid;
          wasBalanced = wasPartitioned = true;
        } else if (k > mid + 1) {
          wasBalanced = leftLen >= thr;
          a = mid + 1;
        } else {
          return;
        }
      } else {
        if (k > mid + 1) {  // recursion into the smaller right side
          a = mid + 1;
          wasBalanced = wasPartitioned = true;
        } else if (k < mid) {
          wasBalanced = rightLen >= thr;
          b = mid;
        } else {
          return;
        }
      }
    }
  }
};

// ------------------------------------- packed wave-parallel restricted replay
// PdqWaveP: the same restricted pdqsort_func replay as PdqWave, on packed elements
// e = key << 16 | original position (rows whose key range and length both fit 16 bits: every
// C3 / C2 row, C5's long rows): a move is one 32-bit LDS access instead of a key and an id.
// The partition is fused into two LDS passes. Go's partition is
//   swap(a, pivot); Hoare pairing over [a+1, b); swap(j, a)      (partitionEqual: no final swap)
// which is one permutation of [a, b). The first pass reads the range through the virtual first
// swap (position `pivot` reads as old e[a]) and scatters the left / right stopper positions; the
// second reads each misplaced pair and the few special positions (a, j, pivot) and writes the final
// arrangement directly: the t-th misplaced left stopper l_t and the t-th misplaced right stopper
// r_t (from the right) exchange; the element paired into j = a + #R goes to a instead (the final
// swap), the pivot element to j; position `pivot` gets old e[a] unless a pair or j covers it.
template <bool GS = false>
struct PdqWaveP {
  uint32_t* e;      // [n] packed elements, permuted in place
  uint16_t* posL;   // [n + 64] stopper scratch (lanes past the range write into the tail)
  uint16_t* posR;   // [n]
  int xs_b, xs_c;
#ifdef KAD_PHASE_PROF
  mutable uint32_t pr[4] = {0, 0, 0, 0};
#endif

  __device__ __forceinline__ uint32_t E(int p) const { return (uint32_t)__builtin_amdgcn_readfirstlane((int)e[p]); }
  __device__ __forceinline__ void swap1(int i, int j) const {
    const uint32_t vi = e[i], vj = e[j];
    wsync<GS>();
    if (lane_id() == 0) {
      e[i] = vj;
      e[j] = vi;
    }
    wsync<GS>();
  }
  // length <= 12: stable rank = #greater + #equal before, from the lanes by readlane
  __device__ void insertion_sort(int a, int b) const {
    const int m = b - a, lane = lane_id();
    const bool in = lane < m;
    const uint32_t vp = e[in ? a + lane : a];
    const uint32_t kp = vp >> 16;
    int r = 0;
#pragma unroll
    for (int q = 0; q < 12; ++q) {
      const uint32_t kq = (uint32_t)__builtin_amdgcn_readlane((int)vp, q) >> 16;
      r += (q < m) & ((int)(kq > kp) | (int)((kq == kp) & (q < lane)));
    }
    wsync<GS>();
    if (in) e[a + r] = vp;
    wsync<GS>();
  }
  __device__ void reverse_range(int a, int b) const {
    const int h = (b - a) / 2;
    for (int x0 = 0; x0 < h; x0 += WAVE) {
      const int x = x0 + lane_id();
      if (x < h) {
        const int i = a + x, j = b - 1 - x;
        const uint32_t vi = e[i], vj = e[j];
        e[i] = vj;
        e[j] = vi;
      }
    }
    wsync<GS>();
  }
  __device__ void break_patterns(int a, int b) const {
    const int length = b - a;
    if (length >= 8) {
      uint64_t r = (uint64_t)length;
      const uint64_t modulus = 1ull << (64 - __clzll((unsigned long long)length));
      const int idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; i++) {
        r ^= r << 13;
        r ^= r >> xs_b;
        r ^= r << xs_c;
        int other = (int)(r & (modulus - 1));
        if (other >= length) other -= length;
        swap1(idx - 1 + i, a + other);
      }
    }
  }
  // choosePivot (Go's medianAdjacent / median order2 sequences, swap counts): lanes 0-2 each read and
  // order one candidate triple in VALU; lane 3 reads e[a - 1] (the partitionEqual test) in the same
  // LDS round trip. Returns the pivot position; *pk its key, *prev the key at a - 1 (a > 0).
  __device__ int choose_pivot(int a, int b, int& hint, uint32_t& pk, uint32_t& prev) const {
    const int lane = lane_id();
    const int l = b - a;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    int swaps = 0;
    const bool adj = l >= 50;
    const int g = lane < 3 ? lane : 0;
    const int base = g == 0 ? i : (g == 1 ? j : k);
    int pa = adj ? base - 1 : base, pb = base, pc = adj ? base + 1 : base;
    uint32_t ka = e[pa] >> 16, kb = e[pb] >> 16, kc = e[pc] >> 16;
    prev = a > 0 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)e[a - 1]) >> 16 : 0u;
    if (l >= 8) {
      int sw = 0;
      if (adj) {
        auto o2 = [&](int& p0, uint32_t& k0, int& p1, uint32_t& k1) {  // order2: less(p1, p0) = k1 > k0
          const bool x = k1 > k0;
          const int tp = x ? p1 : p0, tq = x ? p0 : p1;
          const uint32_t tk = x ? k1 : k0, tl = x ? k0 : k1;
          p0 = tp;
          p1 = tq;
          k0 = tk;
          k1 = tl;
          sw += x;
        };
        o2(pa, ka, pb, kb);
        o2(pb, kb, pc, kc);
        o2(pa, ka, pb, kb);
      }
      i = __builtin_amdgcn_readlane(pb, 0);
      j = __builtin_amdgcn_readlane(pb, 1);
      k = __builtin_amdgcn_readlane(pb, 2);
      uint32_t ki = (uint32_t)__builtin_amdgcn_readlane((int)kb, 0), kj = (uint32_t)__builtin_amdgcn_readlane((int)kb, 1),
               kk = (uint32_t)__builtin_amdgcn_readlane((int)kb, 2);
      if (adj) swaps = __builtin_amdgcn_readlane(sw, 0) + __builtin_amdgcn_readlane(sw, 1) + __builtin_amdgcn_readlane(sw, 2);
      if (kj > ki) { int tp = i; i = j; j = tp; uint32_t tk = ki; ki = kj; kj = tk; swaps++; }
      if (kk > kj) { int tp = j; j = k; k = tp; uint32_t tk = kj; kj = kk; kk = tk; swaps++; }
      if (kj > ki) { int tp = i; i = j; j = tp; uint32_t tk = ki; ki = kj; kj = tk; swaps++; }
      pk = kj;
    } else {
      pk = (uint32_t)__builtin_amdgcn_readlane((int)kb, 1);  // lane 1 read e[j]
    }
    hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
    return j;
  }
  __device__ int first_descent(int i, int b) const {
    for (int p0 = i; p0 < b; p0 += WAVE) {
      const int p = p0 + lane_id();
      const uint64_t m = ballot(p < b && (e[p] >> 16) > (e[p - 1] >> 16));
      if (m) return p0 + __ffsll((unsigned long long)m) - 1;
    }
    return b;
  }
  // the element at j0 moves left while it is less than its left neighbour (down to position 0: Go's
  // loop bound is 1)
  __device__ void shift_left(int j0) const {
    const int lane = lane_id();
    const uint32_t X = E(j0);
    int m = 0;
    for (int q1 = j0; q1 > 0; q1 -= WAVE) {
      const int q = q1 - 1 - lane;
      const uint64_t mm = ballot(q >= 0 && (e[q] >> 16) >= (X >> 16));
      if (mm) {
        m = q1 - 1 - (__ffsll((unsigned long long)mm) - 1) + 1;
        break;
      }
    }
    for (int p1 = j0; p1 > m; p1 -= WAVE) {  // [m, j0) → +1, high chunks first
      const int p = p1 - 1 - lane;
      const bool in = p >= m;
      const uint32_t v = in ? e[p] : 0u;
      wsync<GS>();
      if (in) e[p + 1] = v;
      wsync<GS>();
    }
    if (lane == 0) e[m] = X;
    wsync<GS>();
  }
  // the element at j0-1 moves right while its right neighbour is less than it
  __device__ void shift_right(int j0, int b) const {
    const int lane = lane_id();
    const uint32_t Y = E(j0 - 1);
    int mp = b - 1;
    for (int q0 = j0; q0 < b; q0 += WAVE) {
      const int q = q0 + lane;
      const uint64_t mm = ballot(q < b && (e[q] >> 16) <= (Y >> 16));
      if (mm) {
        mp = q0 + __ffsll((unsigned long long)mm) - 2;
        break;
      }
    }
    for (int p0 = j0; p0 <= mp; p0 += WAVE) {  // (j0-1, mp] → -1, low chunks first
      const int p = p0 + lane;
      const bool in = p <= mp;
      const uint32_t v = in ? e[p] : 0u;
      wsync<GS>();
      if (in) e[p - 1] = v;
      wsync<GS>();
    }
    if (lane == 0) e[mp] = Y;
    wsync<GS>();
  }
  __device__ bool partial_insertion_sort(int a, int b) const {
    int i = a + 1;
    for (int step = 0; step < 5; step++) {
      i = first_descent(i, b);
      if (i == b) return true;
      if (b - a < 50) return false;
      swap1(i, i - 1);
      if (i - a >= 2) shift_left(i - 1);
      if (b - i >= 2) shift_right(i + 1, b);
    }
    return false;
  }
  // fused() on ranges of at most 64 positions, in registers: lane x holds position a + x (one LDS read, one
  // LDS write). The virtual first swap puts the pivot element at lane 0 and old e[a] at the pivot's lane;
  // among lanes 1.. the t-th L stopper from the left and the t-th R stopper from the right exchange while
  // the L is left of the R (a prefix of t: Go's Hoare loop); each lane pulls its partner's element
  // (ds_bpermute); strict then swaps lanes j = #R and 0.
  __device__ int fused64(int a, int b, int pivot, uint32_t P, bool strict, int* npairs) const {
    const int lane = lane_id(), len = b - a, px = pivot - a;
    const bool in = lane < len;
    const uint32_t raw = e[in ? a + lane : a];
    const uint32_t Ea = (uint32_t)__builtin_amdgcn_readlane((int)raw, 0);
    const uint32_t Ep = (uint32_t)__builtin_amdgcn_readlane((int)raw, px);
    const uint32_t v = lane == 0 ? Ep : (lane == px ? Ea : raw);
    const uint32_t thr = strict ? ((P << 16) | 0xFFFFu) : ((P << 16) - 1u);
    const bool P0eq = !strict && P == 0;
    const bool scan = in && lane >= 1;
    const bool isR = scan && (P0eq || v > thr);
    const uint64_t mR = ballot(isR), mL = ballot(scan && !isR);
    const int cR = popc64(mR), cL = popc64(mL);
    const int np = cL < cR ? cL : cR;
    // rank: an L lane's from the left, an R lane's from the right; the partner is the other kind's same rank
    const int t = isR ? cR - 1 - mbcnt(mR) : mbcnt(mL);
    const bool paired = scan && t < np;
    const int partner = isR ? nth_bit(mL, t) : nth_bit(mR, cR - 1 - t);
    const bool sw = paired && (isR ? partner < lane : lane < partner);
    uint32_t nv = (uint32_t)__builtin_amdgcn_ds_bpermute((sw ? partner : lane) << 2, (int)v);
    if (strict) {  // swap(j, a): j = a + #R
      const uint32_t vj = (uint32_t)__builtin_amdgcn_readlane((int)nv, cR);
      const uint32_t v0 = (uint32_t)__builtin_amdgcn_readlane((int)nv, 0);
      nv = lane == 0 ? vj : (lane == cR ? v0 : nv);
    }
    if (in) e[a + lane] = nv;
    wsync<GS>();
    *npairs = popc64(ballot(sw && !isR));
    return cR;
  }
  // Fused partition / partitionEqual of [a, b) around the element at `pivot` (key P). strict:
  // right stoppers R = key > P (partition, with the final swap); else R = key >= P (partitionEqual).
  // Returns #R; *npairs = number of misplaced pairs (Go's swap count in the Hoare loop).
  __device__ int fused(int a, int b, int pivot, uint32_t P, bool strict, int* npairs) const {
    const int lane = lane_id();
    const uint32_t Ea = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[a]);  // S[pivot] = old e[a]
    // thresholds on packed values: key > P <=> v > P << 16 | 0xFFFF; key >= P <=> v >= P << 16
    const uint32_t thr = strict ? ((P << 16) | 0xFFFFu) : ((P << 16) - 1u);  // R: v > thr (P = 0: all)
    const bool P0eq = !strict && P == 0;
    // pass 1: stoppers of [a+1, b) through the virtual first swap
    int cL = 0, cR = 0;
    for (int c0 = a + 1; c0 < b; c0 += WAVE) {
      const int p = c0 + lane;
      const bool in = p < b;
      const uint32_t raw = e[in ? p : b - 1];
      const uint32_t v = p == pivot ? Ea : raw;
      const bool isR = in && (P0eq || v > thr);
      const uint64_t mR = ballot(isR);
      const int rR = mbcnt(mR);
      uint16_t* dst = isR ? posR + (cR + rR) : posL + (cL + lane - rR);
      *dst = (uint16_t)p;
      const int nin = b - c0 < WAVE ? b - c0 : WAVE;
      const int nr = popc64(mR);
      cR += nr;
      cL += nin - nr;
    }
    wsync<GS>();
    const int m = cR;
    const int j = a + m;  // partition: the pivot's final position
    // the special positions, read before any pair is written: S[j] (strict), the pivot element
    const uint32_t Ep = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[pivot]);  // the pivot element (memory)
    const uint32_t Sj = j == pivot ? Ea : (j == a ? Ep : (uint32_t)__builtin_amdgcn_readfirstlane((int)e[j]));
    // a misplaced position holds the wrong kind for its region: L in [a+1, a+m], R in [a+m+1, b)
    const bool Ea_R = P0eq || Ea > thr;
    const bool pivot_paired = pivot != a && (pivot <= j ? !Ea_R : Ea_R);
    const bool j_paired = strict && m > 0 && !(P0eq || Sj > thr);
    const int np = cL < cR ? cL : cR;
    int t_n = 0;
    for (int t0 = 0; t0 < np; t0 += WAVE) {
      const int t = t0 + lane;
      const int l = posL[t];  // t < np + 64 <= n + 64: inside posL
      const int ri = cR - 1 - t;
      const int r = posR[ri > 0 ? ri : 0];
      const bool sw = t < np && l < r;
      const uint64_t mk = ballot(sw);
      t_n += popc64(mk);
      if (sw) {
        const uint32_t el = e[l], er = e[r];
        const uint32_t vl = l == pivot ? Ea : el, vr = r == pivot ? Ea : er;
        e[r] = vl;
        e[strict && l == j ? a : l] = vr;  // the element paired into j takes the final swap to a
      }
      if (~mk) break;  // a prefix: once a t fails, every later t fails
    }
    if (lane == 0) {
      if (strict) {
        if (m > 0 && !j_paired) e[a] = Sj;  // final swap(j, a): S[j] to a ...
        e[j] = Ep;                          // ... and the pivot element to j (m = 0: j = a)
      } else if (pivot != a) {
        e[a] = Ep;  // the first swap: the pivot element to a
      }
      if (pivot != a && !pivot_paired && !(strict && pivot == j)) e[pivot] = Ea;  // old e[a] to `pivot`
    }
    wsync<GS>();
    *npairs = t_n;
    return m;
  }
  // ---- workgroup-wide replay of the long ranges (schedule_row_kernel): every wave of the block runs the
  // same scalar control flow on the same LDS data; partitions of ranges longer than `thr` are split over
  // the waves, the rare O(1) / rare-path steps run on wave 0 between barriers. The state is then handed to
  // wave 0 (select_from) for the short ranges.
  struct State {
    int a, b, limit;
    bool wasBalanced, wasPartitioned, done;
  };
  // partition / partitionEqual of [a, b) over nw waves (fused(), same permutation): pass 1 counts each
  // wave's stoppers over its contiguous chunk segment, scatters them at the block offsets; pass 2 hands
  // t-chunks of the stopper pairs round-robin to the waves. sh: LDS ints [3 * nw]. Returns #R; *swapped:
  // some misplaced pair was exchanged (Go's alreadyPartitioned is its negation). Callers barrier before
  // (every wave's earlier reads of e are done); returns after a barrier.
  __device__ int fused_block(int a, int b, int pivot, uint32_t P, bool strict, bool* swapped, int nw, int wv,
                             int* sh) const {
    const int lane = lane_id();
    const uint32_t Ea = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[a]);
    const uint32_t thr = strict ? ((P << 16) | 0xFFFFu) : ((P << 16) - 1u);
    const bool P0eq = !strict && P == 0;
    const int first = a + 1;
    const int nchunk = (b - first + WAVE - 1) / WAVE;
    const int per = (nchunk + nw - 1) / nw;
    const int c_lo = wv * per, c_hi = (c_lo + per) < nchunk ? (c_lo + per) : nchunk;
    auto classify = [&](int c, int& p) -> bool {
      p = first + c * WAVE + lane;
      const bool in = p < b;
      const uint32_t raw = e[in ? p : b - 1];
      const uint32_t v = p == pivot ? Ea : raw;
      return in && (P0eq || v > thr);
    };
    int myR = 0, myL = 0;
    for (int c = c_lo; c < c_hi; ++c) {
      int p;
      const int nr = popc64(ballot(classify(c, p)));
      const int nin = b - (first + c * WAVE) < WAVE ? b - (first + c * WAVE) : WAVE;
      myR += nr;
      myL += nin - nr;
    }
    if (lane == 0) {
      sh[wv] = myR;
      sh[nw + wv] = myL;
    }
    __syncthreads();
    int offR = 0, offL = 0, cR = 0, cL = 0;
    for (int i = 0; i < nw; ++i) {
      const int r = sh[i], l = sh[nw + i];
      offR += i < wv ? r : 0;
      offL += i < wv ? l : 0;
      cR += r;
      cL += l;
    }
    for (int c = c_lo; c < c_hi; ++c) {  // only the range's last chunk has lanes past b: into posL's tail
      int p;
      const bool isR = classify(c, p);
      const uint64_t mR = ballot(isR);
      const int rR = mbcnt(mR);
      uint16_t* dst = isR ? posR + (offR + rR) : posL + (offL + lane - rR);
      *dst = (uint16_t)p;
      const int nin = b - (first + c * WAVE) < WAVE ? b - (first + c * WAVE) : WAVE;
      const int nr = popc64(mR);
      offR += nr;
      offL += nin - nr;
    }
    __syncthreads();
    const int m = cR;
    const int j = a + m;
    const uint32_t Ep = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[pivot]);
    const uint32_t Sj = j == pivot ? Ea : (j == a ? Ep : (uint32_t)__builtin_amdgcn_readfirstlane((int)e[j]));
    __syncthreads();  // every wave read the special positions before any pair is written
    const bool Ea_R = P0eq || Ea > thr;
    const bool pivot_paired = pivot != a && (pivot <= j ? !Ea_R : Ea_R);
    const bool j_paired = strict && m > 0 && !(P0eq || Sj > thr);
    const int np = cL < cR ? cL : cR;
    bool any = false;
    for (int t0 = wv * WAVE; t0 < np; t0 += nw * WAVE) {
      const int t = t0 + lane;
      const int l = posL[t];  // t < np + 64 <= n + 64: inside posL
      const int ri = cR - 1 - t;
      const int r = posR[ri > 0 ? ri : 0];
      const bool sw = t < np && l < r;
      const uint64_t mk = ballot(sw);
      any |= mk != 0;
      if (sw) {
        const uint32_t el = e[l], er = e[r];
        const uint32_t vl = l == pivot ? Ea : el, vr = r == pivot ? Ea : er;
        e[r] = vl;
        e[strict && l == j ? a : l] = vr;
      }
      if (~mk) break;  // a prefix: every later t fails
    }
    if (lane == 0) sh[2 * nw + wv] = any ? 1 : 0;
    __syncthreads();
    if (wv == 0 && lane == 0) {
      if (strict) {
        if (m > 0 && !j_paired) e[a] = Sj;
        e[j] = Ep;
      } else if (pivot != a) {
        e[a] = Ep;
      }
      if (pivot != a && !pivot_paired && !(strict && pivot == j)) e[pivot] = Ea;
    }
    int anyall = 0;
    for (int i = 0; i < nw; ++i) anyall |= sh[2 * nw + i];
    __syncthreads();
    *swapped = anyall != 0;
    return m;
  }
  __device__ State select_block(int n, int k, int thr, int nw, int wv, int* sh) const {
    State s{0, n, 32 - __clz(n), true, true, false};
    while (s.a < k && k < s.b && s.b - s.a > thr) {  // thr >= 12: no insertion sort here
      const int a = s.a, b = s.b, length = b - a;
      if (s.limit == 0) {
        if (wv == 0 && lane_id() == 0) {
          PackedLdsStore st{e};
          PdqT<PackedLdsStore> hs{st, xs_b, xs_c};
          hs.heap_sort(a, b);
        }
        __syncthreads();
        s.done = true;
        return s;
      }
      if (!s.wasBalanced) {
        if (wv == 0) break_patterns(a, b);
        __syncthreads();
        s.limit--;
      }
      int hint;
      uint32_t pk, prev;
      int pivot = choose_pivot(a, b, hint, pk, prev);
      if (hint == 2) {
        __syncthreads();
        if (wv == 0) reverse_range(a, b);
        __syncthreads();
        pivot = (b - 1) - (pivot - a);
        hint = 1;
      }
      if (s.wasBalanced && s.wasPartitioned && hint == 1) {
        __syncthreads();
        if (wv == 0) {
          const bool d = partial_insertion_sort(a, b);
          if (lane_id() == 0) sh[0] = d ? 1 : 0;
        }
        __syncthreads();
        const bool d = __builtin_amdgcn_readfirstlane(sh[0]) != 0;
        if (d) {
          __syncthreads();
          s.done = true;
          return s;
        }
        pk = E(pivot) >> 16;
        if (a > 0) prev = E(a - 1) >> 16;
      }
      __syncthreads();  // every wave's reads of e are done before the partition writes
      bool swapped;
      if (a > 0 && !(prev > pk)) {  // !less(a-1, pivot): partitionEqual
        s.a = a + 1 + fused_block(a, b, pivot, pk, false, &swapped, nw, wv, sh);
        continue;
      }
      const int mid = a + fused_block(a, b, pivot, pk, true, &swapped, nw, wv, sh);
      s.wasPartitioned = !swapped;
      const int leftLen = mid - a, rightLen = b - mid, bt = length / 8;
      if (leftLen < rightLen) {
        if (k < mid) {
          s.b = mid;
          s.wasBalanced = s.wasPartitioned = true;
        } else if (k > mid + 1) {
          s.wasBalanced = leftLen >= bt;
          s.a = mid + 1;
        } else {
          s.done = true;
          return s;
        }
      } else {
        if (k > mid + 1) {
          s.a = mid + 1;
          s.wasBalanced = s.wasPartitioned = true;
        } else if (k < mid) {
          s.wasBalanced = rightLen >= bt;
          s.b = mid;
        } else {
          s.done = true;
          return s;
        }
      }
    }
    return s;
  }
  __device__ void select(int n, int k) const { select_from(State{0, n, 32 - __clz(n), true, true, false}, k); }
  __device__ void select_from(State st, int k) const {
    if (st.done) return;
    int a = st.a, b = st.b;
    int limit = st.limit;
    bool wasBalanced = st.wasBalanced, wasPartitioned = st.wasPartitioned;
    while (a < k && k < b) {
      const int length = b - a;
      if (length <= 12) {
        PQ_T(i0);
        insertion_sort(a, b);
        PQ_T(i1);
        PQ_ADD(2, i1 - i0);
        return;
      }
      if (limit == 0) {
        if (lane_id() == 0) {
          PackedLdsStore st{e};
          PdqT<PackedLdsStore> s{st, xs_b, xs_c};
          s.heap_sort(a, b);
        }
        wsync<GS>();
        return;
      }
      PQ_T(c0);
      if (!wasBalanced) {
        break_patterns(a, b);
        limit--;
      }
      int hint;
      uint32_t pk, prev;
      int pivot = choose_pivot(a, b, hint, pk, prev);
      if (hint == 2) {
        reverse_range(a, b);
        pivot = (b - 1) - (pivot - a);
        hint = 1;
      }
      PQ_T(c1);
      PQ_ADD(1, c1 - c0);
      if (wasBalanced && wasPartitioned && hint == 1) {
        const bool done = partial_insertion_sort(a, b);
        PQ_T(c2);
        PQ_ADD(2, c2 - c1);
        if (done) return;
        // the shifts may have moved another element to the pivot's position, and (Go's shift-left bound
        // is 1) across a
        pk = E(pivot) >> 16;
        if (a > 0) prev = E(a - 1) >> 16;
      }
      PQ_T(c3);
      PQ_ADD(3, 1);
      int T;
      if (a > 0 && !(prev > pk)) {  // !less(a-1, pivot): partitionEqual
        a = a + 1 + (length <= WAVE ? fused64(a, b, pivot, pk, false, &T) : fused(a, b, pivot, pk, false, &T));
        PQ_T(c4);
        PQ_ADD(0, c4 - c3);
        continue;
      }
      const int mid = a + (length <= WAVE ? fused64(a, b, pivot, pk, true, &T) : fused(a, b, pivot, pk, true, &T));
      PQ_T(c5);
      PQ_ADD(0, c5 - c3);
      wasPartitioned = T == 0;
      const int leftLen = mid - a, rightLen = b - mid, thr = length / 8;
      if (leftLen < rightLen) {
        if (k < mid) {  // recursion into the smaller left side
          b = mid;
          wasBalanced = wasPartitioned = true;
        } else if (k > mid + 1) {
          wasBalanced = leftLen >= thr;
          a = mid + 1;
        } else {
          return;
        }
      } else {
        if (k > mid + 1) {  // recursion into the smaller right side
          a = mid + 1;
          wasBalanced = wasPartitioned = true;
        } else if (k < mid) {
          wasBalanced = rightLen >= thr;
          b = mid;
        } else {
          return;
        }
      }
    }
  }
};

__device__ __forceinline__ uint64_t okey(int64_t x) { return (uint64_t)x ^ 0x8000000000000000ull; }

// Per-wave selection workspace (pointers into LDS or global scratch). The
// feasible clusters have been compacted, in snapshot order, to positions
// j = 0..n-1 (the order of the reference's feasible list).
struct SelWs {
  int64_t* tot;     // [n] total score of position j
  uint64_t* sel;    // [ceil(n/64)] output: selected positions
  uint16_t* perm;   // [n] permutation buffer for the straddle replay
  uint32_t* hist;   // [256]
  uint16_t* posl;   // [n] replay scratch
  uint16_t* posr;   // [n]
};

// Select the first-k set of positions 0..n-1 under Go's sort.Slice by
// descending total. Returns KAD_RF_TIE_STRADDLE if the pdqsort replay ran.
template <bool GSCR>
__device__ uint32_t select_topk(const SelWs& ws, int n, int64_t k, int64_t row_min, int64_t row_max, int xs_b,
                                int xs_c) {
  const int lane = lane_id();
  const int nch = (n + 63) >> 6;
  if (k >= n || k <= 0) {
    const bool all = k > 0;
    for (int ch = lane; ch < nch; ch += WAVE) {
      const int rem = n - ch * WAVE;
      ws.sel[ch] = all ? (rem >= WAVE ? ~0ull : ((1ull << rem) - 1)) : 0ull;
    }
    wsync<GSCR>();
    return 0;
  }
  // ---- radix select of the k-th largest total (8-bit digits over total - min)
  const uint64_t umin = okey(row_min);
  const uint64_t range = okey(row_max) - umin;
  uint64_t prefix = 0, pmask = 0;
  int64_t kk = k;
  if (range != 0) {
    const int bits = 64 - __clzll((unsigned long long)range);
    for (int shift = ((bits + 7) / 8 - 1) * 8; shift >= 0; shift -= 8) {
      for (int i = lane; i < 256; i += WAVE) ws.hist[i] = 0;
      wsync<GSCR>();
      for (int j = lane; j < n; j += WAVE) {
        const uint64_t v = okey(ws.tot[j]) - umin;
        if ((v & pmask) == prefix) atomicAdd(&ws.hist[(v >> shift) & 255], 1u);
      }
      wsync<GSCR>();
      // lane l owns digits 255-4l .. 252-4l (descending)
      int h[4];
      int s4 = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        h[q] = (int)ws.hist[255 - 4 * lane - q];
        s4 += h[q];
      }
      const int incl = wave_incl_sum_i32(s4);
      const int excl = incl - s4;
      const bool mine = excl < kk && kk <= incl;
      int digit = 0, above = 0;
      if (mine) {
        int cum = excl;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (cum + h[q] >= kk) {
            digit = 255 - 4 * lane - q;
            above = cum;
            break;
          }
          cum += h[q];
        }
      }
      const uint64_t who = ballot(mine);
      const int src = __ffsll((unsigned long long)who) - 1;
      digit = __shfl(digit, src);
      above = __shfl(above, src);
      kk -= above;
      prefix |= (uint64_t)digit << shift;
      pmask |= 0xFFull << shift;
      wsync<GSCR>();
    }
  }
  const int64_t T = (int64_t)((prefix + umin) ^ 0x8000000000000000ull);
  // ---- counts above / at the threshold
  int g = 0, e = 0;
  for (int j = lane; j < n; j += WAVE) {
    const int64_t t = ws.tot[j];
    g += t > T;
    e += t == T;
  }
  g = wave_sum_i32(g);
  e = wave_sum_i32(e);
  if (k - g == e) {  // the cut takes every tied element: no sort needed
    for (int ch = 0; ch < nch; ++ch) {
      const int j = ch * WAVE + lane;
      const uint64_t m = ballot(j < n && ws.tot[j] >= T);
      if (lane == 0) ws.sel[ch] = m;
    }
    wsync<GSCR>();
    return 0;
  }
  // ---- straddle: replay pdqsort on positions (input order) restricted to k,
  // keys permuted in place (tot is not read after the selection)
  if (range < 65536u && n < 65536) {
    // packed replay: (total - min) << 16 | position, written over tot in place (chunk c's words overlap
    // totals 32c..32c+31, read by this or an earlier chunk)
    uint32_t* e = reinterpret_cast<uint32_t*>(ws.tot);
    for (int j0 = 0; j0 < n; j0 += WAVE) {
      const int j = j0 + lane;
      const uint32_t v = j < n ? ((uint32_t)(okey(ws.tot[j]) - umin) << 16) | (uint32_t)j : 0u;
      wsync<GSCR>();
      if (j < n) e[j] = v;
    }
    for (int ch = lane; ch < nch; ch += WAVE) ws.sel[ch] = 0;
    wsync<GSCR>();
    {
      PdqWaveP<GSCR> pw{e, ws.posl, ws.posr, xs_b, xs_c};
      pw.select(n, (int)k);
    }
    wsync<GSCR>();
    for (int i = lane; i < k; i += WAVE) {
      const int j = (int)(e[i] & 0xFFFFu);
      atomicOr((unsigned long long*)&ws.sel[j >> 6], 1ull << (j & 63));
    }
    wsync<GSCR>();
    return KAD_RF_TIE_STRADDLE;
  }
  for (int j = lane; j < n; j += WAVE) ws.perm[j] = (uint16_t)j;
  for (int ch = lane; ch < nch; ch += WAVE) ws.sel[ch] = 0;
  wsync<GSCR>();
  {
    PdqWave<int64_t, GSCR> pw{ws.tot, ws.perm, ws.posl, ws.posr, xs_b, xs_c};
    pw.select(n, (int)k);
  }
  wsync<GSCR>();
  for (int i = lane; i < k; i += WAVE) {
    const int j = ws.perm[i];
    atomicOr((unsigned long long*)&ws.sel[j >> 6], 1ull << (j & 63));
  }
  wsync<GSCR>();
  return KAD_RF_TIE_STRADDLE;
}

}  // namespace kad

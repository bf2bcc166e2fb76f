// Wavefront (64-lane) primitives for gfx950 and Go integer semantics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kad {

constexpr int WAVE = 64;
constexpr int64_t I64_MAX = INT64_MAX;
constexpr int64_t I64_MIN = INT64_MIN;
constexpr int64_t NEG_INF = INT64_MIN;  // "no floor" in the clamp monoid

// opaque at every call: a comparison with the lane index is computed where it is used, not hoisted out of
// the loops around it and kept live as a 64-bit mask (which the long kernels then spill to VGPR lanes)
__device__ __forceinline__ int lane_id() {
  int l = __lane_id();
  asm volatile("" : "+v"(l));
  return l;
}
// the plain lane index (the compiler may hoist comparisons with it): the planner, whose row loop keeps
// its lane masks in registers with room to spare, is faster with them hoisted
__device__ __forceinline__ int lane_id_h() { return __lane_id(); }

// Load through the constant address space: for a wave-uniform address this
// becomes a scalar (s_load) access served by the scalar cache. Only for data
// that no kernel writes while it runs (packed snapshot / batch, requirement rows).
template <class T>
__device__ __forceinline__ T ldc(const T* p) {
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p));
}

// Launder a wave-uniform value through an empty asm: the compiler can neither
// hoist loads that depend on it out of the enclosing loop nor keep their
// results live across the kernel (each use re-loads from the scalar cache
// instead of spilling SGPRs to VGPR lanes).
template <class T>
__device__ __forceinline__ T opq(T v) {
  asm volatile("" : "+s"(v));
  return v;
}

// Global load at a 32-bit element index from a wave-uniform base: selects the
// saddr form (SGPR base + 32-bit VGPR byte offset), one VALU op per address.
template <class T>
__device__ __forceinline__ T ldg(const T* base, uint32_t i) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + (size_t)(uint32_t)(i * (uint32_t)sizeof(T)));
}
template <class T>
__device__ __forceinline__ void stg(T* base, uint32_t i, T v) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (size_t)(uint32_t)(i * (uint32_t)sizeof(T))) = v;
}

// Order LDS traffic between the lanes of one wave: one wave's LDS operations
// execute in order, so this only has to stop the compiler from moving them.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// Same for per-wave state kept in a global scratch slab (rows too large for LDS).
__device__ __forceinline__ void wave_sync_global() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
template <bool GSCR>
__device__ __forceinline__ void wsync() {
  if (GSCR)
    wave_sync_global();
  else
    wave_sync();
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ int popc64(uint64_t x) { return __popcll(x); }
// position of the s-th (0-based) set bit of m (per lane; s < popc(m)), by halving popcounts
__device__ __forceinline__ int nth_bit(uint64_t m, int s) {
  uint32_t w = (uint32_t)m;
  int pos = 0, c = __builtin_popcount(w);
  if (s >= c) {
    s -= c;
    w = (uint32_t)(m >> 32);
    pos = 32;
  }
#pragma unroll
  for (int half = 16; half >= 1; half >>= 1) {
    c = __builtin_popcount(w & ((1u << half) - 1u));
    if (s >= c) {
      s -= c;
      w >>= half;
      pos += half;
    }
  }
  return pos;
}

// number of set bits of m in lanes below this lane
// this lane's bit of a wave-uniform mask: the mask's SGPR pair is the lane predicate (v_cndmask
// reads it directly, no shift / compare)
__device__ __forceinline__ bool lane_on(uint64_t uniform_mask) { return __builtin_amdgcn_inverse_ballot_w64(uniform_mask); }
__device__ __forceinline__ int mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

__device__ __forceinline__ int64_t shfl_i64(int64_t v, int src) {
  int lo = __shfl((int)(uint32_t)v, src);
  int hi = __shfl((int)(uint32_t)((uint64_t)v >> 32), src);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t shfl_up_i64(int64_t v, int d) {
  int lo = __shfl_up((int)(uint32_t)v, d);
  int hi = __shfl_up((int)(uint32_t)((uint64_t)v >> 32), d);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t shfl_xor_i64(int64_t v, int m) {
  int lo = __shfl_xor((int)(uint32_t)v, m);
  int hi = __shfl_xor((int)(uint32_t)((uint64_t)v >> 32), m);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// ------------------------------------------------ DPP wave reductions (gfx9)
// row_shr 1/2/4/8 then row_bcast 15/31 leave the reduction of all 64 lanes in
// lane 63; readlane makes it wave-uniform (SGPR). Every lane must be active.
template <int CTRL, int RM>
__device__ __forceinline__ int dpp32(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xf, false);
}
#define KAD_DPP_STEPS(OP, ID)              \
  v = OP(v, dpp32<0x111, 0xf>(ID, v));     \
  v = OP(v, dpp32<0x112, 0xf>(ID, v));     \
  v = OP(v, dpp32<0x114, 0xf>(ID, v));     \
  v = OP(v, dpp32<0x118, 0xf>(ID, v));     \
  v = OP(v, dpp32<0x142, 0xa>(ID, v));     \
  v = OP(v, dpp32<0x143, 0xc>(ID, v));     \
  return __builtin_amdgcn_readlane(v, 63)
__device__ __forceinline__ int imax_(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int imin_(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ int iadd_(int a, int b) { return a + b; }
__device__ __forceinline__ int wave_max_u_i32(int v) { KAD_DPP_STEPS(imax_, INT32_MIN); }
__device__ __forceinline__ int wave_min_u_i32(int v) { KAD_DPP_STEPS(imin_, INT32_MAX); }
__device__ __forceinline__ int wave_sum_u_i32(int v) { KAD_DPP_STEPS(iadd_, 0); }
#undef KAD_DPP_STEPS

// min and max of one value together: the two DPP chains interleave, so each
// fills the other's DPP read-after-write wait states
__device__ __forceinline__ void wave_minmax_u_i32(int vmin, int vmax, int& rmin, int& rmax) {
  vmin = imin_(vmin, dpp32<0x111, 0xf>(INT32_MAX, vmin));
  vmax = imax_(vmax, dpp32<0x111, 0xf>(INT32_MIN, vmax));
  vmin = imin_(vmin, dpp32<0x112, 0xf>(INT32_MAX, vmin));
  vmax = imax_(vmax, dpp32<0x112, 0xf>(INT32_MIN, vmax));
  vmin = imin_(vmin, dpp32<0x114, 0xf>(INT32_MAX, vmin));
  vmax = imax_(vmax, dpp32<0x114, 0xf>(INT32_MIN, vmax));
  vmin = imin_(vmin, dpp32<0x118, 0xf>(INT32_MAX, vmin));
  vmax = imax_(vmax, dpp32<0x118, 0xf>(INT32_MIN, vmax));
  vmin = imin_(vmin, dpp32<0x142, 0xa>(INT32_MAX, vmin));
  vmax = imax_(vmax, dpp32<0x142, 0xa>(INT32_MIN, vmax));
  vmin = imin_(vmin, dpp32<0x143, 0xc>(INT32_MAX, vmin));
  vmax = imax_(vmax, dpp32<0x143, 0xc>(INT32_MIN, vmax));
  rmin = __builtin_amdgcn_readlane(vmin, 63);
  rmax = __builtin_amdgcn_readlane(vmax, 63);
}

// 64-bit max / min: reduce the high words, then the low words of the lanes
// holding the winning high word (unsigned), all wave-uniform results.
__device__ __forceinline__ int64_t wave_max_u_i64(int64_t v) {
  const int hi = (int)(v >> 32);
  const int mh = wave_max_u_i32(hi);
  const uint32_t lo = hi == mh ? (uint32_t)v : 0u;
  const uint32_t ml = (uint32_t)wave_max_u_i32((int)(lo ^ 0x80000000u)) ^ 0x80000000u;
  return (int64_t)(((uint64_t)(uint32_t)mh << 32) | ml);
}
__device__ __forceinline__ int64_t wave_min_u_i64(int64_t v) {
  const int hi = (int)(v >> 32);
  const int mh = wave_min_u_i32(hi);
  const uint32_t lo = hi == mh ? (uint32_t)v : 0xFFFFFFFFu;
  const uint32_t ml = (uint32_t)wave_min_u_i32((int)(lo ^ 0x80000000u)) ^ 0x80000000u;
  return (int64_t)(((uint64_t)(uint32_t)mh << 32) | ml);
}

// 64-bit DPP move: lanes without a source in this step get `old`
template <int CTRL, int RM>
__device__ __forceinline__ int64_t dpp64(int64_t old, int64_t v) {
  const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)old, (int)(uint32_t)v, CTRL, RM, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)((uint64_t)old >> 32), (int)(uint32_t)((uint64_t)v >> 32),
                                             CTRL, RM, 0xf, false);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {  // wrapping (Go int64); every lane active
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x111, 0xf>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x112, 0xf>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x114, 0xf>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x118, 0xf>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x142, 0xa>(0, v));
  v = (int64_t)((uint64_t)v + (uint64_t)dpp64<0x143, 0xc>(0, v));
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), 63);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) { return wave_max_u_i64(v); }
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) { return wave_min_u_i64(v); }
__device__ __forceinline__ int wave_sum_i32(int v) { return wave_sum_u_i32(v); }
// inclusive prefix sum of i32 across the wave (DPP Hillis-Steele within rows, then row broadcasts)
__device__ __forceinline__ int wave_incl_sum_i32(int v) {
  v += dpp32<0x111, 0xf>(0, v);
  v += dpp32<0x112, 0xf>(0, v);
  v += dpp32<0x114, 0xf>(0, v);
  v += dpp32<0x118, 0xf>(0, v);
  v += dpp32<0x142, 0xa>(0, v);
  v += dpp32<0x143, 0xc>(0, v);
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {  // exact for integer-valued sums < 2^53
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
// inclusive scan (sum) of i64 across the wave
__device__ __forceinline__ int64_t wave_incl_sum_i64(int64_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    int64_t o = shfl_up_i64(v, d);
    if (l >= d) v = (int64_t)((uint64_t)v + (uint64_t)o);
  }
  return v;
}

// ----------------------------------------------------------- Go integer ops
__device__ __forceinline__ int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__device__ __forceinline__ int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
__device__ __forceinline__ int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
// Go `a / b` (truncating; MinInt64 / -1 wraps to MinInt64)
__device__ __forceinline__ int64_t go_div(int64_t a, int64_t b) {
  if (b == -1) return (int64_t)(0 - (uint64_t)a);
  return a / b;
}
// floor(num / den) for 0 <= num, 0 < den when the quotient is small (< 2^20):
// f32 reciprocal estimate + exact integer correction — avoids the 64-bit
// division sequence on the hot score path.
__device__ __forceinline__ int64_t small_quot(int64_t num, int64_t den) {
  float q = (float)num * __builtin_amdgcn_rcpf((float)den);
  int64_t qi = (int64_t)q;
  int64_t r = num - qi * den;
  while (r < 0) { qi--; r += den; }
  while (r >= den) { qi++; r -= den; }
  return qi;
}
// Go float64 → int64 on amd64: NaN / out of range → MinInt64
__device__ __forceinline__ int64_t go_f2i(double x) {
  if (!(x < 9223372036854775808.0) || !(x >= -9223372036854775808.0)) return I64_MIN;
  return (int64_t)x;
}

// FNV-1 32 continuation (hash/fnv New32)
__device__ __forceinline__ uint32_t fnv_cont(uint32_t h, const uint8_t* p, int n) {
  for (int i = 0; i < n; i++) {
    h *= 16777619u;
    h ^= p[i];
  }
  return h;
}

}  // namespace kad

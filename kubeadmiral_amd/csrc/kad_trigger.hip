// Scheduling-trigger hashes (schedulingtriggers.go:106-147) on gfx950.
//
// The reference hashes, per federated object, FNV-1 32 over json.Marshal of
// {object part ‖ cluster part}; the cluster part (labels, taints and API
// resources of every joined cluster, :193-262) is identical for every object
// of a pass and is nearly all of the bytes (≈1.6 MB at 256 clusters against
// ≈200 B of object part). The reference folds it once per object.
//
// FNV-1 step: h' = (h·p mod 2^32) ⊕ b. The low byte of h' depends only on the
// low byte of h (the product's low byte is (h mod 256)·(p mod 256) mod 256 and
// ⊕b touches only the low byte), and ⊕b adds a value that depends only on that
// low byte. Unrolled over a byte string B of length L:
//      F_B(h) = T_B[h & 255] + (h & ~255)·p^L            (mod 2^32)
// with T_B[r] = F_B(r) for the 256 residues r. Two strings compose as
//      T_AB[r] = T_B[T_A[r] & 255] + (T_A[r] & ~255)·P_B,   P_AB = P_A·P_B.
// So the cluster part is summarised by a 256-entry table, built in parallel:
//   1. trig_segment_kernel  one workgroup per L-byte segment, one lane per
//                           residue: T_seg[r] = FNV fold of the segment from r
//                           (segment bytes are wave-uniform: scalar loads)
//   2. trig_compose_kernel  groups of G segment tables → one table (LDS),
//                           repeated until one table is left
//   3. trig_object_kernel   one lane per object: fold its own bytes → h0,
//                           hash = T[h0 & 255] + (h0 & ~255)·P
// Work: 256·|cluster part| FNV steps per pass + each object's own bytes,
// instead of |cluster part| per object.
#include "kad_device.h"

namespace kad {

constexpr uint32_t kFnvPrime = 16777619u;
constexpr uint32_t kFnvOffset = 2166136261u;
constexpr int kComposeGroup = 32;  // tables composed per workgroup (32 KiB of LDS)

__host__ __device__ inline uint32_t fnv_pow(uint64_t n) {
  uint32_t r = 1u, b = kFnvPrime;
  while (n) {
    if (n & 1) r *= b;
    b *= b;
    n >>= 1;
  }
  return r;
}

__device__ __forceinline__ uint32_t fnv_word(uint32_t h, uint32_t w) {
  h = (h * kFnvPrime) ^ (w & 0xffu);
  h = (h * kFnvPrime) ^ ((w >> 8) & 0xffu);
  h = (h * kFnvPrime) ^ ((w >> 16) & 0xffu);
  return (h * kFnvPrime) ^ (w >> 24);
}

// grid = n_seg workgroups of 256 lanes (lane = residue). seg_len is a multiple of 64.
__global__ __launch_bounds__(256) void trig_segment_kernel(const uint32_t* __restrict__ suf, int64_t nbytes,
                                                           int64_t seg_len, uint32_t* __restrict__ tab,
                                                           uint32_t* __restrict__ pw) {
  const int64_t a = (int64_t)blockIdx.x * seg_len;
  const int64_t e = a + seg_len < nbytes ? a + seg_len : nbytes;
  uint32_t h = threadIdx.x;
  const int64_t nblk = (e - a) >> 6;
  const uint32_t* p0 = suf + (a >> 2);
  for (int64_t blk = 0; blk < nblk; ++blk) {
    const uint32_t* p = p0 + (blk << 4);
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = p[t];
#pragma unroll
    for (int t = 0; t < 16; ++t) h = fnv_word(h, w[t]);
  }
  const uint8_t* bytes = reinterpret_cast<const uint8_t*>(suf);
  for (int64_t q = a + (nblk << 6); q < e; ++q) h = (h * kFnvPrime) ^ bytes[q];
  tab[(size_t)blockIdx.x * 256 + threadIdx.x] = h;
  if (threadIdx.x == 0) pw[blockIdx.x] = fnv_pow((uint64_t)(e - a));
}

// grid = ceil(n_in / G) workgroups of 256 lanes: compose tables [g·G, min((g+1)·G, n_in)) in order.
__global__ __launch_bounds__(256) void trig_compose_kernel(const uint32_t* __restrict__ tin,
                                                           const uint32_t* __restrict__ pin, int n_in,
                                                           uint32_t* __restrict__ tout, uint32_t* __restrict__ pout) {
  __shared__ uint32_t lt[kComposeGroup][256];
  const int k0 = blockIdx.x * kComposeGroup;
  const int nk = n_in - k0 < kComposeGroup ? n_in - k0 : kComposeGroup;
  for (int k = 0; k < nk; ++k) lt[k][threadIdx.x] = tin[(size_t)(k0 + k) * 256 + threadIdx.x];
  __syncthreads();
  uint32_t v = lt[0][threadIdx.x];
  uint32_t pp = pin[k0];
  for (int k = 1; k < nk; ++k) {
    const uint32_t pk = pin[k0 + k];  // uniform: scalar load
    v = lt[k][v & 255u] + (v & ~255u) * pk;
    pp *= pk;
  }
  tout[(size_t)blockIdx.x * 256 + threadIdx.x] = v;
  if (threadIdx.x == 0) pout[blockIdx.x] = pp;
}

// one lane per object; tab/pw: the cluster part's table (nullptr: empty cluster part)
__global__ __launch_bounds__(256) void trig_object_kernel(const uint8_t* __restrict__ pre,
                                                          const int64_t* __restrict__ off, int n,
                                                          const uint32_t* __restrict__ tab,
                                                          const uint32_t* __restrict__ pw,
                                                          uint32_t* __restrict__ out) {
  __shared__ uint32_t lt[256];
  if (tab) lt[threadIdx.x] = tab[threadIdx.x];
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int64_t a = off[i];
  const int64_t b = off[i + 1];
  uint32_t h = kFnvOffset;
  for (; a < b && (a & 3); ++a) h = (h * kFnvPrime) ^ pre[a];
  const uint32_t* w = reinterpret_cast<const uint32_t*>(pre);
  for (; a + 4 <= b; a += 4) h = fnv_word(h, w[a >> 2]);
  for (; a < b; ++a) h = (h * kFnvPrime) ^ pre[a];
  out[i] = tab ? lt[h & 255u] + (h & ~255u) * pw[0] : h;
}

int64_t trigger_segment_len(int64_t nbytes) {
  // ~8k segments (2M residue lanes) at the sizes that matter, each ≥ 64 B
  int64_t L = (nbytes / 8192 + 63) & ~(int64_t)63;
  return L < 64 ? 64 : L;
}

int64_t trigger_table_count(int64_t nbytes) {
  if (nbytes <= 0) return 0;
  const int64_t L = trigger_segment_len(nbytes);
  int64_t k = (nbytes + L - 1) / L, tot = k;
  while (k > 1) {
    k = (k + kComposeGroup - 1) / kComposeGroup;
    tot += k;
  }
  return tot;
}

hipError_t launch_trigger_summary(const TriggerDev& t, hipStream_t st) {
  if (t.suffix_len <= 0) return hipSuccess;
  const int64_t L = trigger_segment_len(t.suffix_len);
  int k = (int)((t.suffix_len + L - 1) / L);
  uint32_t* tab = t.tables;
  uint32_t* pw = t.powers;
  trig_segment_kernel<<<k, 256, 0, st>>>(t.suffix, t.suffix_len, L, tab, pw);
  while (k > 1) {
    const int k2 = (k + kComposeGroup - 1) / kComposeGroup;
    trig_compose_kernel<<<k2, 256, 0, st>>>(tab, pw, k, tab + (size_t)k * 256, pw + k);
    tab += (size_t)k * 256;
    pw += k;
    k = k2;
  }
  return hipGetLastError();
}

const uint32_t* trigger_final_table(const TriggerDev& t, const uint32_t** pw) {
  const int64_t tot = trigger_table_count(t.suffix_len);
  if (tot == 0) {
    *pw = nullptr;
    return nullptr;
  }
  *pw = t.powers + (tot - 1);
  return t.tables + (size_t)(tot - 1) * 256;
}

hipError_t launch_trigger_objects(const TriggerDev& t, hipStream_t st) {
  if (t.n <= 0) return hipSuccess;
  const uint32_t* pw = nullptr;
  const uint32_t* tab = trigger_final_table(t, &pw);
  trig_object_kernel<<<(t.n + 255) / 256, 256, 0, st>>>(t.prefix, t.prefix_off, t.n, tab, pw, t.out);
  return hipGetLastError();
}

}  // namespace kad

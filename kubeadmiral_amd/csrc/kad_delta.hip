// kad_snapshot_update on gfx950: in-place cluster column updates of the resident snapshot.
//
// A cluster status/label/taint event (scheduler.go:157-177) rewrites a few
// clusters; the snapshot is attribute-major (attr[r*C + c]), so one changed
// cluster touches one element in every row of every array. The delta blob
// holds those elements row by row ([r][j]); one lane moves one element.
#include "kad_device.h"

namespace kad {

__global__ __launch_bounds__(256) void snapshot_delta_kernel(DeltaDev d) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= d.start[KAD_S_NARRAYS]) return;
  int a = 0;
  while (e >= d.start[a + 1]) ++a;  // 17 arrays: uniform scalar loads, short scan
  const int64_t k = e - d.start[a];
  const int64_t r = k / d.n;
  const int j = (int)(k - r * d.n);
  const int64_t dst = (int64_t)d.s_off[a] + (r * d.C + d.idx[j]) * d.esz[a];
  const int64_t src = (int64_t)d.d_off[a] + k * d.esz[a];
  switch (d.esz[a]) {
    case 8: *reinterpret_cast<uint64_t*>(d.snap + dst) = *reinterpret_cast<const uint64_t*>(d.delta + src); break;
    case 4: *reinterpret_cast<uint32_t*>(d.snap + dst) = *reinterpret_cast<const uint32_t*>(d.delta + src); break;
    default: d.snap[dst] = d.delta[src]; break;
  }
}

hipError_t launch_snapshot_delta(const DeltaDev& d, hipStream_t st) {
  const int64_t n = d.start[KAD_S_NARRAYS];
  if (n <= 0) return hipSuccess;
  snapshot_delta_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d);
  return hipGetLastError();
}

}  // namespace kad

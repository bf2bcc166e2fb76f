// Result application diff (§8 f3) on gfx950: which units' results change their federated object.
//
// applySchedulingResult (pkg/controllers/scheduler/scheduler.go:632-695) rewrites the scheduler's placement
// when the result's cluster SET differs from the placement's (SetPlacementNames, reflect.DeepEqual of two
// map[string]struct{}, types/v1alpha1/extensions_placements.go:78-103; an empty result deletes the placement,
// a change iff it existed) and the replicas overrides when OverrideUpdateNeeded (scheduler/util.go:154-185)
// finds a replicas-path patch whose value is not a float64, whose cluster has no replica count in the result,
// or whose int64(value) differs from it, or when the number of matching patches is not the number of result
// entries with a replica count. One lane per unit: the result slots of a unit are ascending cluster
// positions (every schedule / plan kernel writes them so), the canonical placement ids too (host-sorted,
// unique), so the set test is one pass and each patch a binary search.
#include "kad_device.h"

namespace kad {

__global__ __launch_bounds__(256) void result_diff_kernel(ResultDiffDev d) {
  const int w = (int)(blockIdx.x * 256 + threadIdx.x);
  if (w >= d.W) return;
  const int32_t st = d.status[w];
  uint32_t f = 0;
  if (st == KAD_ST_ERR_SCORE || st == KAD_ST_ERR_SELECT || st == KAD_ST_ERR_REPLICAS) {
    d.out[w] = KAD_DIFF_SKIP;  // Schedule returned an error: nothing is applied
    return;
  }
  if (st == KAD_ST_STICKY) {
    d.out[w] = KAD_DIFF_STICKY;
    return;
  }
  const int n = st == KAD_ST_OK ? d.count[w] : 0;  // NO_FEASIBLE: the nil map
  const int32_t* cl = d.cluster + d.out_off[w];
  const int64_t* rp = d.replicas + d.out_off[w];
  // ---- placement: SetPlacementNames(controller, result cluster set)
  const uint8_t uf = d.uflag[w];
  const int p0 = d.pl_off[w], np = d.pl_off[w + 1] - p0;
  bool pc;
  if (n == 0) {
    pc = uf & 1;  // DeletePlacement: a change iff the placement existed
  } else {
    pc = (uf & 2) || np != n;  // a name outside the snapshot never is in the result
    for (int i = 0; !pc && i < n; ++i) pc = d.pl_id[p0 + i] != cl[i];
  }
  if (pc) f |= KAD_DIFF_PLACEMENT;
  // ---- overrides: OverrideUpdateNeeded(typeConfig, overrides, {cluster: replicas} of the non-nil counts)
  int nres = 0;
  for (int i = 0; i < n; ++i) nres += rp[i] >= 0;  // Duplicate results carry nil (-1) counts
  const int o0 = d.ov_off[w], o1 = d.ov_off[w + 1];
  bool oc = false;
  int checked = 0;
  for (int o = o0; o < o1 && !oc; ++o) {
    if (d.ov_kind[o] != 0) {
      oc = true;  // the value is not a float64
      break;
    }
    const int id = d.ov_id[o];
    int lo = 0, hi = n;  // first slot with cluster >= id
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cl[mid] < id)
        lo = mid + 1;
      else
        hi = mid;
    }
    if (id < 0 || lo >= n || cl[lo] != id || rp[lo] < 0 || rp[lo] != d.ov_val[o]) oc = true;
    ++checked;
  }
  if (oc || checked != nres) f |= KAD_DIFF_OVERRIDES;
  d.out[w] = f;
}

hipError_t launch_result_diff(const ResultDiffDev& d, hipStream_t st) {
  if (d.W <= 0) return hipSuccess;
  result_diff_kernel<<<(unsigned)((d.W + 255) / 256), 256, 0, st>>>(d);
  return hipGetLastError();
}

}  // namespace kad

// Device-side views of the packed snapshot / batch (include/kad_sched.h) and
// the kernel launchers of libkad.so. gfx950 (MI355X) only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kad_sched.h"

namespace kad {

struct SnapDev {
  int C, GW, TW, K, S;
  const int64_t *alloc_cpu, *alloc_mem, *used_cpu, *used_mem, *alloc_s, *used_s, *alloc_cores, *avail_cores;
  const uint64_t *gvk, *nsne, *ne, *pns;
  const int32_t* lval;
  const int64_t* lint;
  const uint8_t* lok;
  const uint32_t* name_fnv;
};

struct BatchDev {
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
  const int64_t *pref_w, *pref_min, *pref_max, *pref_cap;
  const uint32_t* pref_fl;
  const int32_t* key_off;
  const uint8_t* key;
  const int64_t* out_off;
  int NR;                   // distinct requirements
  const int32_t *req_off, *req;
  uint64_t* req_mask;       // device workspace [NR][ceil(C/64)]: requirement × cluster bitmask
};

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

// bytes of per-wave scratch for the filter/score/select kernel at C clusters
size_t select_wave_bytes(int C);
size_t plan_wave_bytes(int K);

// phase counters of a -DKAD_PHASE_PROF build (returns 0 in product builds)
int debug_phase_counters(uint64_t* out, int reset);

hipError_t launch_req_masks(const SnapDev& s, const BatchDev& b, hipStream_t st);
hipError_t launch_schedule(const SnapDev& s, const BatchDev& b, const OutDev& o, const ProfDev& p,
                           void* global_scratch, size_t scratch_bytes, hipStream_t st);
hipError_t launch_plan(const SnapDev& s, const BatchDev& b, const OutDev& o, const ProfDev& p, const int32_t* rows,
                       int n_rows, int kmax, void* global_scratch, size_t scratch_bytes, hipStream_t st);
hipError_t launch_select_rows(int n_rows, const int32_t* row_off, const int64_t* scores, const int64_t* maxc,
                              uint32_t pflags, int kmax, int32_t* out_count, int32_t* out_sel, int32_t* out_status,
                              void* global_scratch, size_t scratch_bytes, hipStream_t st);
hipError_t launch_plan_rows(const PlanRowsDev& r, int kmax, void* global_scratch, size_t scratch_bytes,
                            hipStream_t st);

}  // namespace kad

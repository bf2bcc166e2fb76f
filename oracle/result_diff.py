"""TEST INFRASTRUCTURE ONLY — restatement of the two result-dependent halves of applySchedulingResult.

``pkg/controllers/scheduler/scheduler.go:632-695``: for one unit's ScheduleResult and its federated object,
* placementUpdated = SetPlacementNames(controller, result.ClusterSet())
  (``pkg/apis/types/v1alpha1/extensions_placements.go:78-103``): an empty set deletes the controller's
  placement (a change iff it existed, ``:55-76``); otherwise the first placement of the controller
  (created empty if missing) changes iff its cluster-name SET differs (reflect.DeepEqual of two maps);
* overridesUpdated = OverrideUpdateNeeded(typeConfig, overrides, desired)
  (``pkg/controllers/scheduler/util.go:154-185``) with desired = {cluster: *replicas} of the non-nil counts.
Written over kad_result_state's arrays (one unit's placement ids / override patches) and a BatchResult, the
form the device kernel reads; tests pin it against the object-level functions of kubeadmiral_amd/objects.py
(which restate the same Go on unstructured objects) and check the GPU's kad_result_diff against it.
"""

from __future__ import annotations

import numpy as np

PLACEMENT, OVERRIDES, SKIP, STICKY = 1, 2, 4, 8
ST_OK, ST_STICKY, ST_NO_FEASIBLE = 0, 1, 2


def diff_flags(res, out_off, state) -> np.ndarray:
    """Per unit KAD_DIFF_* flags (res: BatchResult of the schedule; out_off: the batch's slot offsets)."""
    W = len(state["place_has"])
    out = np.zeros(W, np.uint32)
    po, pc_, ph = state["place_off"], state["place_cluster"], state["place_has"]
    oo, oc_, ov, ok = state["ovr_off"], state["ovr_cluster"], state["ovr_value"], state["ovr_kind"]
    for w in range(W):
        st = int(res.status[w])
        if st == ST_STICKY:
            out[w] = STICKY
            continue
        if st not in (ST_OK, ST_NO_FEASIBLE):
            out[w] = SKIP  # Schedule returned an error: nothing applied (scheduler.go:505-517)
            continue
        n = int(res.count[w]) if st == ST_OK else 0
        a = int(out_off[w])
        result = {int(res.cluster[a + i]): int(res.replicas[a + i]) for i in range(n)}
        f = 0
        old = {int(x) for x in pc_[po[w]:po[w + 1]]}
        if not result:
            if ph[w]:
                f |= PLACEMENT  # DeletePlacement
        elif old != set(result):  # -1 (a name outside the snapshot) never is a result cluster
            f |= PLACEMENT
        desired = {c: r for c, r in result.items() if r >= 0}  # Duplicate: nil counts (-1)
        checked = 0
        changed = False
        for i in range(oo[w], oo[w + 1]):
            if ok[i] != 0:  # the value is not a float64
                changed = True
                break
            c = int(oc_[i])
            if c not in desired or int(ov[i]) != desired[c]:
                changed = True
                break
            checked += 1
        if changed or checked != len(desired):
            f |= OVERRIDES
        out[w] = f
    return out

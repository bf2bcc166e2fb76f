"""Batch results ↔ ScheduleResult objects (include/kad_sched.h, kad_result_view)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Union

import numpy as np

from . import types as T
from .pack import ST_ERR_REPLICAS, ST_ERR_SCORE, ST_ERR_SELECT, ST_NO_FEASIBLE, ST_OK, ST_STICKY, Batch

_ERR_STAGE = {ST_ERR_SCORE: "scoreClusters", ST_ERR_SELECT: "selectClusters", ST_ERR_REPLICAS: "replicaScheduling"}


@dataclass
class BatchResult:
    status: np.ndarray    # i32[W]
    count: np.ndarray     # i32[W]
    flags: np.ndarray     # u32[W]
    cluster: np.ndarray   # i32[n_out_slots]
    replicas: np.ndarray  # i64[n_out_slots]
    out_off: np.ndarray   # i64[W+1]

    @staticmethod
    def empty(batch: Batch) -> "BatchResult":
        W, n = batch.W, max(1, batch.n_out_slots)
        return BatchResult(np.zeros(W, np.int32), np.zeros(W, np.int32), np.zeros(W, np.uint32),
                           np.full(n, -1, np.int32), np.zeros(n, np.int64), batch.out_off)

    @staticmethod
    def pinned(W: int, n_slots: int) -> "BatchResult":
        """Page-locked result arrays (kad_host_alloc) for Context.download(out=...): the D2H copies then DMA
        straight into them. Reuse them across batches of at most W units / n_slots slots."""
        from .runtime import host_array

        return BatchResult(host_array(W, np.int32), host_array(W, np.int32), host_array(W, np.uint32),
                           host_array(n_slots, np.int32), host_array(n_slots, np.int64), np.zeros(1, np.int64))

    def row(self, w: int):
        """(status, [(cluster_id, replicas), ...]) for unit w, ascending cluster id."""
        o = int(self.out_off[w])
        k = int(self.count[w])
        return int(self.status[w]), list(zip(self.cluster[o:o + k].tolist(), self.replicas[o:o + k].tolist()))

    def equal_rows(self, other: "BatchResult") -> np.ndarray:
        """Boolean[W]: row w identical (status, count, pairs) in both results."""
        eq = (self.status == other.status) & (self.count == other.count)
        W = len(self.status)
        if W == 0:
            return eq
        # compare slot contents within each row's used range
        idx = np.arange(len(self.cluster))
        row = np.searchsorted(self.out_off, idx, side="right") - 1
        row = np.clip(row, 0, W - 1)
        used = (idx - self.out_off[row]) < self.count[row]
        diff = used & ((self.cluster != other.cluster) | (self.replicas != other.replicas))
        bad = np.zeros(W, bool)
        np.logical_or.at(bad, row[diff], True)
        return eq & ~bad


def to_schedule_result(res: BatchResult, w: int, unit: T.SchedulingUnit, names: List[str]
                       ) -> Union[T.ScheduleResult, T.ScheduleError]:
    """Rebuild the Go-side ScheduleResult (generic_scheduler.go:92-150) for unit w."""
    st, pairs = res.row(w)
    if st == ST_STICKY:
        return T.ScheduleResult(unit.current_clusters)
    if st == ST_NO_FEASIBLE:
        return T.ScheduleResult(None)
    if st in _ERR_STAGE:
        return T.ScheduleError(_ERR_STAGE[st])
    if st != ST_OK:
        raise RuntimeError(f"unit {w}: invalid status {st}")
    return T.ScheduleResult({names[c]: (None if r < 0 else int(r)) for c, r in pairs})


def to_schedule_result_cols(res: BatchResult, w: int, cols, names: List[str]
                            ) -> Union[T.ScheduleResult, T.ScheduleError]:
    """:func:`to_schedule_result` for unit w of a columnar batch (``columns.SUColumns``): a sticky unit keeps its
    CurrentClusters, read from the columns."""
    if int(res.status[w]) == ST_STICKY:
        C = cols.cols
        S = cols.strings()
        a, b = int(C["cur_off"][w]), int(C["cur_off"][w + 1])
        cur = {S[C["cur_name"][i]]: (int(C["cur_rep"][i]) if C["cur_has_rep"][i] else None) for i in range(a, b)}
        return T.ScheduleResult(cur)  # sticky: CurrentClusters is non-empty (generic_scheduler.go:98-104)
    return to_schedule_result(res, w, None, names)

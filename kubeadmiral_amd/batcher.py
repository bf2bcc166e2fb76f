"""Coalescing ``ScheduleAlgorithm``: per-unit Schedule calls from many workers, one GPU batch.

The reference calls ``ScheduleAlgorithm.Schedule(ctx, fwk, su, clusters)``
once per object from each of ``--worker-count`` reconcile goroutines
(``scheduler.go:507``, worker pool ``pkg/controllers/util/worker/worker.go:
125-174``). :class:`CoalescingScheduler` keeps that call shape —
:meth:`CoalescingScheduler.schedule` blocks and returns the unit's
``ScheduleResult`` or raises its ``ScheduleError`` — while a dispatcher thread
gathers the calls that arrive together (up to ``max_batch`` units, or until
``max_wait_s`` after the first one) and runs them as one
:class:`~kubeadmiral_amd.runtime.BatchScheduler` batch per (framework,
cluster-list content) pair. Between batches the cluster list may change: the
BatchScheduler applies it as an in-place snapshot delta when it can.
"""

from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import Dict, List, Optional, Tuple

from . import types as T
from .framework import Framework


class CoalescingScheduler:
    def __init__(self, scheduler=None, max_batch: int = 65536, max_wait_s: float = 0.002, device: int = 0,
                 devices=None):
        """``devices``: run each gathered batch split over these GPUs (runtime.GroupContext)."""
        if scheduler is None:
            from .runtime import BatchScheduler

            scheduler = BatchScheduler(device=device, devices=devices)
        self.scheduler = scheduler
        self.max_batch = max_batch
        self.max_wait_s = max_wait_s
        self._q: "queue.Queue[Optional[tuple]]" = queue.Queue()
        self._closed = False
        self._lock = threading.Lock()
        self.batches: List[int] = []  # units per dispatched batch (observability)
        self._thread = threading.Thread(target=self._run, name="kad-coalescer", daemon=True)
        self._thread.start()

    # -------------------------------------------------------------- callers
    def submit(self, fwk: Framework, su: T.SchedulingUnit, clusters: List[T.FederatedCluster]) -> Future:
        fut: Future = Future()
        with self._lock:
            if self._closed:
                raise RuntimeError("CoalescingScheduler is closed")
            self._q.put((fwk, su, clusters, fut))
        return fut

    def schedule(self, fwk: Framework, su: T.SchedulingUnit, clusters: List[T.FederatedCluster]) -> T.ScheduleResult:
        """Schedule (generic_scheduler.go:92-150) for one unit: its result, or raise its ScheduleError."""
        r = self.submit(fwk, su, clusters).result()
        if isinstance(r, T.ScheduleError):
            raise r
        return r

    def close(self):
        with self._lock:
            if self._closed:
                return
            self._closed = True
            self._q.put(None)
        self._thread.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ----------------------------------------------------------- dispatcher
    def _gather(self, first) -> Tuple[list, bool]:
        items, stop = [first], False
        deadline = time.monotonic() + self.max_wait_s
        while len(items) < self.max_batch:
            left = deadline - time.monotonic()
            try:
                it = self._q.get(timeout=left) if left > 0 else self._q.get_nowait()
            except queue.Empty:
                break
            if it is None:
                stop = True
                break
            items.append(it)
        return items, stop

    def _run(self):
        stop = False
        while not stop:
            first = self._q.get()
            if first is None:
                break
            items, stop = self._gather(first)
            self.batches.append(len(items))
            # one batch per (framework, cluster list): a batch is packed against one snapshot and one profile
            # grouped by cluster-list CONTENT: the reference lists clusters afresh on every reconcile
            # (scheduler.go:334), so equal lists arrive as distinct objects; fingerprinted once per list
            # object of the window (the items keep those objects alive)
            groups: Dict[tuple, list] = {}
            fps: Dict[int, bytes] = {}
            for it in items:
                fwk, _, clusters, _ = it
                fp = fps.get(id(clusters))
                if fp is None:
                    fp = fps[id(clusters)] = T.clusters_fingerprint(clusters)
                groups.setdefault((bytes(fwk.to_c()), fp), []).append(it)
            for members in groups.values():
                fwk, clusters = members[0][0], members[0][2]
                live = [m for m in members if m[3].set_running_or_notify_cancel()]
                if not live:
                    continue
                try:
                    res = self.scheduler.schedule(fwk, [m[1] for m in live], clusters)
                except BaseException as e:  # a failed batch fails each of its calls, the dispatcher keeps going
                    for m in live:
                        m[3].set_exception(e)
                    continue
                for m, r in zip(live, res):
                    m[3].set_result(r)
        # drain whatever raced with close()
        while True:
            try:
                it = self._q.get_nowait()
            except queue.Empty:
                break
            if it is not None and it[3].set_running_or_notify_cancel():
                it[3].set_exception(RuntimeError("CoalescingScheduler closed"))

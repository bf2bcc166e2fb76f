"""Multi-GPU layout of the hot path: units sharded over ranks, snapshot replicated.

The reference schedules every SchedulingUnit independently against the same
cluster list (generic_scheduler.go:92-150 reads no other unit), so a batch
shards by unit with no data-path exchange: each rank owns a contiguous slice
of units and one replica of the packed cluster snapshot. The only collective
is the snapshot broadcast when the cluster list changes (rank 0 packs, every
rank receives the blob — RCCL over xGMI on the GPU, gloo in the CPU tests)
and, for callers that want one result set, a gather of per-unit rows.
"""

from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import numpy as np

from .pack import SnapshotHeader


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of n units for `rank` (sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def blob_fingerprint(blob: np.ndarray) -> int:
    """Snapshot fingerprint stored in a packed snapshot blob's header."""
    return int(SnapshotHeader.from_buffer_copy(bytes(blob[:ctypes.sizeof(SnapshotHeader)])).fingerprint)


def broadcast_blob(blob: Optional[np.ndarray], dist, device="cpu", src: int = 0):
    """Broadcast a packed blob (uint8) from `src` to every rank; returns a torch uint8 tensor on `device`.

    Non-source ranks pass blob=None. Two collectives: the length, then the bytes.
    """
    import torch

    rank = dist.get_rank()
    n = torch.tensor([0 if blob is None else int(blob.nbytes)], dtype=torch.int64, device=device)
    dist.broadcast(n, src=src)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    if rank == src:
        buf.copy_(torch.from_numpy(np.ascontiguousarray(blob).view(np.uint8)))
    dist.broadcast(buf, src=src)
    return buf


def check_snapshot(blob: np.ndarray, fingerprint: int):
    """Fail loudly if a received snapshot is not the one this rank's batches were packed against."""
    got = blob_fingerprint(blob)
    if got != fingerprint:
        raise RuntimeError(f"snapshot fingerprint mismatch: received {got:#x}, packed against {fingerprint:#x}")


def rows_of(res, lo: int = 0, hi: Optional[int] = None) -> List[tuple]:
    """Per-unit (status, flags, pairs) rows of a BatchResult, in unit order."""
    hi = len(res.status) if hi is None else hi
    out = []
    for w in range(lo, hi):
        st, pairs = res.row(w)
        out.append((st, int(res.flags[w]), pairs))
    return out


def gather_rows(rows: List[tuple], dist, dst: int = 0) -> Optional[List[tuple]]:
    """Concatenate every rank's rows (rank order = unit order under shard_range) on `dst`."""
    parts = [None] * dist.get_world_size() if dist.get_rank() == dst else None
    dist.gather_object(rows, parts, dst=dst)
    if parts is None:
        return None
    return [r for p in parts for r in p]

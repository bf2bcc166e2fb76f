"""The device's MaxCluster selection = first-k SET of Go 1.19 sort.Slice.

The HIP kernel does not sort: it finds the k-th largest score by a radix
select and, only when the cut falls inside a run of equal scores, replays
pdqsort restricted to the sub-ranges that straddle position k (a range that
lies wholly before or after k cannot change which elements end in [0, k),
because pdqsort only permutes within [a, b) after a partition). This test
restates that restricted replay in Python (``pdq_select``) and checks it
against the full GoSort on tie-heavy inputs, including every pdqsort branch
(insertion sort, partial insertion sort, partitionEqual, breakPatterns,
reverse, heapsort fallback).
"""

import numpy as np
import pytest

from oracle.gosem import GoSort, XorShiftVariant, go_sort_slice


def pdq_select(scores, k, triple=XorShiftVariant.GO119, stats=None):
    """Restricted replay: returns the set of indices in positions [0, k)."""
    v = list(range(len(scores)))
    n = len(v)

    def less(i, j):
        return scores[v[i]] > scores[v[j]]

    def swap(i, j):
        v[i], v[j] = v[j], v[i]

    g = GoSort(less, swap, triple)
    if k <= 0:
        return set()
    if k >= n:
        return set(v)
    a, b = 0, n
    limit = n.bit_length()
    was_balanced = was_partitioned = True
    while True:
        if not (a < k < b):
            break
        length = b - a
        if length <= 12:
            g.insertion_sort(a, b)
            break
        if limit == 0:
            g.heap_sort(a, b)
            if stats is not None:
                stats["heap"] = stats.get("heap", 0) + 1
            break
        if not was_balanced:
            g.break_patterns(a, b)
            limit -= 1
            if stats is not None:
                stats["break"] = stats.get("break", 0) + 1
        pivot, hint = g.choose_pivot(a, b)
        if hint == g.DECREASING:
            g.reverse_range(a, b)
            pivot = (b - 1) - (pivot - a)
            hint = g.INCREASING
        if was_balanced and was_partitioned and hint == g.INCREASING:
            if g.partial_insertion_sort(a, b):
                break
        if a > 0 and not less(a - 1, pivot):
            a = g.partition_equal(a, b, pivot)
            if stats is not None:
                stats["eq"] = stats.get("eq", 0) + 1
            continue
        mid, already = g.partition(a, b, pivot)
        was_partitioned = already
        left, right = mid - a, b - mid
        thr = length // 8
        if left < right:
            if k < mid:  # recursion into the smaller (left) side: fresh state
                b = mid
                was_balanced = was_partitioned = True
            elif k > mid + 1:
                was_balanced = left >= thr
                a = mid + 1
            else:
                break
        else:
            if k > mid + 1:  # recursion into the smaller (right) side
                a = mid + 1
                was_balanced = was_partitioned = True
            elif k < mid:
                was_balanced = right >= thr
                b = mid
            else:
                break
    return set(v[:k])


def full_first_k(scores, k, triple=XorShiftVariant.GO119):
    items = [[i, s] for i, s in enumerate(scores)]
    go_sort_slice(items, lambda x, y: x[1] > y[1], triple)
    return {i for i, _ in items[:max(0, min(k, len(items)))]}


@pytest.mark.parametrize("triple", [XorShiftVariant.GO119, XorShiftVariant.GO121])
def test_pdq_select_equals_full_sort(triple):
    rng = np.random.default_rng(1234)
    stats = {}
    for it in range(3000):
        n = int(rng.integers(1, 400))
        kind = it % 5
        if kind == 0:
            s = rng.integers(0, 4, n)
        elif kind == 1:
            s = rng.integers(0, 101, n)
        elif kind == 2:  # sorted / reversed runs trigger partialInsertionSort / reverse
            s = np.sort(rng.integers(0, 30, n))
            if rng.random() < 0.5:
                s = s[::-1]
            s = s.copy()
            if n > 3:
                s[rng.integers(0, n)] = rng.integers(0, 30)
        elif kind == 3:  # organ pipe / sawtooth: unbalanced partitions, breakPatterns, heapsort
            s = np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]]) % int(rng.integers(2, 50))
        else:
            s = np.full(n, 7)
            s[rng.integers(0, n, max(1, n // 10))] = rng.integers(0, 10, max(1, n // 10))
        s = [int(x) for x in s]
        k = int(rng.integers(0, n + 1))
        assert pdq_select(s, k, triple, stats) == full_first_k(s, k, triple), (s, k)
    assert stats.get("eq", 0) > 0 and stats.get("break", 0) > 0

"""``sort.Slice`` of Go 1.19 (``pdqsort_func``, src/sort/zsortfunc.go) for host-side lists.

The scheduling-trigger hash sorts taints and API resources with comparators
that are not strict weak orders (``schedulingtriggers.go:215-227`` compares
values where it means effects; ``:241-257`` returns ``Kind != Kind``), so the
order it hashes is whatever Go's pattern-defeating quicksort makes of them.
This module replays that algorithm step for step on a Python list; the GPU
selection kernels replay the same algorithm on score arrays (kad_select.h).
"""

from __future__ import annotations

from typing import Callable, List

_M64 = (1 << 64) - 1


def sort_slice(x: List, less: Callable[[object, object], bool], xorshift=(13, 17, 5)) -> None:
    """In-place ``sort.Slice(x, func(i, j int) bool { return less(x[i], x[j]) })``."""
    n = len(x)

    def lt(i, j):
        return less(x[i], x[j])

    def sw(i, j):
        x[i], x[j] = x[j], x[i]

    def insertion(a, b):
        for i in range(a + 1, b):
            j = i
            while j > a and lt(j, j - 1):
                sw(j, j - 1)
                j -= 1

    def sift(lo, hi, first):
        root = lo
        while True:
            c = 2 * root + 1
            if c >= hi:
                return
            if c + 1 < hi and lt(first + c, first + c + 1):
                c += 1
            if not lt(first + root, first + c):
                return
            sw(first + root, first + c)
            root = c

    def heap(a, b):
        hi = b - a
        for i in range((hi - 1) // 2, -1, -1):
            sift(i, hi, a)
        for i in range(hi - 1, -1, -1):
            sw(a, a + i)
            sift(0, i, a)

    def median(p, q, r, cnt):
        # order2 three times, counting swaps
        if lt(q, p):
            cnt[0] += 1
            p, q = q, p
        if lt(r, q):
            cnt[0] += 1
            q, r = r, q
        if lt(q, p):
            cnt[0] += 1
            p, q = q, p
        return q

    def pivot_of(a, b):
        ln = b - a
        cnt = [0]
        q = ln // 4
        i, j, k = a + q, a + 2 * q, a + 3 * q
        if ln >= 8:
            if ln >= 50:
                i = median(i - 1, i, i + 1, cnt)
                j = median(j - 1, j, j + 1, cnt)
                k = median(k - 1, k, k + 1, cnt)
            j = median(i, j, k, cnt)
        hint = 1 if cnt[0] == 0 else (2 if cnt[0] == 12 else 0)  # increasing / decreasing / unknown
        return j, hint

    def partial_insertion(a, b):
        i = a + 1
        for _ in range(5):
            while i < b and not lt(i, i - 1):
                i += 1
            if i == b:
                return True
            if b - a < 50:
                return False
            sw(i, i - 1)
            if i - a >= 2:
                j = i - 1
                while j >= 1 and lt(j, j - 1):  # lower bound 1, as in Go
                    sw(j, j - 1)
                    j -= 1
            if b - i >= 2:
                j = i + 1
                while j < b and lt(j, j - 1):
                    sw(j, j - 1)
                    j += 1
        return False

    def break_patterns(a, b):
        ln = b - a
        if ln < 8:
            return
        r = ln
        s1, s2, s3 = xorshift
        mask = (1 << ln.bit_length()) - 1
        idx = a + (ln // 4) * 2 - 1
        for t in range(3):
            r ^= (r << s1) & _M64
            r ^= r >> s2
            r ^= (r << s3) & _M64
            other = r & mask
            if other >= ln:
                other -= ln
            sw(idx - 1 + t, a + other)

    def partition(a, b, p):
        sw(a, p)
        i, j = a + 1, b - 1
        while i <= j and lt(i, a):
            i += 1
        while i <= j and not lt(j, a):
            j -= 1
        if i > j:
            sw(j, a)
            return j, True
        sw(i, j)
        i, j = i + 1, j - 1
        while True:
            while i <= j and lt(i, a):
                i += 1
            while i <= j and not lt(j, a):
                j -= 1
            if i > j:
                break
            sw(i, j)
            i, j = i + 1, j - 1
        sw(j, a)
        return j, False

    def partition_equal(a, b, p):
        sw(a, p)
        i, j = a + 1, b - 1
        while True:
            while i <= j and not lt(a, i):
                i += 1
            while i <= j and lt(a, j):
                j -= 1
            if i > j:
                return i
            sw(i, j)
            i, j = i + 1, j - 1

    def pdq(a, b, limit):
        balanced = partitioned = True
        while True:
            ln = b - a
            if ln <= 12:
                insertion(a, b)
                return
            if limit == 0:
                heap(a, b)
                return
            if not balanced:
                break_patterns(a, b)
                limit -= 1
            p, hint = pivot_of(a, b)
            if hint == 2:
                i, j = a, b - 1
                while i < j:
                    sw(i, j)
                    i, j = i + 1, j - 1
                p = (b - 1) - (p - a)
                hint = 1
            if balanced and partitioned and hint == 1 and partial_insertion(a, b):
                return
            if a > 0 and not lt(a - 1, p):
                a = partition_equal(a, b, p)
                continue
            mid, partitioned = partition(a, b, p)
            left, right = mid - a, b - mid
            if left < right:
                balanced = left >= ln // 8
                pdq(a, mid, limit)
                a = mid + 1
            else:
                balanced = right >= ln // 8
                pdq(mid + 1, b, limit)
                b = mid

    pdq(0, n, n.bit_length())

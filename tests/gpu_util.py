"""Helpers shared by the GPU parity tests."""
import os

import numpy as np

from kubeadmiral_amd import pack
from oracle import ref


def c_oracle(snap, batch, fwk):
    return ref.schedule(snap, batch, fwk, n_threads=min(16, os.cpu_count() or 1))


def assert_same(got, want, what=""):
    eq = got.equal_rows(want) & (got.flags == want.flags)
    bad = np.nonzero(~eq)[0]
    if len(bad):
        w = int(bad[0])
        raise AssertionError(f"{what}: {len(bad)} rows differ; first w={w}: gpu={got.row(w)} flags={got.flags[w]} "
                             f"oracle={want.row(w)} flags={want.flags[w]}")

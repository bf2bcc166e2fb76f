"""Debug: the register planner vs the LDS-workspace planner on small rows (prints both)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from kubeadmiral_amd import k8s, runtime  # noqa: E402

ctx = runtime.Context(0)
rows = []
for total in (1, 2, 3, 5):
    for avoid in (False, True):
        for keep in (False, True):
            rows.append({"elems": [{"hash": k8s.fnv1_32(n.encode()), "weight": 1, "min": 0, "max": None, "cap": None,
                                    "current": 0} for n in "AB"], "total": total, "avoid": avoid, "keep": keep})
def row(ws, total, avoid=True, cur=None):
    return {"elems": [{"hash": k8s.fnv1_32(chr(65 + i).encode()), "weight": w, "min": 0, "max": None, "cap": None,
                       "current": (cur or [0] * len(ws))[i]} for i, w in enumerate(ws)],
            "total": total, "avoid": avoid, "keep": False}
rows += [row([1, 0], 2), row([1], 1), row([1], 5), row([3, 1, 1], 1), row([3, 1, 1], 4), row([1, 1], 1, cur=[0, 0]),
         row([1, 1], 2, cur=[1, 0]), row([1, 1], 1, cur=[1, 1]), row([1, 1, 1, 1], 3, cur=[0, 0, 0, 0])]
rng = np.random.default_rng(1)
for _ in range(6):
    K = int(rng.integers(1, 8))
    rows.append({"elems": [{"hash": int(rng.integers(0, 1 << 32)), "weight": int(rng.integers(0, 5)), "min": 0,
                            "max": None, "cap": None, "current": 0} for _ in range(K)],
                 "total": int(rng.integers(1, 20)), "avoid": False, "keep": False})
os.environ.pop("KAD_PLAN_FORCE_WS", None)
a = ctx.plan_rows(rows)
os.environ["KAD_PLAN_FORCE_WS"] = "1"
b = ctx.plan_rows(rows)
for r, x, y in zip(rows, a, b):
    print(r["total"], r["avoid"], r["keep"], [e["weight"] for e in r["elems"]], "lanes", x[0], "ws", y[0],
          "" if x == y else "DIFF")

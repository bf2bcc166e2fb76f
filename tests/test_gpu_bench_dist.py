"""bench.py's multi-GPU path on the one-GPU box: `--gpus 2` starts two ranks itself (torch.distributed.run),
`--share-gpu` puts both on device 0 and `--backend gloo` stands in for RCCL (two ranks on one GPU cannot use
RCCL). Checks the line the driver parses: world size, whole-job value, the timed placement all-gather, and
that the gathered placements of every rank equal a single-rank run of its shard."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_share_one_gpu():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mode", "ranks", "--share-gpu", "--backend", "gloo",
           "--config", "c2", "--units", "20000", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-extra"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    r0 = "\n".join(ln for ln in p.stderr.splitlines() if ln.startswith("[rank0]"))
    assert p.returncode == 0, (r0 or p.stderr)[-4000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["rccl_world_size"] == 2
    assert line["config"]["units_total"] == 20000 and line["config"]["units_per_gpu"] == 10000
    assert line["value"] > 0 and line["scaling"] == "strong"
    assert line["allgather"] is not None and line["allgather"]["ms"] > 0
    # every gathered field of both ranks was compared with a single-rank run of the same shard blob
    assert line["allgather"]["verified"] and "2 ranks" in line["allgather"]["verified"]


def _group_line(extra_env=None, launcher=False):
    args = ["--gpus", "4", "--group-devices", "0,0,0,0", "--config", "c3", "--units", "200000", "--steps", "3",
            "--warmup", "1"]
    if launcher:  # the driver's SCALE launch: one rank per GPU, rank 0 drives the group
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
               "--master-addr=127.0.0.1", "--master-port=29517", os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **(extra_env or {}))
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("launcher", [False, True])
def test_bench_group_mode_four_members_on_one_gpu(launcher):
    """--gpus 4 in the default group mode (kad_group over 4 members, here all on device 0), alone and under
    torch.distributed.run with 4 ranks (rank 0 drives the group, the others join the barriers): the whole
    batch's rows equal the C oracle's (verify_rows), the line names the group."""
    line = _group_line(launcher=launcher)
    assert line["n_gpus"] == 4 and line["config"]["units_total"] == 200000
    assert line["config"]["units_per_gpu"] == 50000 and "kad_group" in line["config"]["parallelism"]
    assert line["value"] > 0 and line["scaling"] == "strong"
    assert line["parity"]["mismatches"] == 0 and line["parity"]["units_checked"] > 0
    assert line["group"]["devices"] == [0, 0, 0, 0]

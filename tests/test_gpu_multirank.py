"""bench.py's multi-rank launch rehearsed on the one GPU of the box (VERDICT r3 "next" 7).

The driver's SCALE run launches ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``, one
process per GPU.  Here both ranks of a 2-process launch are put on device 0 (SO100_BENCH_DEVICE, a test hook),
and the run is checked against a single-process run of the same workload: the two shards' final states must
equal the ``env_offset`` slices of the one-process state bit for bit, and rank 0 alone prints one JSON line
with ``n_gpus: 2``."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(cmd, env, timeout=240):
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


def test_two_rank_launch_matches_one_process(tmp_path):
    total, steps = 2048, 12
    common = ["--total-envs", str(total), "--steps", str(steps), "--warmup", "3", "--no-cpu-baseline",
              "--contact-steps", "2"]
    env = dict(os.environ, SO100_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    lines2 = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                   "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                   *common, "--dump-state", str(tmp_path / "two")], env)
    lines1 = _run([sys.executable, "bench.py", "--gpus", "1", *common, "--dump-state", str(tmp_path / "one")],
                  dict(os.environ, OMP_NUM_THREADS="2"))
    assert len(lines2) == 1 and len(lines1) == 1
    l2 = lines2[0]
    assert l2["n_gpus"] == 2 and l2["config"]["envs_total"] == total and l2["config"]["envs_per_gpu"] == total // 2
    assert l2["value"] > 0 and l2["scaling"] == "strong" and l2["cpu_baseline"] is None
    one = np.load(tmp_path / "one" / "state_rank0.npz")
    for r in range(2):
        part = np.load(tmp_path / "two" / f"state_rank{r}.npz")
        o, c = int(part["offset"]), int(part["count"])
        assert (o, c) == (r * total // 2, total // 2)
        for k in ("qpos", "qvel", "obs", "reward", "episode"):
            np.testing.assert_array_equal(part[k], one[k][o:o + c], err_msg=f"rank {r} {k}")

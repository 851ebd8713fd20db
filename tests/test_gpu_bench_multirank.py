"""bench.py's N > 1 path under test. The driver launches
`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` on an
8-GPU node at round end; here two gloo ranks share cuda:0
(VMP_DIST_BACKEND=gloo, bench.py:111-117) and run every leg at reduced
sizes: NCCL-free init, barriers, max-over-ranks timing, the replica
all-reduce / all-gather, the parity leg on rank 0, and the
data-parallel PPO legs. The replica counters must equal ONE rank holding
all envs over the same seeds (4 x global index) and the same phase groups
(bench.fast_forward assigns them by global index)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_LOCAL = 1024
SMALL = ["--steps", "5", "--warmup", "2", "--no-cpu", "--ff-steps", "300",
         "--phase-delta", "10", "--rollout-k", "20", "--ext-steps", "5"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(cmd, timeout):
    env = dict(os.environ, VMP_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stdout[-3000:]
    return json.loads(lines[-1])


def test_bench_two_ranks_gloo_every_leg():
    two = _bench([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                  "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                  str(_free_port()), "bench.py", "--gpus", "2", "--envs", str(N_LOCAL)] + SMALL
                 + ["--period-steps", "20", "--period-ff", "100", "--nominal-steps", "5",
                    "--ppo-envs", "128", "--ppo-eval-envs", "256", "--ppo-updates", "1",
                    "--stress-ff", "100", "--stress-steps", "2"], timeout=420)
    assert two["n_gpus"] == 2 and two["config"]["global_envs"] == 2 * N_LOCAL
    assert two["value"] > 0 and two["ms_per_step"] > 0
    rep = two["replicas"]
    assert rep["returns_gathered"] == 2 * N_LOCAL
    assert "RCCL" in rep["collectives"]  # the N > 1 wording (gloo stands in for it here)
    par = two["parity"]
    assert par["counters_equal"] and par["reward_max_abs_err"] == 0.0
    for leg in ("ppo_train", "ppo_train_bf16", "ppo_eval", "stress_p1000_v10000",
                "stress_p1000_v10000_2048envs", "period", "nominal_load", "external_actions"):
        assert isinstance(two[leg], dict) and "error" not in two[leg], (leg, two[leg])
    for leg in ("ppo_train", "ppo_train_bf16"):
        assert two[leg]["global_envs"] == 2 * 128 and "x2" in two[leg]["parallelism"]
    # one rank, all 2 048 envs, the same seeds and phase groups: same counter sums
    one = _bench([sys.executable, "bench.py", "--gpus", "1", "--envs", str(2 * N_LOCAL)] + SMALL
                 + ["--period-steps", "0", "--nominal-steps", "0", "--no-ppo"], timeout=300)
    assert one["n_gpus"] == 1 and one["replicas"]["returns_gathered"] == 2 * N_LOCAL
    assert one["replicas"]["counters_sum"] == rep["counters_sum"]
    assert abs(one["replicas"]["return_mean"] - rep["return_mean"]) <= 1e-12 * max(
        1.0, abs(rep["return_mean"]))

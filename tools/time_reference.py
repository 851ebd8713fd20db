"""Time the UNMODIFIED reference `VmEnv.step` (vmenv/envs/env.py:66-103) in this
container (container only: the reference never ships to the GPU box). Writes
tests/golden/ref_cpu_timing.json, which bench.py carries beside its
cpu_baseline as the reference's own CPU step rate, labelled as measured on a
different box.

Run:  python tools/time_reference.py [--procs 8]
Per config (training mode, info = {} as in env.py:168; FirstFit actions from
the reference's own FirstFitAgent, computed outside the timed calls):
  single_core  steps/s of env.step alone on one process (OMP_NUM_THREADS=1)
  procs_8      aggregate step-only steps/s of 8 processes x 1 env (the exp.py:1
               fan-out pattern), every process timing its own steps
"""
import json
import os
import platform
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "ref_cpu_timing.json")

CONFIGS = {
    # BASELINE config 1 shape (config/10.yml)
    "10yml": dict(pms=10, vms=30, arrival_rate=0.0182, service_length=1000,
                  training_steps=10000, eval_steps=100000, seed=1, reward_function="wr",
                  sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True),
    # bench.py's headline workload (config/100.yml with vms = 1000)
    "p100v1000": dict(pms=100, vms=1000, arrival_rate=1.8182, service_length=1000,
                      training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
                      sequence="uniform", cap_target_util=True, beta=0.5,
                      allow_null_action=True),
}
WARM, TIMED = 300, 300

if os.environ.get("VMP_REF_CHILD") != "1":
    import multiprocessing  # noqa: F401

    env = dict(os.environ)
    env.update(VMP_REF_CHILD="1", PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg",
               OMP_NUM_THREADS="1", PYTHONPATH=os.path.join(HERE, "oracle_stubs") + ":" + REF)
    sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                             env=env, cwd=REF))

import oracle_boot  # noqa: E402,F401  (tensorboard stub)
import numpy as np  # noqa: E402
import gymnasium as gym  # noqa: E402
import vmenv  # noqa: E402,F401
from vmenv.envs.config import Config  # noqa: E402
from src.agents.firstfit import FirstFitAgent  # noqa: E402


def run_one(args):
    """One env: WARM untimed steps, then TIMED steps with only env.step timed."""
    name, seed = args
    c = dict(CONFIGS[name], seed=seed)
    e = gym.make("VmEnv-v1", config=Config(**c))
    e.reset(seed=seed)
    ag = FirstFitAgent(e)
    obs = e._get_obs()
    for _ in range(WARM):
        obs, *_ = e.step(np.asarray(ag.act(obs)).astype(np.int64))
    spent = 0.0
    for _ in range(TIMED):
        a = np.asarray(ag.act(obs)).astype(np.int64)
        t0 = time.perf_counter()
        obs, *_ = e.step(a)
        spent += time.perf_counter() - t0
    return TIMED / spent


def main():
    import multiprocessing as mp
    procs = 8
    if "--procs" in sys.argv:
        procs = int(sys.argv[sys.argv.index("--procs") + 1])
    res = {}
    for name in CONFIGS:
        single = run_one((name, CONFIGS[name]["seed"]))
        with mp.get_context("fork").Pool(procs) as pool:
            per = pool.map(run_one, [(name, CONFIGS[name]["seed"] + 4 * i) for i in range(procs)])
        res[name] = {"config": CONFIGS[name],
                     "single_core_steps_per_s": single,
                     f"procs_{procs}_aggregate_steps_per_s": float(np.sum(per)),
                     "per_process_steps_per_s": [float(x) for x in per]}
        print(name, res[name]["single_core_steps_per_s"], np.sum(per), flush=True)
    out = {"what": "unmodified reference VmEnv.step (vmenv/envs/env.py:66-103), training mode, "
                   "FirstFit actions (src/agents/firstfit.py:21-38) computed outside the timed "
                   "calls; steps after a warm-up of %d steps" % WARM,
           "timed_steps_per_env": TIMED,
           "box": {"cpu": platform.processor() or platform.machine(),
                   "model": _cpu_model(), "logical_cpus": os.cpu_count(),
                   "numpy": np.__version__, "python": platform.python_version()},
           "note": "measured in the build container, NOT on the GPU box (the reference "
                   "never ships there)",
           "results": res}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()

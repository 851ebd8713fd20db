"""Device Record metrics (vmp_record_*, record.py:34-134) on the MI355X:
every published firstfit/bestfit row of data/exp_suspension/data.csv (100k-step
evals of config/100.yml: served, valid suspends, valid actions, mean life,
mean pending, mean/max slowdown) and the literal host restatement of
record.py (tests/record_literal.py, fed by Base.record_testing_step from
eval-mode info) on a trajectory with random suspensions and placements."""
import csv
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _rows():
    with open(os.path.join(GOLDEN, "exp_suspension_data.csv")) as f:
        return [r for r in csv.reader(f) if r[0] in ("firstfit", "bestfit")]


@pytest.mark.parametrize("half", [0, 1])
def test_published_exp_suspension_rows_with_record_metrics(half):
    """exp_suspension.py:12-58 for every heuristic row (half of them per case),
    each a 100k-step eval recorded on the device (rollout with the recorder on,
    one launch per step)."""
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    rows, envs, streams = _rows()[half::2], [], []
    for r in rows:
        agent, load, L = r[0], float(r[1]), int(r[2])
        cfg = Config(pms=100, vms=300, service_length=L, training_steps=10000, eval_steps=100000,
                     seed=0, reward_function="wr", sequence="uniform", cap_target_util=True,
                     beta=0.5, allow_null_action=True,
                     arrival_rate=float(np.round(100 / 0.55 / L * load, 3)))
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            env = BatchedVmEnv(cfg, 1, seeds=[0], device="cuda:0")
            env.eval(True)
            env.reset(torch.tensor([0]))
            env.record(True)
        envs.append(env)
        streams.append(s)
    # the 16 single-env evals run side by side, one stream each
    for _ in range(50):
        for r, env, s in zip(rows, envs, streams):
            with torch.cuda.stream(s):
                env.rollout(r[0], 2000)
    torch.cuda.synchronize()
    bad = []
    for r, env, s in zip(rows, envs, streams):
        with torch.cuda.stream(s):
            sm = env.record_summary()[0]
        got = [sm["total served VMs"], sm["total suspend actions"],
               sm["total suspend actions"] + sm["total place actions"], "%d" % sm["_mean_life"],
               "%.3f" % sm["_mean_pending"], "%.3f" % sm["_mean_slowdown"],
               "%.3f" % sm["_max_slowdown"]]
        want = [int(r[3]), int(r[4]), int(r[5]), r[6].strip(), r[7].strip(), r[8].strip(),
                r[9].strip()]
        if got != want:
            bad.append((r[:3], got, want))
        env.close()
    assert not bad, bad


def _random_actions(b, g, p_susp=0.03, p_place=0.3):
    """Perturbed actions from the current placements: random suspensions of
    running VMs and random PM targets for waiting ones (some invalid)."""
    st = b.state()["vm_placement"][0].cpu()
    V, P = st.numel(), b.P
    a = st.clone()
    u = torch.rand(V, generator=g)
    tgt = torch.randint(0, P, (V,), generator=g)
    running, waiting = st < P, st == P
    a[running & (u < p_susp)] = P
    a[waiting & (u < p_place)] = tgt[waiting & (u < p_place)]
    return a.numpy()


@pytest.mark.parametrize("seed", [3, 11])
def test_device_record_matches_literal_record(seed):
    from vmp.agents import Base
    from vmp.config import Config
    from vmp.env import VmEnv
    cfg = Config(pms=10, vms=30, arrival_rate=0.6, service_length=25, training_steps=1000,
                 eval_steps=500, seed=seed, reward_function="kl", allow_null_action=True)
    env = VmEnv(cfg, device="cuda:0")
    env.eval(True)
    obs, _ = env.reset(seed=seed)
    env._b.record(True)
    base = Base("literal", env, None)
    g = torch.Generator().manual_seed(seed)
    done = False
    while not done:
        a = _random_actions(env._b, g)
        obs, reward, done, _, info = env.step(a)
        base.record_testing_step(reward, info)
    from tests import record_literal
    lit = record_literal.summary(vars(base.record), cfg.pms)
    dev = env._b.record_summary()[0]
    assert lit["total suspend actions"] > 0
    for k, v in lit.items():
        if isinstance(v, (int, np.integer)):
            assert dev[k] == v, (k, dev[k], v)
        else:
            assert abs(float(dev[k]) - float(v)) <= 1e-3 + 1e-9 * abs(float(v)), (k, dev[k], v)
    for k in ("average VM life", "average pending", "median pending", "max pending",
              "average slowdown", "median slowdown", "max slowdown", "drop rate", "rank mean"):
        assert dev[k] == lit[k], (k, dev[k], lit[k])
    env.close()


def test_base_test_summary_is_the_device_summary(tmp_path):
    """Base.test (base.py:63-118) returns a Record whose summary comes from the
    device recorder; it equals the host restatement on the recorded traces,
    and a saved record re-imports with that summary (record.py:136-168)."""
    import json
    from tests import record_literal
    from vmp.agents import FirstFitAgent
    from vmp.config import Config
    from vmp.env import VmEnv
    from vmp.record import Record
    cfg = Config(pms=10, vms=30, arrival_rate=0.9, service_length=40, training_steps=1000,
                 eval_steps=400, seed=7, reward_function="ut", allow_null_action=True)
    env = VmEnv(cfg, device="cuda:0")
    rec = FirstFitAgent(env).test(output=str(tmp_path / "r.json"))
    got, lit = rec.get_summary(), record_literal.summary(vars(rec), cfg.pms)
    assert list(got) == list(lit)
    for k, v in lit.items():
        assert abs(float(got[k]) - float(v)) <= 1e-3 + 1e-9 * abs(float(v)), (k, got[k], v)
    back = Record.import_record("FirstFitAgent", json.load(open(tmp_path / "r.json")))
    assert back.get_summary() == json.loads(json.dumps(got, default=float))
    env.close()

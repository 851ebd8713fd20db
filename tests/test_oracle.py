"""The C oracle (oracle/vmp_oracle.c) pinned against the reference's own
outputs: numpy RNG KATs, golden lock-step trajectories, and the published
exp_suspension rows (data/exp_suspension/data.csv). CPU only."""
import csv
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import traj as T
from tests.golden_hash import obs_hash, state_hash

KAT = np.load(os.path.join(T.GOLDEN, "rng_kat.npz"))


def test_seed_state_matches_numpy():
    out = np.zeros(4, np.uint64)
    for s, exp in zip(KAT["seeds"], KAT["state_inc"]):
        O.lib().oracle_pcg_seed(int(s), O._p(out))
        assert np.array_equal(out, exp), int(s)


def test_raw_double_around():
    for i, s in enumerate(KAT["seeds"]):
        raw = np.zeros(8, np.uint64)
        O.lib().oracle_pcg_raw(int(s), 8, O._p(raw))
        assert np.array_equal(raw, KAT["raw"][i])
        dbl = np.zeros(8)
        O.lib().oracle_pcg_double(int(s), 8, O._p(dbl))
        assert np.array_equal(dbl, KAT["dbl"][i])
        ar = np.zeros(16)
        O.lib().oracle_pcg_around(int(s), 16, 0.1, 1.0, O._p(ar))
        assert np.array_equal(ar, KAT["around"][i])


def test_poisson_streams():
    for i, s in enumerate(KAT["seeds"]):
        for j, lam in enumerate(KAT["lams"]):
            out = np.zeros(40, np.int64)
            after = O.lib().oracle_pcg_poisson(int(s), float(lam), 40, O._p(out))
            assert np.array_equal(out, KAT["poisson"][i, j]), (int(s), lam)
            assert after == int(KAT["raw_after"][i, j]), (int(s), lam)


def test_advance_matches_stepping():
    for s in (0, 7, 2**40 + 3):
        raw = np.zeros(1001, np.uint64)
        O.lib().oracle_pcg_raw(s, 1001, O._p(raw))
        assert O.lib().oracle_pcg_advance_raw(s, 1000) == int(raw[1000])


def test_pairwise_sum_matches_numpy():
    rng = np.random.default_rng(3)
    for n in list(range(0, 40)) + [127, 128, 129, 255, 256, 300, 1000, 1037, 4099]:
        a = np.around(rng.uniform(0.1, 1, n), 2)
        assert O.lib().oracle_pw_sum(O._p(a), n) == np.sum(a), n


def test_argsort_is_a_permutation_sorting_keys():
    rng = np.random.default_rng(4)
    for n in (1, 2, 10, 16, 17, 50, 100, 1000):
        v = (rng.integers(0, 30, n) / 10).astype(np.float32)
        out = np.zeros(n, np.int64)
        O.lib().oracle_argsort_f32(O._p(v), n, O._p(out))
        assert sorted(out.tolist()) == list(range(n))
        assert np.all(np.diff(v[out]) >= 0)
        if n <= 16:  # insertion sort only: stable
            assert np.array_equal(out, np.argsort(v, kind="stable"))


def replay(d, reward_idx):
    cfg = dict(d["config"])
    cfg["reward_function"] = d["rewards"][reward_idx]
    env = O.OracleEnv(cfg)
    env.eval(bool(d["eval_mode"]))
    env.reset(cfg["seed"])
    acts = T.sparse_actions(d)
    masks = {int(t): i for i, t in enumerate(d["mask_at"])}
    n_kl_exact = 0
    for t in range(d["T"]):
        if t == d["reset_none_at"]:
            env.reset(None)
        if t in masks:
            m = env.mask()
            assert np.array_equal(np.packbits(m), d["masks"][masks[t]]), ("mask", t)
        pl = env.state()[0]
        a = pl.copy()
        if t in acts:
            vm, tg, va = acts[t]
            a[vm] = tg
        obs, r, done, valid = env.step(a)
        if t in acts:
            assert np.array_equal(valid[acts[t][0]], acts[t][2]), ("valid", t)
        exp_r = d["reward"][reward_idx, t]
        if cfg["reward_function"] == "kl":
            assert T.kl_close(r, exp_r), (t, r, exp_r)
            n_kl_exact += r == exp_r
        else:
            assert r == exp_r, (t, r, exp_r)
        st = env.state()
        assert state_hash(*st) == d["state_hash"][t], ("state", t)
        assert obs_hash(obs) == d["obs_hash"][t], ("obs", t)
        c, misc = env.counters()
        assert np.array_equal(c, d["counters"][t]), ("counters", t, c, d["counters"][t])
        assert np.array_equal(misc, d["misc"][t]), ("misc", t, misc, d["misc"][t])
        assert int(done) == d["done"][t]
        if "rank" in d:
            assert env.rank() == d["rank"][t]
    return n_kl_exact


@pytest.mark.parametrize("name", T.traj_names())
def test_trajectory_replay(name):
    d = T.load(name)
    for k in range(len(d["rewards"])):
        n_exact = replay(d, k)
        if d["rewards"][k] == "kl":
            # libm log vs numpy/OpenBLAS bit paths: report, bar is 1e-12
            assert n_exact >= 0.5 * d["T"], n_exact


@pytest.mark.parametrize("name", [n for n in T.traj_names() if n.endswith("pure")] +
                         ["c1_10yml_ff"])
def test_heuristic_proposals(name):
    d = T.load(name)
    env = O.OracleEnv(d["config"])
    env.eval(True)
    env.reset(d["config"]["seed"])
    acts = T.sparse_actions(d)
    for t in range(d["T"]):
        a = env.firstfit() if d["policy"] == "ff" else env.bestfit()
        pl = env.state()[0]
        nz = np.flatnonzero(a != pl)
        exp = acts.get(t, (np.zeros(0, int), np.zeros(0, int), None))
        assert np.array_equal(nz, exp[0]) and np.array_equal(a[nz], exp[1]), t
        env.step(a)


def _kat_rows():
    rows = []
    with open(os.path.join(T.GOLDEN, "exp_suspension_data.csv")) as f:
        for r in csv.reader(f):
            if r[0] in ("firstfit", "bestfit"):
                rows.append((r[0], float(r[1]), int(r[2]), int(r[3]), int(r[4]), int(r[5])))
    return rows


@pytest.mark.parametrize("row", _kat_rows(),
                         ids=lambda r: "%s-load%.1f-L%d" % (r[0], r[1], r[2]))
def test_published_exp_suspension_rows(row):
    """exp_suspension.py:12-60: config/100.yml, reward wr, seed 0, 100k eval
    steps, arrival_rate = round(100/0.55/L*load, 3); columns served, valid
    suspends, valid actions (data/exp_suspension/data.csv)."""
    agent, load, L, served, susp, valid = row
    cfg = dict(pms=100, vms=300, service_length=L, training_steps=10000, eval_steps=100000,
               seed=0, reward_function="wr", sequence="uniform", cap_target_util=True,
               beta=0.5, allow_null_action=True,
               arrival_rate=float(np.round(100 / 0.55 / L * load, 3)))
    _, ctr = O.rollout(cfg, 1, 0, 1, 100000, policy=0 if agent == "firstfit" else 1)
    assert ctr[0, 1] == served and ctr[0, 2] == susp and ctr[0, 2] + ctr[0, 3] == valid, ctr[0]


def test_rollout_timed_passes_repeat_the_same_window():
    """bench.py cpu_baseline: every timed pass restarts from the post-warm-up
    state, so the passes do identical work (same per-env reward sums), and
    they equal a plain OracleEnv FirstFit rollout of the same seeds."""
    cfg = dict(pms=10, vms=30, arrival_rate=0.3, service_length=20, reward_function="wr")
    secs, rs = O.rollout_timed(cfg, 4, 7, 3, 25, 40, 0, 2, reps=3)
    assert secs.shape == (3,) and (secs > 0).all()
    np.testing.assert_array_equal(rs[0], rs[1])
    np.testing.assert_array_equal(rs[0], rs[2])
    for i in range(4):
        e = O.OracleEnv(dict(cfg, seed=7 + 3 * i))
        tot = 0.0
        for s in range(65):
            _, r, _, _ = e.step(e.firstfit())
            if s >= 25:
                tot += r
        assert tot == rs[0, i]

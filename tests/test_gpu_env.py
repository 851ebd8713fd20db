"""HIP path parity (MI355X): libvmp.so through the C ABI against the golden
reference fixtures and the C oracle. Integer state/counters must be bit-exact;
wr/ut rewards bit-exact; kl within 1e-12 relative (device log/exp vs glibc)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import traj as T
from tests.golden_hash import obs_hash, state_hash

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _cfg(d, **over):
    from vmp.config import Config
    c = dict(d)
    c.update(over)
    return Config(**c)


def _np_state(b, i=0):
    return {k: v[i].cpu().numpy() for k, v in b.state().items()}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")


@pytest.mark.parametrize("big", [False, True], ids=["wave", "block"])
@pytest.mark.parametrize("name", T.traj_names())
def test_trajectory_replay_hip(name, big, monkeypatch):
    """Every golden trajectory through the wave-per-env kernel (k_env) and the
    block-per-env kernel of large V (k_env_big, forced with VMP_BIG_KERNEL=1)."""
    from vmp.batched import BatchedVmEnv
    if big:
        monkeypatch.setenv("VMP_BIG_KERNEL", "1")
    d = T.load(name)
    envs = []
    for r in d["rewards"]:
        b = BatchedVmEnv(_cfg(d["config"], reward_function=r), 1, seeds=[d["config"]["seed"]],
                         device=DEV)
        b.eval(bool(d["eval_mode"]))
        envs.append(b)
    acts = T.sparse_actions(d)
    masks = {int(t): i for i, t in enumerate(d["mask_at"])}
    V = d["config"]["vms"]
    for t in range(d["T"]):
        if t == d["reset_none_at"]:
            for b in envs:
                b.reset(None)
        b0 = envs[0]
        if t in masks:
            m = b0.mask()[0].cpu().numpy()
            assert np.array_equal(np.packbits(m), d["masks"][masks[t]]), ("mask", t)
            bits = b0.mask_bits()[0].cpu().numpy().view(np.uint32)
            unpacked = ((bits[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(V, -1)
            assert np.array_equal(unpacked[:, :b0.A].astype(bool), m)
        pl = _np_state(b0)["vm_placement"]
        a = pl.copy()
        if t in acts:
            a[acts[t][0]] = acts[t][1]
        at = torch.tensor(a, dtype=torch.int32, device=DEV).reshape(1, V)
        for k, b in enumerate(envs):
            obs, rew, done, valid = b.step(at)
            r, exp_r = float(rew[0]), d["reward"][k, t]
            if d["rewards"][k] == "kl":
                assert T.kl_close(r, exp_r), (t, r, exp_r)
            else:
                assert r == exp_r, (d["rewards"][k], t, r, exp_r)
            if k == 0:
                v = valid[0].cpu().numpy()
                if t in acts:
                    assert np.array_equal(v[acts[t][0]], acts[t][2]), ("valid", t)
                assert int(done[0]) == d["done"][t]
                assert obs_hash(obs[0].cpu().numpy()) == d["obs_hash"][t], ("obs", t)
        st = _np_state(b0)
        h = state_hash(st["vm_placement"], st["vm_cpu"], st["vm_memory"], st["cpu"],
                       st["memory"], st["vm_remaining_runtime"])
        assert h == d["state_hash"][t], ("state", t)
        assert np.array_equal(b0.counters()[0].cpu().numpy(), d["counters"][t]), ("ctr", t)
        assert np.array_equal(b0.stats()[0].cpu().numpy(), d["misc"][t]), ("misc", t)
        if "rank" in d:
            assert int(b0.rank()[0]) == d["rank"][t]


@pytest.mark.parametrize("big", [False, True], ids=["wave", "block"])
@pytest.mark.parametrize("name", [n for n in T.traj_names() if n.endswith("pure")] +
                         ["c1_10yml_ff"])
def test_heuristic_act_hip(name, big, monkeypatch):
    """Act-only launches (vmp_heuristic_act, k_steps == 0) of both env kernels."""
    from vmp.batched import BatchedVmEnv
    if big:
        monkeypatch.setenv("VMP_BIG_KERNEL", "1")
    d = T.load(name)
    b = BatchedVmEnv(_cfg(d["config"]), 1, seeds=[d["config"]["seed"]], device=DEV)
    b.eval(True)
    acts = T.sparse_actions(d)
    for t in range(d["T"]):
        a = b.heuristic_act(d["policy"].replace("ff", "firstfit").replace("bf", "bestfit"))
        an = a[0].cpu().numpy()
        pl = _np_state(b)["vm_placement"]
        nz = np.flatnonzero(an != pl)
        exp = acts.get(t, (np.zeros(0, int), np.zeros(0, int), None))
        assert np.array_equal(nz, exp[0]) and np.array_equal(an[nz], exp[1]), t
        b.step(a)


BATCH_CFGS = [
    dict(pms=100, vms=300, arrival_rate=1.8182, service_length=150, reward_function="wr"),
    dict(pms=100, vms=300, arrival_rate=0.909, service_length=1000, reward_function="kl"),
    dict(pms=10, vms=30, arrival_rate=0.3, service_length=60, reward_function="ut"),
    dict(pms=100, vms=1000, arrival_rate=1.8182, service_length=300, reward_function="wr"),
    dict(pms=37, vms=130, arrival_rate=12.0, service_length=25, reward_function="kl",
         sequence="lowuniform"),
]


@pytest.mark.parametrize("big", [False, True], ids=["wave", "block"])
@pytest.mark.parametrize("policy", ["firstfit", "bestfit"])
@pytest.mark.parametrize("ci", range(len(BATCH_CFGS)))
def test_batched_heuristic_vs_oracle(ci, policy, big, monkeypatch):
    """N envs (seeds base + 4i, incl. > 2**32) stepped by the fused act+step kernel
    against the oracle env by env; then a fused K-step rollout continues and must
    equal the oracle's next K steps (both env kernels)."""
    from vmp.batched import BatchedVmEnv
    if big:
        monkeypatch.setenv("VMP_BIG_KERNEL", "1")
    base = dict(training_steps=10000, eval_steps=100000, allow_null_action=True, seed=0)
    base.update(BATCH_CFGS[ci])
    N, steps, K = 24, 120, 60
    seeds = np.array([7 + 4 * i for i in range(N - 2)] + [2**32 + 3, 2**40 + 11], np.int64)
    b = BatchedVmEnv(_cfg(base), N, seeds=seeds, device=DEV)
    b.eval(True)
    oes = []
    for s in seeds:
        e = O.OracleEnv(dict(base, seed=int(s)))
        e.eval(True)
        e.reset(int(s))
        oes.append(e)
    kl = base["reward_function"] == "kl"
    for t in range(steps):
        obs, rew, done, valid, act = b.heuristic_step(policy, want_actions=True, want_valid=True)
        rew, act = rew.cpu().numpy(), act.cpu().numpy()
        obs = obs.cpu().numpy()
        for i, e in enumerate(oes):
            a = e.firstfit() if policy == "firstfit" else e.bestfit()
            assert np.array_equal(a, act[i]), (t, i)
            o, r, _, _ = e.step(a)
            assert (T.kl_close(rew[i], r) if kl else rew[i] == r), (t, i, rew[i], r)
            assert np.array_equal(o, obs[i]), (t, i)
    rs, _ = b.rollout(policy, K)
    rs = rs.cpu().numpy()
    ctr = b.counters().cpu().numpy()
    for i, e in enumerate(oes):
        for k in range(K):
            a = e.firstfit() if policy == "firstfit" else e.bestfit()
            _, r, _, _ = e.step(a)
            assert (T.kl_close(rs[k, i], r) if kl else rs[k, i] == r), (k, i)
        assert np.array_equal(ctr[i], e.counters()[0]), i
        st = _np_state(b, i)
        assert state_hash(*[st[k] for k in ("vm_placement", "vm_cpu", "vm_memory", "cpu",
                                             "memory", "vm_remaining_runtime")]) == \
            state_hash(*e.state()), i


def test_external_random_actions_vs_oracle():
    """Dense, mostly-invalid external actions (every VM proposes every step) —
    the many-events path of the ordered per-PM replay."""
    from vmp.batched import BatchedVmEnv
    base = dict(pms=20, vms=200, arrival_rate=4.0, service_length=30, training_steps=10000,
                eval_steps=100000, allow_null_action=True, seed=0, reward_function="kl")
    N = 16
    seeds = np.arange(N, dtype=np.int64) * 4 + 100
    b = BatchedVmEnv(_cfg(base), N, seeds=seeds, device=DEV)
    oes = [O.OracleEnv(dict(base, seed=int(s))) for s in seeds]
    for e, s in zip(oes, seeds):
        e.reset(int(s))
    rng = np.random.default_rng(0)
    A = 22
    for t in range(150):
        acts = rng.integers(-1, A + 1, size=(N, 200))
        obs, rew, done, valid = b.step(torch.tensor(acts, dtype=torch.int32, device=DEV))
        rew, valid, obs = rew.cpu().numpy(), valid.cpu().numpy(), obs.cpu().numpy()
        for i, e in enumerate(oes):
            o, r, _, v = e.step(acts[i])
            assert T.kl_close(rew[i], r), (t, i)
            assert np.array_equal(v, valid[i]), (t, i)
            assert np.array_equal(o, obs[i]), (t, i)


def test_reset_masks_and_reseed():
    from vmp.batched import BatchedVmEnv
    base = dict(pms=10, vms=30, arrival_rate=0.5, service_length=20, training_steps=50,
                eval_steps=100, allow_null_action=True, seed=0)
    N = 8
    b = BatchedVmEnv(_cfg(base), N, device=DEV)
    for _ in range(60):
        _, _, done, _, _ = b.heuristic_step("firstfit")
    assert bool(done.all())
    mask = torch.zeros(N, dtype=torch.bool)
    mask[::2] = True
    new = torch.arange(N, dtype=torch.int64) * 4 + 1000
    b.reset(new, mask=mask)
    ctr = b.counters().cpu().numpy()
    assert np.all(ctr[::2, 5] == 1) and np.all(ctr[1::2, 5] == 61)
    e = O.OracleEnv(dict(base, seed=1000))
    e.reset(1000)
    for t in range(30):
        _, rew, _, _, _ = b.heuristic_step("firstfit")
        _, r, _, _ = e.step(e.firstfit())
        assert float(rew[0]) == r


def test_gae_matches_reference_loop():
    from vmp import _lib
    Tn, N = 100, 37
    g = torch.Generator().manual_seed(0)
    r = torch.randn(Tn, N, generator=g)
    d = (torch.rand(Tn, N, generator=g) < 0.05).float()
    v = torch.randn(Tn, N, generator=g)
    nv = torch.randn(Tn, N, generator=g)
    adv_ref = torch.zeros(Tn, N)
    gae = torch.zeros(N)
    for i in reversed(range(Tn)):  # ppo.py:237-242
        delta = r[i] + (1 - d[i]) * 0.99 * nv[i] - v[i]
        gae = delta + (1 - d[i]) * 0.99 * 0.98 * gae
        adv_ref[i] = gae
    dr, dd, dv, dnv = (x.to(DEV) for x in (r, d, v, nv))
    adv = torch.empty_like(dr)
    ret = torch.empty_like(dr)
    _lib.check(_lib.lib().vmp_gae(Tn, N, _lib.ptr(dr), _lib.ptr(dd), _lib.ptr(dv), _lib.ptr(dnv),
                                  0.99, 0.98, _lib.ptr(adv), _lib.ptr(ret), None))
    torch.cuda.synchronize()
    assert torch.allclose(adv.cpu(), adv_ref, atol=1e-5, rtol=1e-5)
    assert torch.allclose(ret.cpu(), adv_ref + v, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("policy,reward", [("firstfit", "wr"), ("bestfit", "kl"), (None, "ut")])
def test_large_v_block_kernel_vs_oracle(policy, reward):
    """V > 1024 runs k_env_big (one workgroup per env): P1000 / V3000 and
    P200 / V10000 (the stress config's slot count) against the C oracle,
    heuristic act+step and random external actions, bit-exact. The third case
    (2000 arrivals and hundreds of finishers per step at P1000 / V10000) runs
    the block kernel's > 512-event chunks of the accept and free phases."""
    from vmp.batched import BatchedVmEnv
    for P, V, lam, L, steps in ((1000, 3000, 9.0, 300, 40), (200, 10000, 30.0, 400, 25),
                                (1000, 10000, 2000.0, 2, 8)):
        cfg = dict(pms=P, vms=V, arrival_rate=lam, service_length=L, training_steps=10000,
                   eval_steps=100000, seed=5, reward_function=reward, sequence="uniform",
                   cap_target_util=True, beta=0.5, allow_null_action=True)
        n = 2
        seeds = np.array([5, 9], dtype=np.int64)
        b = BatchedVmEnv(_cfg(cfg), n, seeds=seeds, device=DEV)
        b.eval(True)
        orc = [O.OracleEnv(dict(cfg, seed=int(s))) for s in seeds]
        for e, s in zip(orc, seeds):
            e.eval(True)
            e.reset(int(s))
        g = np.random.default_rng(1)
        for t in range(steps):
            if policy is None:
                st = b.state()["vm_placement"].cpu().numpy()
                a = st.copy()
                u = g.random(st.shape)
                a[(st == P) & (u < 0.3)] = g.integers(0, P, size=int(((st == P) & (u < 0.3)).sum()))
                a[(st < P) & (u < 0.02)] = P
                _, rew, _, _ = b.step(torch.tensor(a, dtype=torch.int32, device=DEV))
                acts = a
            else:
                pre = b.heuristic_act(policy).cpu().numpy()  # act-only launch
                _, rew, _, _, act = b.heuristic_step(policy, want_actions=True)
                acts = act.cpu().numpy()
                assert np.array_equal(pre, acts), (P, V, t)
            rew = rew.cpu().numpy()
            for i, e in enumerate(orc):
                if policy is not None:
                    exp = e.firstfit() if policy == "firstfit" else e.bestfit()
                    assert np.array_equal(exp, acts[i]), (P, V, t, i)
                _, r, _, _ = e.step(acts[i].astype(np.int64))
                assert r == rew[i] or abs(r - rew[i]) <= 1e-12 * max(1.0, abs(r)), (P, V, t, i)
        sd = b.state()
        # stats() at V > 1024 derives the target means with k_target_means_lds
        # (its own LDS carve; the wr/ut steps do not compute them)
        stats = b.stats().cpu().numpy()
        for i, e in enumerate(orc):
            so = e.state()
            assert np.array_equal(sd["vm_placement"][i].cpu().numpy(), so[0]), (P, V)
            assert np.array_equal(sd["cpu"][i].cpu().numpy(), so[3]), (P, V)
            assert np.array_equal(b.counters()[i].cpu().numpy(), e.counters()[0]), (P, V)
            assert np.array_equal(stats[i], e.counters()[1]), (P, V, i, stats[i], e.counters()[1])
        b.close()


def test_c5_steady_state_bestfit_kl_vs_oracle():
    """BASELINE config 5 (P1000 / V10000, lambda = 1000/0.55/1000,
    L = 1000, reward kl, BestFit) from reset through the 2·L-step fill into the
    steady state (~1600 running and ~380 waiting VMs per env): 2000 fused
    rollout steps whose every reward must equal the oracle's, then 200 per-step
    act+step launches checked on actions, rewards and observations, then the
    full state and counters. Seeds 4·i as bench.py's."""
    from vmp.batched import BatchedVmEnv
    P, V = 1000, 10000
    cfg = dict(pms=P, vms=V, arrival_rate=round(1000 / 0.55 / 1000, 3), service_length=1000,
               training_steps=10000, eval_steps=100000, seed=0, reward_function="kl",
               sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
    seeds = np.array([0, 4], dtype=np.int64)
    b = BatchedVmEnv(_cfg(cfg), 2, seeds=seeds, device=DEV)
    b.eval(True)
    orc = [O.OracleEnv(dict(cfg, seed=int(s))) for s in seeds]
    for e, s in zip(orc, seeds):
        e.eval(True)
        e.reset(int(s))
    FF, T_CHECK = 2000, 200
    for k0 in range(0, FF, 250):
        rs, _ = b.rollout("bestfit", 250)
        rs = rs.cpu().numpy()
        for k in range(250):
            for i, e in enumerate(orc):
                _, r, _, _ = e.step(e.bestfit())
                assert T.kl_close(rs[k, i], r), (k0 + k, i, rs[k, i], r)
    pl = b.state()["vm_placement"].cpu().numpy()
    assert (pl < P).sum(1).min() > 1400 and (pl == P).sum(1).min() > 100, "not at steady state"
    for t in range(T_CHECK):
        obs, rew, _, _, act = b.heuristic_step("bestfit", want_actions=True)
        rew, act, obs = rew.cpu().numpy(), act.cpu().numpy(), obs.cpu().numpy()
        for i, e in enumerate(orc):
            a = e.bestfit()
            assert np.array_equal(a, act[i]), (t, i)
            o, r, _, _ = e.step(a)
            assert T.kl_close(rew[i], r), (t, i, rew[i], r)
            assert np.array_equal(o, obs[i]), (t, i)
    sd = b.state()
    ctr = b.counters().cpu().numpy()
    for i, e in enumerate(orc):
        so = e.state()
        for j, k in enumerate(("vm_placement", "vm_cpu", "vm_memory", "cpu", "memory",
                               "vm_remaining_runtime")):
            assert np.array_equal(sd[k][i].cpu().numpy(), so[j]), (k, i)
        assert np.array_equal(ctr[i], e.counters()[0]), i
    b.close()


@pytest.mark.parametrize("lam, FF", [(1.8182, 2900), (0.182, 2000)])
def test_headline_steady_state_firstfit_vs_oracle(lam, FF):
    """The bench workload (BASELINE headline: config/100.yml with vms = 1000,
    L = 1000, reward wr, FirstFit, training mode) at its steady state, at the
    shipped lambda = 1.8182 (10x load, ~800 waiting VMs) and at SURVEY §8(d)
    C-main's nominal lambda = 0.182 (100 % load, exp_suspension.py:19: ~724
    NULL slots, ~121 waiting): 256 envs (seeds 4·i as bench.py's)
    fast-forwarded FF >= 2·L steps by the fused rollout, whose rewards must
    equal the oracle's, then 200 per-step act+step launches (k_env<16, true>)
    with VMs finishing, checked on actions, rewards and observations, then 20
    external-action steps (k_env_ext) and the full state (remaining runtimes
    exported from the finish keys) and counters, for 4 envs."""
    from vmp.batched import BatchedVmEnv
    cfg = dict(pms=100, vms=1000, arrival_rate=lam, service_length=1000,
               training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
               sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
    N, CHK = 256, [0, 1, 97, 255]
    seeds = 4 * np.arange(N, dtype=np.int64)
    b = BatchedVmEnv(_cfg(cfg), N, seeds=seeds, device=DEV)
    orc = {i: O.OracleEnv(dict(cfg, seed=int(seeds[i]))) for i in CHK}
    for i, e in orc.items():
        e.eval(False)
        e.reset(int(seeds[i]))
    for k0 in range(0, FF, 100):
        rs, _ = b.rollout("firstfit", 100)
        rs = rs.cpu().numpy()
        for k in range(100):
            for i, e in orc.items():
                _, r, _, _ = e.step(e.firstfit())
                assert rs[k, i] == r, (k0 + k, i, rs[k, i], r)
    served0 = b.counters().cpu().numpy()[:, 1].copy()
    for t in range(200):
        obs, rew, _, _, act = b.heuristic_step("firstfit", want_actions=True)
        rew, act, obs = rew.cpu().numpy(), act.cpu().numpy(), obs.cpu().numpy()
        for i, e in orc.items():
            a = e.firstfit()
            assert np.array_equal(a, act[i]), (t, i)
            o, r, _, _ = e.step(a)
            assert rew[i] == r, (t, i, rew[i], r)
            assert np.array_equal(o, obs[i]), (t, i)
    served1 = b.counters().cpu().numpy()[:, 1]
    assert (served1 - served0).sum() > 10 * N, "no finishing VMs in the checked window"
    for t in range(20):
        acts = b.heuristic_act("firstfit")
        obs, rew, _, _ = b.step(acts)
        rew, obs = rew.cpu().numpy(), obs.cpu().numpy()
        for i, e in orc.items():
            o, r, _, _ = e.step(e.firstfit())
            assert rew[i] == r and np.array_equal(o, obs[i]), (t, i)
    sd = b.state()
    ctr = b.counters().cpu().numpy()
    for i, e in orc.items():
        so = e.state()
        for j, k in enumerate(("vm_placement", "vm_cpu", "vm_memory", "cpu", "memory",
                               "vm_remaining_runtime")):
            assert np.array_equal(sd[k][i].cpu().numpy(), so[j]), (k, i)
        assert np.array_equal(ctr[i], e.counters()[0]), i
    b.close()


def test_snapshot_restore_headline_bit_exact():
    """Checkpoint / resume of the batched env state (vmp_snapshot /
    vmp_restore): the headline config (P100 V1000, lambda 1.8182, L 1000, wr,
    FirstFit, training mode), 256 envs run 1 500 steps and are snapshotted;
    the snapshot goes through host memory (as torch.save would keep it) into a
    FRESH handle created with other seeds. Both handles then run the same 200
    steps (100 per-step act+step launches, then 100 fused): rewards, actions
    and observations equal at every step, counters and the full exported state
    equal at the end, and 3 envs equal the oracle replayed over all 1 700
    steps. A snapshot of another config or env count is refused."""
    from vmp._lib import VmpError
    from vmp.batched import BatchedVmEnv
    cfg = dict(pms=100, vms=1000, arrival_rate=1.8182, service_length=1000,
               training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
               sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
    N, CHK, FF = 256, [0, 131, 255], 1500
    seeds = 4 * np.arange(N, dtype=np.int64)
    a = BatchedVmEnv(_cfg(cfg), N, seeds=seeds, device=DEV)
    a.eval(False)
    for _ in range(FF // 100):
        a.rollout("firstfit", 100)
    snap = a.snapshot().cpu()
    b = BatchedVmEnv(_cfg(cfg, seed=7), N, seeds=seeds + 12345, device=DEV)
    b.eval(False)
    b.restore(snap)
    assert torch.equal(a.counters(), b.counters())
    orc = {i: O.OracleEnv(dict(cfg, seed=int(seeds[i]))) for i in CHK}
    for i, e in orc.items():
        e.eval(False)
        e.reset(int(seeds[i]))
        for _ in range(FF):
            e.step(e.firstfit())
    for t in range(100):
        oa, ra, _, _, aa = a.heuristic_step("firstfit", want_actions=True)
        ob, rb, _, _, ab = b.heuristic_step("firstfit", want_actions=True)
        assert torch.equal(ra, rb) and torch.equal(aa, ab) and torch.equal(oa, ob), t
        rb, ab, ob = rb.cpu().numpy(), ab.cpu().numpy(), ob.cpu().numpy()
        for i, e in orc.items():
            act = e.firstfit()
            assert np.array_equal(act, ab[i]), (t, i)
            o, r, _, _ = e.step(act)
            assert rb[i] == r and np.array_equal(o, ob[i]), (t, i)
    ra, _ = a.rollout("firstfit", 100)
    rb, _ = b.rollout("firstfit", 100)
    assert torch.equal(ra, rb)
    rb = rb.cpu().numpy()
    for k in range(100):
        for i, e in orc.items():
            _, r, _, _ = e.step(e.firstfit())
            assert rb[k, i] == r, (k, i)
    assert torch.equal(a.counters(), b.counters())
    sa, sb = a.state(), b.state()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    ctr = b.counters().cpu().numpy()
    for i, e in orc.items():
        so = e.state()
        for j, k in enumerate(("vm_placement", "vm_cpu", "vm_memory", "cpu", "memory",
                               "vm_remaining_runtime")):
            assert np.array_equal(sb[k][i].cpu().numpy(), so[j]), (k, i)
        assert np.array_equal(ctr[i], e.counters()[0]), i
    other = BatchedVmEnv(_cfg(cfg, arrival_rate=0.182), N, seeds=seeds, device=DEV)
    with pytest.raises(VmpError, match="another env count or config"):
        other.restore(snap)
    small = BatchedVmEnv(_cfg(cfg), 8, seeds=seeds[:8], device=DEV)
    with pytest.raises(ValueError, match="snapshot holds"):
        small.restore(snap)
    for e in (a, b, other, small):
        e.close()


_CHECK_QUIET_SCRIPT = r"""
import ctypes, sys
import numpy as np, torch
from vmp import _lib
from vmp.batched import BatchedVmEnv
from vmp.config import Config
L = _lib.lib()
def take():
    n = ctypes.c_int64(-1)
    _lib.check(L.vmp_debug_quiet_violations(ctypes.byref(n)))
    return n.value
cfg = dict(pms=100, vms=1000, arrival_rate=1.8182, service_length=1000, training_steps=10000,
           eval_steps=100000, seed=0, reward_function="wr", sequence="uniform",
           cap_target_util=True, beta=0.5, allow_null_action=True)
N = 256
seeds = 4 * np.arange(N, dtype=np.int64)
a = BatchedVmEnv(Config(**cfg), N, seeds=seeds, device="cuda:0")
take()
for _ in range(25):
    a.rollout("firstfit", 100)
for _ in range(50):
    a.heuristic_step("firstfit")
for t in range(30):   # external steps (k_env_ext clears the bit) between per-step launches
    a.step(a.heuristic_act("firstfit"))
    a.heuristic_step("bestfit" if t % 3 == 0 else "firstfit")
a.reset(seeds, mask=torch.arange(N) % 7 == 0, obs=False)   # masked reset
a.rollout("firstfit", 300)
snap = a.snapshot()
b = BatchedVmEnv(Config(**cfg), N, seeds=seeds + 1, device="cuda:0")
b.restore(snap)
for _ in range(100):
    b.heuristic_step("firstfit")
clean = take()
# negative control: an env whose header says quiet gets its PM loads zeroed
# behind the bit's back (every pending VM now fits): the check must count it
s = snap.cpu().numpy().copy()
hdr = s[256:256 + 256 * N].view(np.uint64).reshape(N, 32)
quiet = np.flatnonzero((hdr[:, 31] >> np.uint64(62)) & np.uint64(1))
assert quiet.size > 0, "no quiet env in the snapshot"
e = int(quiet[0])
pm = s[256 + 256 * N:256 + 256 * N + 16 * N * 100].view(np.float64).reshape(N, 200)
pm[e, :] = 0.0
b.restore(torch.from_numpy(s))
b.heuristic_step("firstfit")
bad = take()
print("RESULT", clean, bad, quiet.size)
"""


def test_quiet_bit_check_build():
    """the quiet-step skip (EnvHdr::pad bit 62) is exact only while
    every writer of env state keeps the bit exact. The -DVMP_CHECK_QUIET build
    (vmp/libvmp_checkquiet.so) evaluates the fit test on quiet steps too and
    counts the contradictions. Headline-config envs driven through every
    state writer — fused rollouts, per-step FirstFit / BestFit, external
    actions, a masked reset, a snapshot restored into a fresh handle — must
    count 0; a negative control (a quiet env's PM loads zeroed in a snapshot,
    so its pending VMs fit) must count > 0. The normal build reports EINVAL."""
    import ctypes
    import os
    import subprocess
    import sys
    from vmp import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(root, "vm-placement-migration-gym_amd")
    so = os.path.join(pkg, "vmp", "libvmp_checkquiet.so")
    assert os.path.exists(so), "build the check variant: make -C vm-placement-migration-gym_amd check-quiet"
    n = ctypes.c_int64()
    rc = _lib.lib().vmp_debug_quiet_violations(ctypes.byref(n))
    assert rc == -1  # VMP_EINVAL in the normal build
    env = dict(os.environ, VMP_LIB_PATH=so, PYTHONPATH=os.pathsep.join([root, pkg]))
    r = subprocess.run([sys.executable, "-c", _CHECK_QUIET_SCRIPT], env=env, cwd=root,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT")][-1]
    clean, bad, n_quiet = (int(x) for x in line.split()[1:])
    assert clean == 0, clean
    assert bad > 0 and n_quiet > 0, (bad, n_quiet)


@pytest.mark.parametrize("big", [False, True], ids=["wave", "block"])
def test_finish_keys_short_service_vs_oracle(big, monkeypatch):
    """Finish keys under churn: service lengths of 1-6 steps
    (Poisson(2) + 1), so VMs placed with one step left finish in the step that
    places them, and external actions that suspend running VMs and re-place
    waiting ones every step (WAIT <-> PM moves rewrite the time word by -t / +t).
    The exported state — remaining runtimes included — and the counters must be
    the oracle's after every step, through both env kernels."""
    from vmp.batched import BatchedVmEnv
    if big:
        monkeypatch.setenv("VMP_BIG_KERNEL", "1")
    base = dict(pms=12, vms=90, arrival_rate=3.0, service_length=2, training_steps=10000,
                eval_steps=100000, allow_null_action=True, seed=0, reward_function="ut")
    N, P = 6, 12
    seeds = np.arange(N, dtype=np.int64) * 4 + 7
    b = BatchedVmEnv(_cfg(base), N, seeds=seeds, device=DEV)
    oes = [O.OracleEnv(dict(base, seed=int(s))) for s in seeds]
    for e, s in zip(oes, seeds):
        e.reset(int(s))
    rng = np.random.default_rng(3)
    keys = ("vm_placement", "vm_cpu", "vm_memory", "cpu", "memory", "vm_remaining_runtime")
    for t in range(120):
        pl = b.state()["vm_placement"].cpu().numpy()
        acts = pl.copy()
        u = rng.random(pl.shape)
        susp = (pl < P) & (u < 0.2)
        acts[susp] = P
        wait = pl == P
        acts[wait & (u < 0.7)] = rng.integers(0, P, size=pl.shape)[wait & (u < 0.7)]
        _, rew, _, valid = b.step(torch.tensor(acts, dtype=torch.int32, device=DEV))
        rew, valid = rew.cpu().numpy(), valid.cpu().numpy()
        sd = {k: v.cpu().numpy() for k, v in b.state().items()}
        ctr = b.counters().cpu().numpy()
        for i, e in enumerate(oes):
            _, r, _, v = e.step(acts[i])
            assert rew[i] == r and np.array_equal(v, valid[i]), (t, i)
            so = e.state()
            for j, k in enumerate(keys):
                assert np.array_equal(sd[k][i], so[j]), (t, i, k)
            assert np.array_equal(ctr[i], e.counters()[0]), (t, i)
    assert int(b.counters().cpu().numpy()[:, 2].sum()) > 100  # suspensions happened


def test_nominal_load_extra_null_slots_do_not_change_the_trajectory():
    """at lambda = 0.182 (100 % load) free slots never run out, so
    V = 300 (config/100.yml) and V = 1000 (the headline's vms) must walk the
    same trajectory: equal rewards at every one of 2 500 fused FirstFit steps,
    equal counters, no drops, equal PM loads. A size-independent check of the
    full-size C-main nominal workload (64 envs per V)."""
    from vmp.batched import BatchedVmEnv
    N = 64
    base = dict(pms=100, arrival_rate=0.182, service_length=1000, training_steps=10000,
                eval_steps=100000, seed=0, reward_function="wr", sequence="uniform",
                cap_target_util=True, beta=0.5, allow_null_action=True)
    seeds = 4 * np.arange(N, dtype=np.int64)
    envs = {V: BatchedVmEnv(_cfg(dict(base, vms=V)), N, seeds=seeds, device=DEV)
            for V in (300, 1000)}
    for k in range(5):
        r = {V: e.rollout("firstfit", 500)[0].cpu().numpy() for V, e in envs.items()}
        assert np.array_equal(r[300], r[1000]), k
    c = {V: e.counters().cpu().numpy() for V, e in envs.items()}
    assert np.array_equal(c[300], c[1000])
    assert c[300][:, 4].sum() == 0, "drops: the invariance does not apply"
    st = {V: e.state() for V, e in envs.items()}
    for k in ("cpu", "memory"):
        assert torch.equal(st[300][k], st[1000][k]), k
    pl3, pl10 = st[300]["vm_placement"].cpu(), st[1000]["vm_placement"].cpu()
    assert torch.equal(pl3, pl10[:, :300]) and bool((pl10[:, 300:] == 101).all())
    for e in envs.values():
        e.close()


def test_unknown_reward_function_asserts_at_first_rewarded_step():
    """env.py:123-156: an unknown reward_function is only reached (assert
    False, 'Function does not exist') once a step has VMs to reward; VmEnv
    constructs, resets and steps with reward 0 until then."""
    from vmp.config import Config
    from vmp.env import VmEnv
    cfg = Config(pms=10, vms=30, arrival_rate=0.05, service_length=20, training_steps=100,
                 eval_steps=100, seed=3, reward_function="nope", allow_null_action=True)
    env = VmEnv(cfg, device=DEV)
    obs, _ = env.reset(seed=3)
    quiet = 0
    with pytest.raises(AssertionError, match="Function does not exist: nope"):
        for _ in range(200):
            obs, r, _, _, _ = env.step(obs[:cfg.vms].astype(np.int64))
            assert r == 0.0
            quiet += 1
    assert quiet >= 1  # arrivals at rate 0.05: the first steps have no VM
    env.close()


@pytest.mark.parametrize("reward", ["wr", "ut"])
@pytest.mark.parametrize("big", [False, True], ids=["wave", "block"])
def test_step_hints_across_launch_kinds_vs_oracle(big, reward, monkeypatch):
    """The header's step hints (EnvHdr::pad: NULL slots left, next finish key,
    the quiet bit and 'some VM exists') are written by one launch and read by
    the next, which may be another kind of launch. A small env that fills up
    (V 60, 2 arrivals a step, service ~12 steps: quiet steps where nothing fits,
    finishes or arrives, between refill bursts) is driven by a fixed mix of
    per-step FirstFit / BestFit launches, fused 3-step rollouts and external
    steps that suspend some VMs; rewards, the full state and the counters must
    be the oracle's after every launch (wr takes the stats skip, ut does not)."""
    from vmp.batched import BatchedVmEnv
    if big:
        monkeypatch.setenv("VMP_BIG_KERNEL", "1")
    base = dict(pms=8, vms=60, arrival_rate=2.0, service_length=12, training_steps=10000,
                eval_steps=100000, allow_null_action=True, seed=0, reward_function=reward,
                sequence="uniform", cap_target_util=True, beta=0.5)
    N, P = 12, 8
    seeds = np.arange(N, dtype=np.int64) * 3 + 11
    b = BatchedVmEnv(_cfg(base), N, seeds=seeds, device=DEV)
    oes = [O.OracleEnv(dict(base, seed=int(s))) for s in seeds]
    for e, s in zip(oes, seeds):
        e.eval(False)
        e.reset(int(s))
    rng = np.random.default_rng(5)
    keys = ("vm_placement", "vm_cpu", "vm_memory", "cpu", "memory", "vm_remaining_runtime")
    kinds = ["ff", "ff", "roll", "bf", "ff", "ext", "ff", "roll", "ff", "ff"]
    n_quiet_like = 0
    for t in range(150):
        kind = kinds[t % len(kinds)]
        if kind == "roll":
            rs = b.rollout("firstfit", 3)[0].cpu().numpy()
            for k in range(3):
                for i, e in enumerate(oes):
                    _, r, _, _ = e.step(e.firstfit())
                    assert rs[k, i] == r, (t, k, i)
        elif kind == "ext":
            pl = b.state()["vm_placement"].cpu().numpy()
            acts = b.heuristic_act("firstfit").cpu().numpy().astype(np.int64)
            susp = (pl < P) & (rng.random(pl.shape) < 0.1)
            acts[susp] = P
            _, rew, _, _ = b.step(torch.tensor(acts, dtype=torch.int32, device=DEV))
            rew = rew.cpu().numpy()
            for i, e in enumerate(oes):
                _, r, _, _ = e.step(acts[i])
                assert rew[i] == r, (t, i)
        else:
            pol = "firstfit" if kind == "ff" else "bestfit"
            c0 = b.counters().cpu().numpy()
            obs, rew, _, _, act = b.heuristic_step(pol, want_actions=True)
            rew, act, obs = rew.cpu().numpy(), act.cpu().numpy(), obs.cpu().numpy()
            d = b.counters().cpu().numpy() - c0
            n_quiet_like += int(((d[:, 1] == 0) & (d[:, 3] == 0)).sum())
            for i, e in enumerate(oes):
                a = e.firstfit() if kind == "ff" else e.bestfit()
                assert np.array_equal(a, act[i]), (t, i)
                o, r, _, _ = e.step(a)
                assert rew[i] == r, (t, i, rew[i], r)
                assert np.array_equal(o, obs[i]), (t, i)
        sd = {k: v.cpu().numpy() for k, v in b.state().items()}
        ctr = b.counters().cpu().numpy()
        for i, e in enumerate(oes):
            so = e.state()
            for j, k in enumerate(keys):
                assert np.array_equal(sd[k][i], so[j]), (t, i, k)
            assert np.array_equal(ctr[i], e.counters()[0]), (t, i)
    assert n_quiet_like > 100, "no quiet per-step launches in the mix"
    b.close()

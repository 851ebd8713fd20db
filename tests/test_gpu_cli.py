"""The reference CLI path (main.py:34-86) on the GPU env: BASELINE config 1
(config/10.yml, firstfit, eval_steps 1000, seed 1) reproduces the reference's
per-step rewards and counters through run()/Base.test/Record, and a PPO eval
with the reference's weights file layout runs end to end."""
import numpy as np
import pytest
import torch

from tests import traj as T

pytestmark = pytest.mark.gpu

ENV10 = dict(pms=10, vms=30, service_length=1000, arrival_rate=0.0182, training_steps=10000,
             eval_steps=1000, seed=1, reward_function="kl", cap_target_util=True,
             sequence="uniform", beta=0.5, allow_null_action=True)


def test_cli_firstfit_c1_matches_reference():
    from vmp.main import Args, run
    d = T.load("c1_10yml_ff")
    rec = run(Args(agent="firstfit", reward="wr", config={"environment": dict(ENV10), "agents": {}},
                   eval=True, silent=True))
    assert np.array_equal(np.array(rec.rewards), d["reward"][0])
    ctr = d["counters"][-1]
    assert rec.total_requests[-1] == ctr[0] and rec.served_requests[-1] == ctr[1]
    assert rec.suspended[-1] == ctr[2] and rec.placed[-1] == ctr[3]
    s = rec.get_summary()
    assert s["total rewards"] == np.round(d["reward"][0].sum(), 3) == -3.103
    assert s["total requests"] == 12


def test_cli_ppo_eval_with_reference_weights(tmp_path):
    from vmp.main import Args, run
    w = np.load(T.GOLDEN + "/ppo10_wr_weights.npz")
    path = str(tmp_path / "ppo-wr.pt")
    torch.save({"_orig_mod." + k: torch.tensor(w[k]) for k in w.files}, path)
    env = dict(ENV10, eval_steps=40, arrival_rate=0.5, service_length=20)
    rec = run(Args(agent="ppo", reward="wr", config={"environment": env, "agents": {
        "ppo": {"hidden_size": 512, "masked": True, "episodes": 1}}}, weightspath=path,
        eval=True, silent=True, output=str(tmp_path / "out.json")))
    assert len(rec.rewards) == 40 and rec.total_requests[-1] > 0
    assert (tmp_path / "out.json").exists()

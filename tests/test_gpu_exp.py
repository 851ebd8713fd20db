"""Batched experiment sweeps (vmp.exp, exp_suspension.py re-expressed): the
published exp_suspension rows come out of the sweep's own CSV writer, and a
PPO cell (weights file in the reference's format) runs through a captured
act+step graph with the device recorder."""
import csv
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _published():
    with open(os.path.join(GOLDEN, "exp_suspension_data.csv")) as f:
        return {(r[0], r[1], r[2]): ",".join(x.strip() for x in r) for r in csv.reader(f)}


def test_suspension_sweep_rows_match_published():
    from vmp.exp import suspension_sweep
    rows = suspension_sweep(agents=("firstfit", "bestfit"), loads=[0.5], lengths=[100])
    pub = _published()
    assert len(rows) == 4
    for row in rows:
        a, ld, sr = row.split(",")[:3]
        assert row == pub[(a, ld, sr)], (row, pub[(a, ld, sr)])


def test_suspension_sweep_ppo_cell(tmp_path):
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.exp import ENV100, PPO100, suspension_sweep
    from vmp.ppo import PPOAgent, PPOConfig
    env = BatchedVmEnv(Config(**ENV100), 1, device="cuda:0")
    path = str(tmp_path / "ppo-test.pt")
    torch.manual_seed(0)
    PPOAgent(env, PPOConfig(**PPO100)).save_model(path)
    env.close()
    rows = suspension_sweep(agents=("ppo",), loads=[1.0], lengths=[], seeds=(0, 1),
                            weights=path, eval_steps=300)
    name, load, sr, served, susp, valid = rows[0].split(",")[:6]
    assert name == "ppo-test" and load == "1.0" and sr == "1000"
    assert int(valid) >= int(susp) >= 0 and int(served) >= 0

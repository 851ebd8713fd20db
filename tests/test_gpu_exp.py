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


def _summary(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return [",".join(x.strip() for x in r) for r in csv.reader(f)][1:]


# exp_performance's published load-1.0 rows carry the wr return (their other
# columns do not depend on the reward), the load-0.6 rows the ut return: each
# cell runs with the reward that printed its row.
def test_performance_rows_match_published():
    """data/exp_performance/summary.csv, heuristic rows: config/100.yml at
    100 % and 60 % load, 5 seeds x 100 000 eval steps per row, every column
    (return, drop rate, served, CPU/memory mean and variance incl. the
    reference's variance-over-seeds memory column, pending, waiting, slowdown)."""
    from vmp import exp
    pub = {tuple(r.split(",")[:2]): r for r in _summary("exp_performance_summary.csv")}
    cells = [exp.performance_cell(ag, ag, ld, "wr" if ld == 1.0 else "ut")
             for ld in (1.0, 0.6) for ag in ("bestfit", "firstfit")]
    rows = exp.performance_sweep(cells)
    for row in rows:
        assert row == pub[tuple(row.split(",")[:2])], row


def test_performance_small_rows_match_published():
    """data/exp_performance_small/summary.csv heuristic rows (config/10.yml, seeds 1..5)."""
    from vmp import exp
    pub = {r.split(",")[0]: r for r in _summary("exp_performance_small_summary.csv")}
    cells = [exp.performance_cell(ag, ag, 1.0, small=True) for ag in ("bestfit", "firstfit")]
    for row in exp.performance_sweep(cells):
        assert row == pub[row.split(",")[0]], row


def test_vm_size_rows_match_published():
    """data/exp_vm_size/summary.csv heuristic rows: lowuniform / highuniform VM
    sizes, reward kl (100 000-step kl returns to 4 decimals)."""
    from vmp import exp
    pub = _summary("exp_vm_size_summary.csv")
    expect = [r for r in pub if not r.startswith("ppo,")]
    cells = [exp.vm_size_cell(ag, seq) for seq in ("lowuniform", "highuniform")
             for ag in ("firstfit", "bestfit")]
    assert exp.vm_size_sweep(cells) == expect


def test_migration_ratio_bestfit_rows_match_published():
    """data/exp_migration_ratio/data.csv bestfit rows (config/100.yml seed 0,
    100 000 steps; BestFit ignores the ratio)."""
    from vmp import exp
    with open(os.path.join(GOLDEN, "exp_migration_ratio_data.csv")) as f:
        pub = {r.strip() for r in f if r.startswith("bestfit,")}
    cells = [exp.migration_cell("bestfit", "ut", r) for r in (0.0, 0.001)]
    rows = exp.migration_sweep(cells)
    assert rows[0] == "bestfit,ut,0.000,0.761,0.000" and set(rows) <= pub, rows


def test_exp_cli(tmp_path, capsys):
    """python -m vmp.exp <experiment>: header plus one row per cell, to --out."""
    from vmp import exp
    out = tmp_path / "m.csv"
    exp.main(["migration_ratio", "--agents", "bestfit", "--eval-steps", "200", "--out", str(out)])
    lines = out.read_text().splitlines()
    assert lines[0] == exp.MIGRATION_HEADER and len(lines) == 11
    exp.main(["performance", "--loads", "1.0,0.6", "--eval-steps", "200"])
    lines = capsys.readouterr().out.splitlines()
    assert lines[-5] == exp.PERFORMANCE_HEADER and len(lines[-4:]) == 4


def test_graph_recorded_rollout_equals_plain_launches():
    """The captured recorded rollout (graph_steps) gives the same Record
    summaries as one launch pair per step, including a remainder."""
    from vmp import exp
    cells = [exp.performance_cell("bestfit", "bestfit", 1.0, "kl", seeds=(0, 1, 2))]
    a = exp.run_cells(cells, eval_steps=1234, graph_steps=100)[0]
    b = exp.run_cells(cells, eval_steps=1234, graph_steps=0)[0]
    for x, y in zip(a, b):
        assert x.keys() == y.keys()
        for key in x:
            assert (x[key] == y[key]) or (x[key] != x[key] and y[key] != y[key]), key

"""Host arithmetic of the batched experiment drivers (vmp.exp): configs and
the summary-row formulas, checked against the reference drivers' numpy
expressions on synthetic per-step series (no GPU)."""
import numpy as np

from vmp import exp


def _summaries(cpu, mem, served=(10, 12, 11)):
    """Device-summary dicts as vmp.record.summary_from_device builds them from
    the recorder's sums, from per-seed [T, P] series."""
    S, T, P = cpu.shape
    col = mem.sum(axis=0)  # [T, P] sum over the handle's envs
    out = []
    for s in range(S):
        out.append({"_return": 1.0 * s, "_drop_rate": 0.1, "total served VMs": served[s],
                    "total suspend actions": 0, "_cpu_mean": cpu[s].mean(),
                    "_cpu_var": cpu[s].var(axis=1).mean(), "_mem_mean": mem[s].mean(),
                    "_mem_var": mem[s].var(axis=1).mean(), "_mem2": (mem[s] ** 2).mean(),
                    "_xmem": (mem[s] * col).sum() / (T * P), "_mean_pending": 0.2,
                    "_waiting": 0.5, "_mean_slowdown": 0.0})
    return out


def test_performance_row_memory_variance_over_seeds():
    """exp_performance.py:107-114 takes np.var(memory, axis=0) (over the seeds);
    the row rebuilds it from per-env E[x^2] and the cross-env sums."""
    rng = np.random.default_rng(3)
    cpu = rng.random((3, 50, 10))
    mem = rng.random((3, 50, 10))
    cell = exp.performance_cell("firstfit", "firstfit", 1.0)
    row = exp.performance_row(cell, _summaries(cpu, mem)).split(",")
    assert float(row[9]) == float("%.3f" % np.mean(np.var(mem, axis=0)))
    assert float(row[7]) == float("%.3f" % np.mean(np.mean(np.var(cpu, axis=2), axis=0)))
    assert row[4] == "11"  # '%d' of the mean served count


def test_experiment_configs():
    c = exp.performance_config(1.0)
    assert c["arrival_rate"] == 0.1818 and c["reward_function"] == "ut"
    assert exp.performance_config(0.6, env=exp.ENV10)["arrival_rate"] == 0.0109
    assert exp.performance_config(1.0, jobname="ppo-unmasked")["allow_null_action"] is False
    assert exp.performance_cell("ppo", "ppo-unmasked", 1.0).ppo == {"masked": False}
    assert exp.performance_cell("firstfit", "firstfit", 1.0, small=True).seeds == (1, 2, 3, 4, 5)
    v = exp.vm_size_config("highuniform")
    assert v["arrival_rate"] == 100 / 0.625 / 1000 and v["reward_function"] == "kl"


def test_reward_and_migration_rows():
    rng = np.random.default_rng(4)
    cpu, mem = rng.random((3, 20, 10)), rng.random((3, 20, 10))
    cell = exp.reward_cell("ppo", "kl", "w.pt")
    row = exp.reward_row(cell, _summaries(cpu, mem)).split(",")
    assert row[:2] == ["ppo", "kl"] and cell.cfg["arrival_rate"] == 0.182
    assert float(row[9]) == float("%.3f" % np.mean(np.mean(np.var(mem, axis=2), axis=0)))
    m = exp.migration_cell("bestfit", "ut", 0.003)
    assert exp.migration_row(m, _summaries(cpu, mem)) == "bestfit,ut,0.003,%.3f,0.000" % cpu[0].mean()

"""Record: per-step evaluation metrics of Base.test, field for field the
reference's src/record.py:5-160 (same attribute names, summary keys and JSON
layout, so plots.ipynb and the exp_* drivers read our files unchanged)."""
import json
import os

import numpy as np


class Record:
    def __init__(self, agent, env_config, agent_config):
        self.agent = agent
        self.env_config = env_config if isinstance(env_config, dict) else vars(env_config)
        self.agent_config = agent_config if isinstance(agent_config, dict) else None
        self.WAIT_STATUS = self.env_config["pms"]
        self.cpu = []
        self.memory = []
        self.used_pm = []
        self.vm_placements = []
        self.waiting_ratio = []
        self.actions = []
        self.rewards = []
        self.dropped_requests = []
        self.total_requests = []
        self.vm_arrival_steps = []
        self.target_cpu_mean = []
        self.target_memory_mean = []
        self.served_requests = []
        self.total_cpu_requested = []
        self.total_memory_requested = []
        self.suspended = []
        self.placed = []
        self.vmsratio = []
        self.rank = []

    # record.py:33-51: split each slot's placement history at its arrival steps
    @property
    def unique_vms_placement(self):
        out = []
        vm_placements = np.transpose(np.array(self.vm_placements))
        for vm, vm_status in enumerate(vm_placements):
            if len(self.vm_arrival_steps[vm]) == 0:
                continue
            start = 0
            for end in self.vm_arrival_steps[vm][1:]:
                end -= 2  # vm_placements starts from timestep 2
                seg = vm_status[start:end]
                out.append(seg[seg <= self.WAIT_STATUS])
                start = end
            seg = vm_status[start:]
            assert seg[seg <= self.WAIT_STATUS].size != 0, seg[seg <= self.WAIT_STATUS]
            out.append(seg[seg <= self.WAIT_STATUS])
        return out

    def _first_run(self, status):
        running = np.where(status < self.WAIT_STATUS)[0]
        return running[0] if running.size > 0 else None

    @property
    def pending_rates(self):  # record.py:53-65 (allocated_at == 0 counts as "never", as there)
        rates = []
        for status in self.unique_vms_placement:
            status = np.array(status)
            at = self._first_run(status)
            rates.append(np.around((at + 1.0) / len(status), 3) if at else 1.0)
        return rates

    @property
    def slowdown_rates(self):  # record.py:67-82
        rates = []
        for status in self.unique_vms_placement:
            status = np.array(status)
            at = self._first_run(status)
            if at:
                slow = np.count_nonzero(status[at:] == self.WAIT_STATUS)
                life = len(status) - at - 1
                rates.append(0 if life == 0 else np.around(slow / life, 3))
        return rates if rates else [0]

    @property
    def vm_lifetime(self):  # record.py:84-95
        life = []
        for status in self.unique_vms_placement:
            status = np.array(status)
            at = self._first_run(status)
            life.append(len(status) - at - 1 if at else 0)
        return life

    @property
    def drop_rate(self):
        dropped = np.array(self.dropped_requests)
        total = np.array(self.total_requests)
        return np.divide(dropped, total, out=np.zeros(dropped.shape, dtype=float),
                         where=total != 0)

    @property
    def total_rewards(self):
        rewards = np.array(self.rewards)
        rewards[rewards < -1e7] = np.mean(rewards[rewards > -1e7])
        return np.round(np.sum(rewards), 3)

    def get_summary(self):  # record.py:110-133, same keys and rounding
        pend = self.pending_rates
        slow = self.slowdown_rates
        return {
            "total rewards": self.total_rewards,
            "total served VMs": self.served_requests[-1],
            "total requests": self.total_requests[-1],
            "total cpu requested": np.round(self.total_cpu_requested, 3),
            "total memory requested": np.round(self.total_memory_requested, 3),
            "total suspend actions": self.suspended[-1],
            "total place actions": self.placed[-1],
            "average VM life": np.round(np.mean(self.vm_lifetime), 3),
            "average pending": np.round(np.mean(pend), 3),
            "median pending": np.round(np.median(pend), 3),
            "max pending": np.round(np.max(pend), 3) if len(pend) > 0 else 0,
            "average slowdown": np.round(np.mean(slow), 3),
            "median slowdown": np.round(np.median(slow), 3),
            "max slowdown": np.round(np.max(slow), 3),
            "drop rate": np.round(np.mean(self.drop_rate), 3),
            "cpu mean": np.round(np.mean(self.cpu), 3),
            "cpu mean target": np.round(np.mean(self.target_cpu_mean), 3),
            "cpu std": np.round(np.std(self.cpu), 3),
            "memory mean": np.round(np.mean(self.memory), 3),
            "memory mean target": np.round(np.mean(self.target_memory_mean), 3),
            "memory std": np.round(np.std(self.memory), 3),
            "rank mean": np.round(np.mean(self.rank), 3),
        }

    def save(self, path: str):
        self.summary = self.get_summary()
        parent = os.path.dirname(path)
        if parent:
            os.makedirs(parent, exist_ok=True)
        with open(path, "w") as f:
            f.write(json.dumps(vars(self), cls=NpEncoder))

    @classmethod
    def import_record(cls, agent: str, jsondict: dict):  # record.py:144-168
        r = cls(agent, jsondict["env_config"], jsondict["agent_config"])
        for k in ("cpu", "memory", "vm_placements", "waiting_ratio", "actions", "rewards",
                  "total_requests", "dropped_requests", "vm_arrival_steps", "target_cpu_mean",
                  "target_memory_mean", "served_requests", "total_cpu_requested",
                  "total_memory_requested", "rank", "suspended"):
            setattr(r, k, jsondict[k])
        for k in ("used_pm", "placed"):
            if k in jsondict:
                setattr(r, k, jsondict[k])
        return r


class NpEncoder(json.JSONEncoder):
    def default(self, obj):
        if isinstance(obj, np.integer):
            return int(obj)
        if isinstance(obj, np.floating):
            return float(obj)
        if isinstance(obj, np.ndarray):
            return obj.tolist()
        return super().default(obj)


# include/vmp.h VMP_REC_* indices of the device recorder's sums
REC_STEPS, REC_REWARD, REC_CPU, REC_CPU2, REC_MEM, REC_MEM2, REC_RANK, REC_DROP = range(8)
REC_TCM, REC_TMM, REC_WAITING, REC_LIFE_SUM, REC_LIVES, REC_REWARD_OK, REC_N_OK, REC_N_BAD = \
    range(8, 16)
REC_CPUVAR, REC_MEMVAR, REC_XMEM = range(16, 19)


def _hist_stats(h):
    """(mean, median, max) of values i/1000 counted by h[i], numpy's definitions."""
    n = int(h.sum())
    if n == 0:
        return None
    idx = np.flatnonzero(h)
    vals = idx / 1000.0
    mean = float((h[idx] * vals).sum() / n)
    cum = np.cumsum(h[idx])
    lo = vals[np.searchsorted(cum, (n - 1) // 2 + 1)]
    hi = vals[np.searchsorted(cum, n // 2 + 1)]
    return mean, (lo + hi) / 2.0, float(vals[-1])


def summary_from_device(hist, sums, counters, stats, pms):
    """Record.get_summary (record.py:110-134) from the device recorder of one env
    (vmp_record_read) plus its counters [total_requests, served, suspend, place,
    dropped, timestep] and stats [waiting, tcm, tmm, total_cpu_req, total_mem_req]."""
    T = sums[REC_STEPS]
    n_eq = T - sums[REC_N_OK] - sums[REC_N_BAD]  # rewards exactly -1e7 stay as they are
    mean_ok = sums[REC_REWARD_OK] / sums[REC_N_OK] if sums[REC_N_OK] else np.nan
    total = sums[REC_REWARD_OK] + n_eq * -1e7 + (sums[REC_N_BAD] * mean_ok if sums[REC_N_BAD] else 0.0)
    pend = _hist_stats(hist[0])
    slow = _hist_stats(hist[1]) or (0.0, 0.0, 0.0)  # slowdown_rates defaults to [0]
    TP = T * pms
    cm, mm = sums[REC_CPU] / TP, sums[REC_MEM] / TP
    return {
        "total rewards": np.round(total, 3),
        "total served VMs": int(counters[1]),
        "total requests": int(counters[0]),
        "total cpu requested": np.round(stats[3], 3),
        "total memory requested": np.round(stats[4], 3),
        "total suspend actions": int(counters[2]),
        "total place actions": int(counters[3]),
        "average VM life": np.round(sums[REC_LIFE_SUM] / sums[REC_LIVES], 3) if sums[REC_LIVES] else np.nan,
        "average pending": np.round(pend[0], 3) if pend else np.nan,
        "median pending": np.round(pend[1], 3) if pend else np.nan,
        "max pending": np.round(pend[2], 3) if pend else 0,
        "average slowdown": np.round(slow[0], 3),
        "median slowdown": np.round(slow[1], 3),
        "max slowdown": np.round(slow[2], 3),
        "drop rate": np.round(sums[REC_DROP] / T, 3),
        "cpu mean": np.round(cm, 3),
        "cpu mean target": np.round(sums[REC_TCM] / T, 3),
        "cpu std": np.round(np.sqrt(max(sums[REC_CPU2] / TP - cm * cm, 0.0)), 3),
        "memory mean": np.round(mm, 3),
        "memory mean target": np.round(sums[REC_TMM] / T, 3),
        "memory std": np.round(np.sqrt(max(sums[REC_MEM2] / TP - mm * mm, 0.0)), 3),
        "rank mean": np.round(sums[REC_RANK] / T, 3),
        # unrounded columns the exp_* drivers print (exp_suspension.py:51-58)
        "_mean_life": sums[REC_LIFE_SUM] / sums[REC_LIVES] if sums[REC_LIVES] else np.nan,
        "_mean_pending": pend[0] if pend else np.nan,
        "_mean_slowdown": slow[0],
        "_max_slowdown": slow[2],
        # per-step series means the exp_performance / exp_vm_size summaries print
        "_return": np.round(total, 3),
        "_drop_rate": sums[REC_DROP] / T,
        "_cpu_mean": cm,
        "_mem_mean": mm,
        "_cpu_var": sums[REC_CPUVAR] / T,
        "_mem_var": sums[REC_MEMVAR] / T,
        "_waiting": sums[REC_WAITING] / T,
        "_mem2": sums[REC_MEM2] / TP,
        "_xmem": sums[REC_XMEM] / TP,
    }

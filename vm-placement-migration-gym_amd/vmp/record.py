"""Record (src/record.py:5-176) for the MI355X env.

The reference derives every evaluation metric on the host from per-step lists
(record.py:34-134: splitting each slot's placement history at its arrival
steps, then pending / slowdown / lifetime per VM life). Here those metrics are
accumulated on the device while the episode runs (vmp_record_enable /
vmp_record_read, csrc/vmp_record.hip) and `summary_from_device` turns the
recorder's sums and rate histograms into get_summary()'s dict. `Record` keeps
the reference's attribute names for the per-step traces Base.test appends, so
save() writes the JSON layout plots.ipynb and the exp_* drivers read, and its
summary is the device one. (The literal host restatement of record.py lives in
tests/record_literal.py, where it checks the device recorder.)
"""
import json
import os

import numpy as np

# Record.get_summary keys in the reference's order (record.py:110-134)
SUMMARY_KEYS = (
    "total rewards", "total served VMs", "total requests", "total cpu requested",
    "total memory requested", "total suspend actions", "total place actions", "average VM life",
    "average pending", "median pending", "max pending", "average slowdown", "median slowdown",
    "max slowdown", "drop rate", "cpu mean", "cpu mean target", "cpu std", "memory mean",
    "memory mean target", "memory std", "rank mean")
TRACE_KEYS = ("cpu", "memory", "used_pm", "vm_placements", "waiting_ratio", "actions", "rewards",
              "dropped_requests", "total_requests", "vm_arrival_steps", "target_cpu_mean",
              "target_memory_mean", "served_requests", "total_cpu_requested",
              "total_memory_requested", "suspended", "placed", "vmsratio", "rank")


class Record:
    """Per-step traces (same attributes as record.py:7-31) + the device summary."""

    def __init__(self, agent, env_config, agent_config):
        self.agent = agent
        self.env_config = env_config if isinstance(env_config, dict) else vars(env_config)
        self.agent_config = agent_config if isinstance(agent_config, dict) else None
        self.WAIT_STATUS = self.env_config["pms"]
        for k in TRACE_KEYS:
            setattr(self, k, [])
        self._device = None  # summary_from_device(...) of the recorded episode

    def set_device_summary(self, summary):
        """Attach the recorder's summary of the episode (Base.test does this)."""
        self._device = dict(summary)

    @property
    def device_summary(self):
        """summary_from_device's full dict (incl. the unrounded `_` columns)."""
        return self._device

    def get_summary(self):
        """record.py:110-134: same keys, same rounding; values from the device."""
        if self._device is None:
            raise RuntimeError("no recorded episode: run Base.test on the GPU env (the metrics "
                               "are accumulated on the device) or import a saved record")
        return {k: self._device[k] for k in SUMMARY_KEYS}

    def save(self, path: str):
        """record.py:136-142: vars(self) as JSON, incl. `summary`."""
        self.summary = self.get_summary()
        parent = os.path.dirname(path)
        if parent:
            os.makedirs(parent, exist_ok=True)
        out = {k: v for k, v in vars(self).items() if k != "_device"}
        with open(path, "w") as f:
            f.write(json.dumps(out, cls=NpEncoder))

    @classmethod
    def import_record(cls, agent: str, jsondict: dict):
        """record.py:144-168: the traces of a saved record, and its saved summary."""
        r = cls(agent, jsondict["env_config"], jsondict.get("agent_config"))
        for k in TRACE_KEYS:
            if k in jsondict:
                setattr(r, k, jsondict[k])
        if "summary" in jsondict:
            r.set_device_summary(jsondict["summary"])
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

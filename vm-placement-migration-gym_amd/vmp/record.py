"""Record (src/record.py:5-176) for the MI355X env.

The reference derives every evaluation metric on the host from per-step lists
(record.py:34-134: splitting each slot's placement history at its arrival
steps, then pending / slowdown / lifetime per VM life). Here those metrics are
accumulated on the device while the episode runs (vmp_record_enable /
vmp_record_read, csrc/vmp_record.hip) and `summary_from_device` turns the
recorder's sums and rate histograms into get_summary()'s dict. `Record` keeps
the reference's attribute names for the per-step traces Base.test appends, so
save() writes the JSON layout plots.ipynb and the exp_* drivers read, and its
summary is the device one.

A Record with no device summary (filled through record_testing_step by a
caller's own loop, or re-imported from JSON) derives the same metrics from its
traces on the host (`_life_table`: cumulative counts over the [step, slot]
placement matrix, evaluated at every life's bounds at once), and exposes the
reference's metric properties (pending_rates, slowdown_rates, vm_lifetime,
drop_rate, total_rewards, unique_vms_placement) on either path, as the
exp_* drivers read them (exp_performance.py:104-105, exp_suspension.py:56-59).
(tests/record_literal.py restates record.py literally and checks both.)
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

    def clear(self):
        """Drop the traces and the device summary (Base.test starts each episode
        with this, so a saved record holds one episode and its own summary)."""
        for k in TRACE_KEYS:
            setattr(self, k, [])
        self._device = None

    def set_device_summary(self, summary):
        """Attach the recorder's summary of the episode (Base.test does this)."""
        self._device = dict(summary)

    # ---- the reference's metric properties (record.py:33-108), host side ----
    def _lives(self):
        return _life_table(self.vm_placements, self.vm_arrival_steps, self.WAIT_STATUS)

    @property
    def unique_vms_placement(self):
        """record.py:33-51: each VM life's existing-state placements."""
        H = np.asarray(self.vm_placements)
        out = []
        for slot, lo, hi in zip(*_life_bounds(self.vm_arrival_steps, len(H))):
            col = H[lo:hi, slot]
            out.append(col[col <= self.WAIT_STATUS])
        return out

    @property
    def pending_rates(self):
        """record.py:54-66: (first running index + 1) / life length, 1.0 if none."""
        return _pending(*self._lives())

    @property
    def slowdown_rates(self):
        """record.py:68-83: waiting steps after the first run / remaining life."""
        return _slowdown(*self._lives())

    @property
    def vm_lifetime(self):
        """record.py:85-96: steps after the first run, 0 if the VM never ran."""
        return _lifetime(*self._lives())

    @property
    def drop_rate(self):
        """record.py:98-102: dropped / requested per step (0 where none)."""
        d = np.asarray(self.dropped_requests, dtype=float)
        t = np.asarray(self.total_requests, dtype=float)
        return np.divide(d, t, out=np.zeros(d.shape, dtype=float), where=t != 0)

    @property
    def total_rewards(self):
        """record.py:104-108: rewards below -1e7 replaced by the mean of those above."""
        if self._device is not None and not self.rewards:
            return self._device["total rewards"]
        r = np.array(self.rewards, dtype=float)
        low = r < -1e7
        if low.any():
            r[low] = r[r > -1e7].mean()
        return np.round(r.sum(), 3)

    def host_summary(self):
        """get_summary() (record.py:110-134) computed from the traces."""
        lives = self._lives()
        pend, slow, life = _pending(*lives), _slowdown(*lives), _lifetime(*lives)
        rnd = lambda x: np.round(x, 3)  # noqa: E731
        return {
            "total rewards": self.total_rewards,
            "total served VMs": self.served_requests[-1],
            "total requests": self.total_requests[-1],
            "total cpu requested": rnd(self.total_cpu_requested),
            "total memory requested": rnd(self.total_memory_requested),
            "total suspend actions": self.suspended[-1],
            "total place actions": self.placed[-1],
            "average VM life": rnd(np.mean(life)),
            "average pending": rnd(np.mean(pend)),
            "median pending": rnd(np.median(pend)),
            "max pending": rnd(np.max(pend)) if pend else 0,
            "average slowdown": rnd(np.mean(slow)),
            "median slowdown": rnd(np.median(slow)),
            "max slowdown": rnd(np.max(slow)),
            "drop rate": rnd(np.mean(self.drop_rate)),
            "cpu mean": rnd(np.mean(self.cpu)),
            "cpu mean target": rnd(np.mean(self.target_cpu_mean)),
            "cpu std": rnd(np.std(self.cpu)),
            "memory mean": rnd(np.mean(self.memory)),
            "memory mean target": rnd(np.mean(self.target_memory_mean)),
            "memory std": rnd(np.std(self.memory)),
            "rank mean": rnd(np.mean(self.rank)),
        }

    @property
    def device_summary(self):
        """summary_from_device's full dict (incl. the unrounded `_` columns)."""
        return self._device

    def get_summary(self):
        """record.py:110-134: same keys, same rounding; from the device recorder
        when Base.test attached its summary, else from the traces."""
        if self._device is not None:
            return {k: self._device[k] for k in SUMMARY_KEYS}
        if not self.vm_placements:
            raise RuntimeError("empty record: no device summary and no recorded steps")
        return self.host_summary()

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
        """record.py:144-168: the traces of a saved record; the summary is
        recomputed from them as the reference does (the saved `summary` is used
        only when the JSON holds no per-step traces)."""
        r = cls(agent, jsondict["env_config"], jsondict.get("agent_config"))
        for k in TRACE_KEYS:
            if k in jsondict:
                setattr(r, k, jsondict[k])
        if "summary" in jsondict and not r.vm_placements:
            r.set_device_summary(jsondict["summary"])
        return r


# Per-life metrics from _life_table's (n, f, w). The reference tests
# `if allocated_at:`, so a first run at index 0 counts as "never ran" (f <= 0).
def _pending(n, f, w):
    return [float(x) for x in np.where(f > 0, np.around((f + 1.0) / np.maximum(n, 1), 3), 1.0)]


def _slowdown(n, f, w):
    ran = f > 0
    rest = (n - f - 1)[ran]
    rates = np.where(rest == 0, 0.0, np.around(w[ran] / np.maximum(rest, 1), 3))
    return [float(x) for x in rates] if rates.size else [0]


def _lifetime(n, f, w):
    return [int(x) for x in np.where(f > 0, n - f - 1, 0)]


def _life_bounds(arrival_steps, n_steps):
    """(slot, lo, hi) of every VM life: the placement history is recorded from
    timestep 2, so the life that starts at arrival step a begins at row a - 2;
    a slot's first life starts at row 0 and its last ends at the last row."""
    slots, lo, hi = [], [], []
    for v, arr in enumerate(arrival_steps):
        if not arr:
            continue
        cuts = [0] + [int(a) - 2 for a in arr[1:]] + [n_steps]
        slots += [v] * (len(cuts) - 1)
        lo += cuts[:-1]
        hi += cuts[1:]
    return (np.asarray(slots, dtype=np.int64), np.asarray(lo, dtype=np.int64),
            np.asarray(hi, dtype=np.int64))


def _life_table(placements, arrival_steps, wait, chunk=256):
    """Per VM life: n = its existing-state entries (placement <= WAIT), f = the
    index among them of the first running entry (< WAIT; -1 if none) and w =
    the WAIT entries from that one on. Cumulative counts over the [step, slot]
    matrix, taken `chunk` slots at a time, are read at every life's bounds."""
    H = np.asarray(placements)
    T = H.shape[0]
    slots, lo, hi = _life_bounds(arrival_steps, T)
    n = np.zeros(slots.size, dtype=np.int64)
    f = np.full(slots.size, -1, dtype=np.int64)
    w = np.zeros(slots.size, dtype=np.int64)
    rows = np.arange(T + 1)[:, None]
    for c0 in range(0, H.shape[1], chunk):
        sel = (slots >= c0) & (slots < c0 + chunk)
        if not sel.any():
            continue
        blk = H[:, c0:c0 + chunk]
        zero = np.zeros((1, blk.shape[1]), dtype=np.int64)
        ex = np.concatenate([zero, np.cumsum(blk <= wait, axis=0)])
        wt = np.concatenate([zero, np.cumsum(blk == wait, axis=0)])
        # next running row at or after each row (T where none)
        run_at = np.where(blk < wait, rows[:-1], T)
        nxt = np.concatenate([np.minimum.accumulate(run_at[::-1], axis=0)[::-1],
                              np.full((1, blk.shape[1]), T)])
        s, a, b = slots[sel] - c0, lo[sel], hi[sel]
        n[sel] = ex[b, s] - ex[a, s]
        r0 = nxt[a, s]
        ran = r0 < b
        f[sel] = np.where(ran, ex[np.minimum(r0, T), s] - ex[a, s], -1)
        w[sel] = np.where(ran, wt[b, s] - wt[np.minimum(r0, T), s], 0)
    return n, f, w


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

"""Host restatement of the reference's Record metrics (src/record.py:34-134),
computed from the per-step traces Base.record_testing_step collects.

TEST INFRASTRUCTURE ONLY: the checker the device recorder (vmp_record_*,
csrc/vmp_record.hip) is compared against in tests/test_gpu_record.py. The
product's Record takes its summary from the device.

Semantics restated (record.py line numbers):
  lives      34-51   each slot's placement history (one row per step, recorded
                     from timestep 2) is cut at its arrival steps after the
                     first (cut index = arrival - 2); a life keeps the entries
                     <= WAIT (existing VM states)
  first run          index of the first entry < WAIT; an index of 0 counts as
                     "never ran" (the reference tests `if allocated_at:`)
  pending    53-65   round((first + 1) / len, 3), else 1.0
  slowdown   67-82   lives that ran: round(#WAIT after first / (len - first - 1), 3),
                     0 when that length is 0; [0] when no life ran
  lifetime   84-95   len - first - 1, else 0
  drop rate  97-101  dropped / total per step (0 where total is 0)
  rewards    103-108 values < -1e7 replaced by the mean of those > -1e7
  summary    110-134 keys and rounding of get_summary
"""
import numpy as np


def lives(placements, arrival_steps, wait):
    hist = np.asarray(placements).T  # [slot, step]
    out = []
    for slot, row in enumerate(hist):
        arr = arrival_steps[slot]
        if not arr:
            continue
        cuts = [a - 2 for a in arr[1:]]
        bounds = [0] + cuts + [len(row)]
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            seg = row[lo:hi]
            out.append(seg[seg <= wait])
        assert out[-1].size, "the open life of a slot has no existing-VM entry"
    return out


def _first_run(seg, wait):
    idx = np.flatnonzero(seg < wait)
    return int(idx[0]) if idx.size and idx[0] != 0 else None


def life_metrics(segs, wait):
    pend, slow, life = [], [], []
    for seg in segs:
        f = _first_run(seg, wait)
        if f is None:
            pend.append(1.0)
            life.append(0)
            continue
        pend.append(np.around((f + 1.0) / len(seg), 3))
        n = len(seg) - f - 1
        life.append(n)
        slow.append(0 if n == 0 else np.around(np.count_nonzero(seg[f:] == wait) / n, 3))
    return pend, (slow or [0]), life


def summary(traces, wait):
    """traces: dict of the Record trace lists -> get_summary()'s dict."""
    pend, slow, life = life_metrics(lives(traces["vm_placements"], traces["vm_arrival_steps"],
                                          wait), wait)
    r = np.array(traces["rewards"], dtype=float)
    r[r < -1e7] = np.mean(r[r > -1e7])
    d, t = np.array(traces["dropped_requests"]), np.array(traces["total_requests"])
    drop = np.divide(d, t, out=np.zeros(d.shape, dtype=float), where=t != 0)
    rnd = lambda x: np.round(x, 3)  # noqa: E731
    return {
        "total rewards": rnd(np.sum(r)),
        "total served VMs": traces["served_requests"][-1],
        "total requests": traces["total_requests"][-1],
        "total cpu requested": rnd(traces["total_cpu_requested"]),
        "total memory requested": rnd(traces["total_memory_requested"]),
        "total suspend actions": traces["suspended"][-1],
        "total place actions": traces["placed"][-1],
        "average VM life": rnd(np.mean(life)),
        "average pending": rnd(np.mean(pend)),
        "median pending": rnd(np.median(pend)),
        "max pending": rnd(np.max(pend)) if pend else 0,
        "average slowdown": rnd(np.mean(slow)),
        "median slowdown": rnd(np.median(slow)),
        "max slowdown": rnd(np.max(slow)),
        "drop rate": rnd(np.mean(drop)),
        "cpu mean": rnd(np.mean(traces["cpu"])),
        "cpu mean target": rnd(np.mean(traces["target_cpu_mean"])),
        "cpu std": rnd(np.std(traces["cpu"])),
        "memory mean": rnd(np.mean(traces["memory"])),
        "memory mean target": rnd(np.mean(traces["target_memory_mean"])),
        "memory std": rnd(np.std(traces["memory"])),
        "rank mean": rnd(np.mean(traces["rank"])),
    }

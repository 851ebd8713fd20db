"""Record's host path (vmp.record: no device summary attached) against the
literal restatement of src/record.py:33-134 (tests/record_literal.py), on
synthetic traces: per slot a sequence of VM lives (NULL until the arrival,
WAIT, running on some PM, suspensions back to WAIT, NULL after the finish),
including the reference's `if allocated_at:` quirk (a life whose first entry
is running counts as never run). Also the metric properties the exp_*
drivers read (exp_performance.py:104-105, exp_suspension.py:56-59) and a
save -> import_record -> get_summary round trip (record.py:136-168)."""
import json

import numpy as np
import pytest

from tests import record_literal
from vmp.record import Record


def _synthetic(seed, T=400, V=23, P=7):
    g = np.random.default_rng(seed)
    WAIT, NULL = P, P + 1
    H = np.full((T, V), NULL, dtype=np.int64)
    arrivals = []
    for v in range(V):
        arr = []
        r = int(g.integers(0, 40))
        while r < T:
            arr.append(r + 2)  # rows are recorded from timestep 2
            n_wait = int(g.integers(0 if g.random() < 0.1 else 1, 12))  # 0: runs at once (quirk)
            life = [WAIT] * n_wait
            for _ in range(int(g.integers(0, 4))):
                pm = int(g.integers(0, P))
                life += [pm] * int(g.integers(1, 30))
                if g.random() < 0.5:
                    life += [WAIT] * int(g.integers(1, 6))  # suspended
            if not life:
                life = [WAIT]
            end = min(T, r + len(life))
            H[r:end, v] = life[:end - r]
            r = end + int(g.integers(0, 25))  # NULL until the next arrival
        arrivals.append(arr)
    dropped = g.integers(0, 3, size=T).cumsum()
    total = dropped + g.integers(0, 5, size=T).cumsum()
    rewards = -g.random(T)
    rewards[g.random(T) < 0.02] = -1e7 - 1.0  # replaced by the mean (record.py:104-108)
    return dict(
        cpu=g.random((T, P)).tolist(), memory=g.random((T, P)).tolist(), used_pm=[0] * T,
        vm_placements=H.tolist(), waiting_ratio=g.random(T).tolist(), actions=H.tolist(),
        rewards=rewards.tolist(), dropped_requests=dropped.tolist(),
        total_requests=total.tolist(), vm_arrival_steps=arrivals,
        target_cpu_mean=g.random(T).tolist(), target_memory_mean=g.random(T).tolist(),
        served_requests=list(range(T)), total_cpu_requested=123.4567,
        total_memory_requested=98.7654, suspended=list(range(T)), placed=list(range(T)),
        vmsratio=[], rank=g.integers(0, P, size=T).tolist()), P


def _record(tr, P):
    r = Record("HostLoop", dict(pms=P, vms=len(tr["vm_arrival_steps"])), None)
    for k, v in tr.items():
        setattr(r, k, v)
    return r


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_host_summary_equals_literal_record(seed):
    tr, P = _synthetic(seed)
    rec = _record(tr, P)
    got, lit = rec.get_summary(), record_literal.summary(tr, P)
    assert list(got) == list(lit)
    for k, v in lit.items():
        assert got[k] == v, (k, got[k], v)
    pend, slow, life = record_literal.life_metrics(
        record_literal.lives(tr["vm_placements"], tr["vm_arrival_steps"], P), P)
    assert rec.pending_rates == [float(x) for x in pend]
    assert rec.slowdown_rates == [float(x) for x in slow]
    assert rec.vm_lifetime == [int(x) for x in life]
    segs = record_literal.lives(tr["vm_placements"], tr["vm_arrival_steps"], P)
    assert len(rec.unique_vms_placement) == len(segs)
    for a, b in zip(rec.unique_vms_placement, segs):
        assert np.array_equal(a, b)
    d, t = np.array(tr["dropped_requests"]), np.array(tr["total_requests"])
    assert np.array_equal(rec.drop_rate, np.divide(d, t, out=np.zeros(d.shape), where=t != 0))
    assert any(f == 1.0 for f in rec.pending_rates)  # lives that never ran (incl. the quirk)


def test_saved_host_record_reimports(tmp_path):
    tr, P = _synthetic(5)
    rec = _record(tr, P)
    rec.save(str(tmp_path / "r.json"))
    back = Record.import_record("HostLoop", json.load(open(tmp_path / "r.json")))
    assert back.get_summary() == json.loads(json.dumps(rec.get_summary(), default=float))
    assert back.total_rewards == rec.total_rewards


def test_empty_record_raises():
    with pytest.raises(RuntimeError):
        Record("x", dict(pms=3, vms=4), None).get_summary()

"""Run the heuristic rows of the reference's published experiment summaries
(data/exp_performance/summary.csv, exp_performance_small, exp_vm_size) through
vmp.exp on the GPU and print our rows; the expected rows live in
tests/golden/exp_published.json.

Usage: python tools/exp_published.py [--which performance,performance_small,vm_size]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="performance,performance_small,vm_size")
    ap.add_argument("--eval-steps", type=int, default=None)
    a = ap.parse_args()
    from vmp import exp
    for which in a.which.split(","):
        t0 = time.time()
        if which == "performance":
            # the published load-1.0 rows' Return is the wr return (their other
            # columns do not depend on the reward), the load-0.6 rows' the ut one
            cells = [exp.performance_cell(ag, ag, ld, "wr" if ld == 1.0 else "ut")
                     for ld in (1.0, 0.6) for ag in ("bestfit", "firstfit")]
            rows = exp.performance_sweep(cells, eval_steps=a.eval_steps)
        elif which == "performance_small":
            cells = [exp.performance_cell(ag, ag, 1.0, small=True) for ag in ("bestfit", "firstfit")]
            rows = exp.performance_sweep(cells, eval_steps=a.eval_steps)
        else:
            cells = [exp.vm_size_cell(ag, seq) for seq in ("lowuniform", "highuniform")
                     for ag in ("firstfit", "bestfit")]
            rows = exp.vm_size_sweep(cells, eval_steps=a.eval_steps)
        print("==", which, "%.1f s" % (time.time() - t0), flush=True)
        for r in rows:
            print(r, flush=True)


if __name__ == "__main__":
    main()

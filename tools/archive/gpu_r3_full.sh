#!/bin/bash
# Round-3 checkpoint: whole -m gpu suite, smoke(), default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-full}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
python - $O/bench.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("headline", round(d["value"] / 1e6, 2), "M/s", "kernel_ms", round(r["kernel_ms"], 4), "frac", round(r["frac"], 4), "B/step", round(r["bytes_per_env_step"]))
for k in ("period", "nominal_load", "external_actions", "stress_p1000_v10000", "stress_p1000_v10000_2048envs"):
    x = d.get(k) or {}
    rr = x.get("roofline", {})
    print(k, {kk: x.get(kk) for kk in ("value", "mean_ms", "kernel_ms", "max_ms", "error")}, "frac", rr.get("frac"))
for k in ("ppo_train", "ppo_train_bf16", "ppo_eval", "fused_rollout", "parity", "cpu_baseline"):
    print(k, str(d.get(k))[:300])
PY

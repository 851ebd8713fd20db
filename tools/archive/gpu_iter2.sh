#!/bin/bash
# Round-2 iteration: env + record parity suites, then the bench (no CPU leg).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_record.py ${EXTRA_TESTS:-} -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
r = d["roofline"]
print("headline", round(d["value"] / 1e6, 2), "M/s kern_ms", round(r["kernel_ms"], 4), "frac", round(r["frac"], 4), "B", round(r["bytes_per_env_step"]), "words", r.get("vm_words_written_per_env_step"))
print("parity", d["parity"])
for k in ("external_actions", "stress_p1000_v10000", "fused_rollout", "ppo_train", "ppo_train_bf16", "ppo_eval"):
    x = d.get(k)
    if isinstance(x, dict):
        print(k, {kk: (round(v, 4) if isinstance(v, float) else v) for kk, v in x.items() if kk in ("value", "kernel_ms", "bytes_per_env_step", "vm_words_written_per_env_step", "mean_running", "mean_waiting", "s_per_update", "error")}, x.get("roofline", {}).get("frac"))
PY
exit 0

#!/bin/bash
# Round-5 GPU steps, one gpurun call: tools/gpu_r5.sh OUT STEP [STEP ...]
#   tests      the whole -m gpu suite
#   t:EXPR     pytest -m gpu -k EXPR
#   smoke      __graft_entry__.smoke()
#   bench      the driver's default bench line (bench.py --gpus 1 --steps 20 --warmup 5)
#   headline   bench.py headline leg only (no PPO / C5 / period legs)
#   ppo16      tools/bench_ppo.py bf16, 8192 envs, 3 updates
#   counters   rocprofv3 -L (the counters this box offers)
# Every step has its own time limit; the first failing step ends the call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:?out dir}; shift; mkdir -p $O
for s in "$@"; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
           rc=$?; tail -1 $O/gpu_tests.log; [ $rc -ne 0 ] && grep -E "FAILED|Error" $O/gpu_tests.log | head -20 ;;
    t:*) k=${s#t:}; timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$k" --timeout 400 --timeout-method thread > $O/t_${k//[^a-zA-Z0-9]/_}.log 2>&1
         rc=$?; tail -1 $O/t_${k//[^a-zA-Z0-9]/_}.log; [ $rc -ne 0 ] && grep -E "FAILED|Error|assert" $O/t_${k//[^a-zA-Z0-9]/_}.log | head -20 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log ;;
    bench) timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1; rc=$?
           grep -v amdgpu.ids $O/bench.log | tail -1 | cut -c1-400 ;;
    headline) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-ppo --period-steps 0 --nominal-steps 0 --no-cpu > $O/headline.log 2>&1; rc=$?
           grep -v amdgpu.ids $O/headline.log | tail -1 | cut -c1-400 ;;
    ppo16) timeout -k 10 300 python tools/bench_ppo.py --precision bf16 --envs 8192 --updates 3 --warmup 1 > $O/ppo_bf16.log 2>&1; rc=$?
           tail -1 $O/ppo_bf16.log | cut -c1-800 ;;
    ppo16s) timeout -k 10 300 python tools/bench_ppo.py --precision bf16 --envs 8192 --updates 3 --warmup 1 --lookahead 0 > $O/ppo_bf16_sync.log 2>&1; rc=$?
           tail -1 $O/ppo_bf16_sync.log | cut -c1-800 ;;
    dwaug) timeout -k 10 120 python tools/bench_dw_aug.py > $O/dwaug.log 2>&1; rc=$?; tail -1 $O/dwaug.log ;;
    hgbench) FWD_ONLY=1 timeout -k 10 300 python tools/bench_actor_head_bf16.py > $O/hgbench.log 2>&1; rc=$?; tail -1 $O/hgbench.log ;;
    timeline) timeout -k 10 300 python tools/update_timeline.py > $O/timeline.log 2>&1; rc=$?; tail -c 600 $O/timeline.log ;;
    hostprof) timeout -k 10 300 python tools/host_prof_values.py > $O/hostprof.log 2>&1; rc=$?; grep -E "get_value|tottime" $O/hostprof.log ;;
    counters) timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1; rc=$? ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  echo "step $s rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0

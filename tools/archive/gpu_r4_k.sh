#!/bin/bash
# Round 4: persistent heavy-first per-step launches: their parity tests, the
# -m gpu suite, smoke, the driver's bench line, then an A/B of the headline and
# period legs with the order off (VMP_LPT=0) and on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4k}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lpt.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/lpt_tests.log 2>&1
rc=$?; echo "lpt_tests_rc=$rc"; tail -3 $O/lpt_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/lpt_tests.log | head; exit $rc; }
bash tools/gpu_r4_final_a.sh ${1:-r4k} || exit 1
ARGS="--no-cpu --no-ppo --ext-steps 0 --nominal-steps 0 --stress-steps 0 --steps 20 --warmup 5"
for l in 0 1 0 1; do
  VMP_LPT=$l timeout -k 10 300 python bench.py $ARGS > $O/ab_lpt$l.log 2>&1
  rc=$?; echo "ab lpt=$l rc=$rc"; tail -1 $O/ab_lpt$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lpt', '$l', d['ms_per_step'], d['roofline']['kernel_ms'], d.get('period',{}).get('mean_ms'), d.get('period',{}).get('ms_by_100_steps'))"; [ $rc -ne 0 ] && exit $rc
done
exit 0

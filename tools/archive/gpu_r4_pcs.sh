#!/bin/bash
# Host-trap PC sampling of the headline step kernel (k_env<16, true>, training
# mode as bench.py): where the waves' time goes, per instruction.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4pcs}; mkdir -p $O
PROF_EVAL=0 PROF_STEPS=${PCS_STEPS:-200} timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
  --pc-sampling-unit time --pc-sampling-interval ${PCS_INTERVAL:-1} --kernel-trace \
  --output-format csv -d $O/pcs -o run -- python tools/prof_step.py > $O/pcs.log 2>&1
rc=$?; echo "pcs rc=$rc"; tail -3 $O/pcs.log | cut -c1-300; ls -la $O/pcs/ 2>/dev/null | head
find $O/pcs -name "*.csv" -size +50M -exec gzip {} \;
exit $rc

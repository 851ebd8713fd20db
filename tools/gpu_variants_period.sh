#!/bin/bash
# Period-leg timing (bench.py --period-only: 1000 launches of phase-aligned
# envs from step 2001) of each library variant in $VARIANTS
# (vm-placement-migration-gym_amd/build/variants/libvmp_<v>.so), twice each,
# interleaved, on one box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/var
for rep in 1 2; do
  for v in ${VARIANTS}; do
    VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_$v.so \
      timeout -k 10 200 python bench.py --period-only --no-cpu --period-ff ${PFF:-2000} > gpurun_out/var/p_${v}_$rep.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/var/p_${v}_$rep.log').read().strip().splitlines()[-1])['period']; print('$v rep$rep mean', round(d['mean_ms'],4), 'max', round(d['max_ms'],4), 'bins', d['ms_by_100_steps'])"
  done
done

set -o pipefail
O=gpurun_out/${1:-res}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_actor_head_bf16.py -k "resident" > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VARS="default hggo hggo@VMP_HG16_RES=1@VMP_HG16_STAG=1 hggo@VMP_HG16_RES=1@VMP_HG16_STAG=4 hggo@VMP_HG16_RES=1@VMP_HG16_STAG=8 default@VMP_HG16_RES=1@VMP_HG16_STAG=4" REPS=1 bash tools/gpu_hgvar.sh ${1:-res}

# Usage: bash tools/gpu_r4e.sh -- the GPU suite on the fused BN finalize build, then A/Bs: fused finalize on / off
# (Res10 bench + kernel traces), the heads' weight gradient after the deconv BN apply, the narrow 1x1 ring routing
# on Res50 1024^2 fp16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf -s tests > $O/r4e_tests.log 2>&1
rc=$?; tail -3 $O/r4e_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_ab2.sh fin SCD_BN_FIN_FUSE=0 SCD_BN_FIN_FUSE=1 || exit 1
bash tools/gpu_ab2.sh hwafter SCD_HEADS_WGRAD_AFTER_BN=0 SCD_HEADS_WGRAD_AFTER_BN=1 || exit 1
for i in 1 2; do
  for E in SCD_GEMM_NARROW_RING=0 SCD_GEMM_NARROW_RING=1; do
    env $E timeout -k 10 300 python bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --steps 10 --warmup 3 --no-cpu-baseline > $O/r4e_res50_${E}_$i.json 2>> $O/r4e_res50.err || exit 1
    python -c "import json; d=json.load(open('$O/r4e_res50_${E}_$i.json')); print('$E', d['value'], d['ms_per_step'])"
  done
done
echo r4e done

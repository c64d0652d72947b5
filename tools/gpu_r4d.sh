# Usage: bash tools/gpu_r4d.sh -- tests touched by the narrow-ring routing and the heads K order, then A/Bs:
# the heads' weight gradient after the deconv BN apply (Res10), the narrow 1x1 ring routing (Res50 1024^2 fp16)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf -s tests/test_kernels_gpu.py tests/test_sparse_heads_gpu.py tests/test_model_gpu.py -k "serpentine or conv_fwd_dgrad_wgrad or dgrad_with_bn or sparse or f3 or bn_backward_sums" > $O/r4d_tests.log 2>&1
rc=$?; tail -3 $O/r4d_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_ab2.sh hwafter SCD_HEADS_WGRAD_AFTER_BN=0 SCD_HEADS_WGRAD_AFTER_BN=1 || exit 1
for i in 1 2; do
  for E in SCD_GEMM_NARROW_RING=0 SCD_GEMM_NARROW_RING=1; do
    env $E timeout -k 10 300 python bench.py --model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --steps 10 --warmup 3 --no-cpu-baseline > $O/r4d_res50_${E}_$i.json 2>> $O/r4d_res50.err || exit 1
    python -c "import json; d=json.load(open('$O/r4d_res50_${E}_$i.json')); print('$E', d['value'], d['ms_per_step'])"
  done
done
echo r4d done

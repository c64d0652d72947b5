# Usage: bash tools/gpu_r4o.sh -- configs[4] (Res50 1024^2 B=16 fp16): narrow 1x1 convs on the ring kernel or the
# register-staged 256 x 64 kernel, re-measured on the fixed ring kernel (the first A/B ran on the regressed build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
BENCH_ARGS="--model centerOffsetRes50 --image-size 1024 --batch 16 --dtype fp16 --steps 8 --warmup 3" bash tools/gpu_abn.sh nring "SCD_GEMM_NARROW_RING=0" "SCD_GEMM_NARROW_RING=1" || exit 1
echo r4o done

# Usage: bash tools/gpu_ab_lib.sh <tag> <libA> <libB> [bench args] -- A/B of two builds of libscdhip on one box
# (SCDHIP_LIB), alternating A B A B, then the GPU test suite on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out
for i in 1 2; do
  for L in $A $B; do
    SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/$L timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab_${TAG}_${L}_$i.json 2>> gpurun_out/ab_${TAG}.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_${L}_$i.json')); print('$L', d['value'], d['ms_per_step'])"
  done
done

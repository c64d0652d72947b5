# Usage: bash tools/gpu_ab_env.sh <tag> "<env A>" "<env B>" [bench args] -- A/B of two environment settings of the
# same build on one box (e.g. "SCD_STEM_FUSED_BWD=0" "SCD_STEM_FUSED_BWD=1"), alternating A B A B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out
for i in 1 2; do
  k=0
  for E in "$A" "$B"; do
    k=$((k+1))
    env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/abe_${TAG}_${k}_$i.json 2>> gpurun_out/abe_${TAG}.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/abe_${TAG}_${k}_$i.json')); print('$E', d['value'], d['ms_per_step'])"
  done
done

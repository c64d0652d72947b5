# Usage: bash tools/gpu_ab_envs.sh <tag> "<env 1>" "<env 2>" ... -- bench of several environment settings of the
# same build on one box, two alternating rounds (use "X=0" for the default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
for i in 1 2; do
  k=0
  for E in "$@"; do
    k=$((k+1))
    env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/abm_${TAG}_${k}_$i.json 2>> gpurun_out/abm_${TAG}.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/abm_${TAG}_${k}_$i.json')); print('$E', d['value'], d['ms_per_step'])"
  done
done

# Usage: bash tools/gpu_ab_env.sh <tag> "<ENV=val ...>" "<ENV=val ...>" -- alternating bench A/B (x2) of two env settings
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; A=$2; B=$3
mkdir -p gpurun_out
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/ab_${TAG}_${v}$r.json 2> gpurun_out/ab_${TAG}_${v}$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${v}$r.json')); print('$v [$E]', d['value'], d['ms_per_step'])"
  done
done

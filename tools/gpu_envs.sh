# Usage: bash tools/gpu_envs.sh <tag> "<env A>" "<env B>" ... -- one bench line per env setting, twice, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out
for r in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/envs_${TAG}_${i}_$r.json 2> gpurun_out/envs_${TAG}_${i}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/envs_${TAG}_${i}_$r.json')); print('[$E]', d['value'], d['ms_per_step'])"
  done
done

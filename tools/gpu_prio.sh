# Usage: bash tools/gpu_prio.sh <tag> -- bench with and without the high-priority step stream
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-prio}
mkdir -p gpurun_out
for v in 0 1 0 1; do
  SCD_STEP_PRIORITY=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/prio_${TAG}_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/prio_${TAG}_$v.json')); print('prio=$v', d['value'], d['ms_per_step'])"
done

# Usage: bash tools/gpu_fuse.sh <tag>  -- all GPU tests, then the step bench with BN-sum fusion off (A) / on (B)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-f}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  SCD_BN_FUSE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
  echo "fuse=$v $(python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['final_loss'])")"
done

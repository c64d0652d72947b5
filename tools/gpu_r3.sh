# Usage: bash tools/gpu_r3.sh <tag> [notests] -- GPU test suite, then bench (no CPU baseline) and kernel stats of it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r}
mkdir -p gpurun_out
if [ "$2" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
  tail -4 gpurun_out/tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cut -c1-260 gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/profbench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit 1
python tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/ksum_$TAG.txt 2>&1
head -30 gpurun_out/ksum_$TAG.txt

# Usage: bash tools/gpu_all.sh <tag>   -- GPU tests, bench and a rocprofv3 kernel-stat profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/profbench_$TAG.json 2> gpurun_out/prof_$TAG.err; rc=$?
find gpurun_out/prof_$TAG -name "*.csv" | head
exit $rc

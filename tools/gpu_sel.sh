# Usage: TESTS="<pytest args>" bash tools/gpu_sel.sh <tag> [prof]  -- selected GPU tests, the bench, and (with
# "prof") a rocprofv3 kernel trace of a short bench run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-sel}
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > gpurun_out/tests_$TAG.log 2>&1; rc=$?
  tail -15 gpurun_out/tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?
cut -c1-330 gpurun_out/bench_$TAG.json; tail -2 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
if [ "$2" = "prof" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > gpurun_out/profbench_$TAG.json 2> gpurun_out/prof_$TAG.err; rc=$?
fi
exit $rc

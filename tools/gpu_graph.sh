# Usage: bash tools/gpu_graph.sh <tag> -- step-graph tests, then the bench with and without the graph
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-g}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_gpu.py \
    tests/test_kernels_gpu.py -k "graph or adam" > gpurun_out/graph_tests_$TAG.log 2>&1; rc=$?
tail -15 gpurun_out/graph_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_graph_$TAG.json 2> gpurun_out/bench_graph_$TAG.err; rc=$?
cat gpurun_out/bench_graph_$TAG.json; tail -3 gpurun_out/bench_graph_$TAG.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --eager > gpurun_out/bench_eager_$TAG.json 2> gpurun_out/bench_eager_$TAG.err; rc=$?
cat gpurun_out/bench_eager_$TAG.json
exit $rc

# Usage: bash tools/gpu_step.sh <tag> [notests] -- GPU test suite, A/B bench of libscdhip_base.so vs the build,
# kernel trace + step timeline of the build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-s}
mkdir -p gpurun_out
if [ "$2" != "notests" ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/tall_$TAG.log 2>&1; rc=$?
  tail -2 gpurun_out/tall_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$ABENV" ]; then bash tools/gpu_ab_env.sh $TAG "$ABENV=0" "$ABENV=1" || exit 1; else bash tools/gpu_ab_lib.sh $TAG libscdhip_base.so libscdhip.so || exit 1; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/profbench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit 1
python tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/ksum_$TAG.txt 2>&1
python tools/step_timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/tl_$TAG.txt 2>&1
tail -3 gpurun_out/tl_$TAG.txt

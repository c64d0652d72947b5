# Usage: bash tools/gpu_halo.sh <tag> -- layer1 kernel tests, A/B bench of libscdhip_base.so vs the build, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-h}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "l1p or layer1 or bn_backward or dgrad_with_bn" > gpurun_out/tk_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/tk_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_lib.sh $TAG libscdhip_base.so libscdhip.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/profbench_$TAG.json 2> gpurun_out/prof_$TAG.err || exit 1
python tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/ksum_$TAG.txt 2>&1
python tools/step_timeline.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/tl_$TAG.txt 2>&1
tail -3 gpurun_out/tl_$TAG.txt

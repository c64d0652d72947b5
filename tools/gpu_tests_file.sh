# Usage: bash tools/gpu_tests_file.sh <tag> <pytest args...> -- selected GPU tests with output (-s)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-t}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -60 gpurun_out/tests_$TAG.log
exit $rc

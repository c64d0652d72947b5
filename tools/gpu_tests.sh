# Usage: bash tools/gpu_tests.sh <tag> [pytest args]  -- GPU test suite only
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-t}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu "$@" > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -40 gpurun_out/tests_$TAG.log
exit $rc

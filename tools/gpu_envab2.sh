# Usage: bash tools/gpu_envab2.sh <tag> <ENVVAR> <pytest targets|-> [bench args...] -- GPU tests (default env), then two
# interleaved rounds of bench.py with ENVVAR=0 and ENVVAR=1
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift; VAR=$1; shift; TGT=$1; shift
mkdir -p gpurun_out
if [ "$TGT" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $TGT -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/eabt_$TAG.log 2>&1; rc=$?
  tail -3 gpurun_out/eabt_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for v in 0 1; do
    echo "== $VAR=$v ($r) $*"
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | cut -c1-170 || exit 1
  done
done

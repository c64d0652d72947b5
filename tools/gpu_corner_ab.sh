# Usage: bash tools/gpu_corner_ab.sh <tag> -- cornerNetCPool: shared input gradient on / off (SCD_SHARED_GRAD), two rounds,
# then a rocprofv3 kernel trace of the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cab}
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1; do
    echo "== SCD_SHARED_GRAD=$v ($r)"
    SCD_SHARED_GRAD=$v timeout -k 10 300 python bench.py --model cornerNetCPool --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof_$TAG -o run -- python3 bench.py --model cornerNetCPool --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cprofbench_$TAG.json 2> gpurun_out/cprof_$TAG.err || exit 1
echo ok

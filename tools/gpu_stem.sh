# Usage: bash tools/gpu_stem.sh <tag> -- stem kernel timings + per-kernel PMC (instruction mix, waits) of the same run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-stem}
mkdir -p gpurun_out
timeout -k 10 120 python tools/stem_bench.py > gpurun_out/stem_$TAG.txt 2>&1; rc=$?
cat gpurun_out/stem_$TAG.txt
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/stempmc_$TAG -o run -- python3 tools/stem_bench.py --reps 2 > /dev/null 2>&1; rc=$?
exit $rc

# Usage: bash tools/gpu_ablib.sh <tag> <pytest target|-> <variant libs...>  -- optional GPU tests on the main library,
# then dgrad_bench and two interleaved bench runs per library (main + each scdhip/libscdhip_<variant>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift; TGT=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.txt
: > $OUT
if [ "$TGT" != "-" ]; then
  timeout -k 10 500 python -u -m pytest $TGT -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abt_$TAG.log 2>&1; rc=$?
  tail -3 gpurun_out/abt_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for v in base "$@"; do
  if [ "$v" = base ]; then LIBP=scd-resnet_amd/scdhip/libscdhip.so; else LIBP=scd-resnet_amd/scdhip/libscdhip_$v.so; fi
  echo "== dgrad $v" >> $OUT
  SCDHIP_LIB=$LIBP timeout -k 10 120 python tools/dgrad_bench.py >> $OUT 2>/dev/null || exit 1
done
for round in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then LIBP=scd-resnet_amd/scdhip/libscdhip.so; else LIBP=scd-resnet_amd/scdhip/libscdhip_$v.so; fi
    echo "== bench $v ($round)" >> $OUT
    SCDHIP_LIB=$LIBP timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-190 >> $OUT || exit 1
  done
done
cat $OUT

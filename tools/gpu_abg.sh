# Usage: bash tools/gpu_abg.sh <tag> <pytest targets|-> <gemm_bench --only filter> <variant libs...> -- GPU tests on the main
# library, then gemm_bench rows and two interleaved bench runs per library (main = "base", + scdhip/libscdhip_<v>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift; TGT=$1; shift; ONLY=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/abg_$TAG.txt
: > $OUT
if [ "$TGT" != "-" ]; then
  timeout -k 10 500 python -u -m pytest $TGT -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abgt_$TAG.log 2>&1; rc=$?
  tail -3 gpurun_out/abgt_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
lib() { if [ "$1" = base ]; then echo scd-resnet_amd/scdhip/libscdhip.so; else echo scd-resnet_amd/scdhip/libscdhip_$1.so; fi; }
for v in base "$@"; do
  echo "== gemm $v" >> $OUT
  SCDHIP_LIB=$(lib $v) timeout -k 10 120 python tools/gemm_bench.py --only "$ONLY" 2>/dev/null >> $OUT || exit 1
done
for round in 1 2; do
  for v in base "$@"; do
    echo "== bench $v ($round)" >> $OUT
    SCDHIP_LIB=$(lib $v) timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-190 >> $OUT || exit 1
  done
done
cat $OUT

# Usage: bash tools/gpu_cachepol.sh <tag> <variant libs...> -- heads GEMM rows, in-step bench and PMC traffic of the
# heads kernel per variant library (cache-policy experiments), plus the BN-backward dgrad shapes (PP on / off)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/cp_$TAG.txt
: > $OUT
timeout -k 10 120 python tools/dgrad_bench.py >> $OUT 2>&1 || exit 1
SCD_GEMM_PP=0 timeout -k 10 120 python tools/dgrad_bench.py >> $OUT 2>&1 || exit 1
bash tools/gpu_variants.sh heads 20 "$@" >> $OUT 2>&1 || exit 1
for v in base "$@"; do
  if [ "$v" = base ]; then LIBP=scd-resnet_amd/scdhip/libscdhip.so; else LIBP=scd-resnet_amd/scdhip/libscdhip_$v.so; fi
  echo "== bench $v" >> $OUT
  SCDHIP_LIB=$LIBP timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $OUT 2>/dev/null || exit 1
done
for v in base "$@"; do
  if [ "$v" = base ]; then LIBP=scd-resnet_amd/scdhip/libscdhip.so; else LIBP=scd-resnet_amd/scdhip/libscdhip_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    SCDHIP_LIB=$LIBP timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/cp_${TAG}_${v}_$c -o run -- python3 tools/gemm_bench.py --only heads --reps 3 > /dev/null 2>&1 || exit 1
  done
done
echo done >> $OUT

# Usage: bash tools/gpu_abn.sh <tag> "<cfg 1>" "<cfg 2>" ... -- A/B/C... on one box: each cfg is a list of
# environment settings ("X=1 Y=0"; a word ending in .so is a library under scdhip/, loaded through SCDHIP_LIB),
# run round-robin twice (Res10 bench line: img/s, ms/step), then one rocprofv3 kernel trace of each with its kernel
# summary: gpurun_out/abn_<tag>_<i>_kernel_summary.txt.  BENCH_ARGS (environment): other bench arguments, e.g. another
# model / size, with its own step counts (default --steps 30 --warmup 5; the traces take --steps 10 --warmup 3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out
mkdir -p $O
envof() { for w in $1; do case "$w" in *.so) echo -n "SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/$w " ;; *) echo -n "$w " ;; esac; done; }
for i in 1 2; do
  k=0
  for c in "$@"; do
    k=$((k+1))
    env $(envof "$c") timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 30 --warmup 5} --no-cpu-baseline --no-calib > $O/abn_${TAG}_${k}_$i.json 2>> $O/abn_${TAG}.err || exit 1
    python -c "import json; d=json.load(open('$O/abn_${TAG}_${k}_$i.json')); print('$k [$c]', d['value'], d['ms_per_step'])"
  done
done
k=0
for c in "$@"; do
  k=$((k+1))
  env $(envof "$c") timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/abn_${TAG}_${k}_prof -o run -- python3 bench.py ${BENCH_ARGS:---steps 10 --warmup 3} --no-cpu-baseline --no-calib > /dev/null 2>> $O/abn_${TAG}.err || exit 1
  python tools/prof_summary.py $O/abn_${TAG}_${k}_prof/run_kernel_trace.csv $O/abn_${TAG}_${k}_kernel_stats.csv > $O/abn_${TAG}_${k}_kernel_summary.txt 2>&1
  python tools/step_timeline.py $O/abn_${TAG}_${k}_prof/run_kernel_trace.csv > $O/abn_${TAG}_${k}_step_timeline.txt 2>&1
  rm -rf $O/abn_${TAG}_${k}_prof
done
echo abn done

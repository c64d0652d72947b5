# Usage: bash tools/gpu_benchrr.sh <tag> "<cfg 1>" "<cfg 2>" ... -- bench lines only (no profiler), each setting run
# round-robin three times; a cfg is a list of environment settings (BENCH_ARGS: other bench arguments)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out
mkdir -p $O
for i in 1 2 3; do
  k=0
  for c in "$@"; do
    k=$((k+1))
    env $c timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 30 --warmup 5} --no-cpu-baseline > $O/rr_${TAG}_${k}_$i.json 2>> $O/rr_${TAG}.err || exit 1
    python -c "import json; d=json.load(open('$O/rr_${TAG}_${k}_$i.json')); print('$k [$c]', d['value'], d['ms_per_step'])"
  done
done
echo rr done

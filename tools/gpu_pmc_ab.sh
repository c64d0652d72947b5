# Usage: bash tools/gpu_pmc_ab.sh <tag> "<env A>" "<env B>" [kernel substring] -- HBM bytes per launch (rocprofv3 PMC
# FETCH_SIZE and WRITE_SIZE, separate passes, tools/pmc_summary.py corrections) of the Res10 bench command under two
# environment settings; prints the rows of the kernels matching the substring (default: heads384)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; K=${4:-heads384}
O=gpurun_out
mkdir -p $O
for k in A B; do
  if [ $k = A ]; then E="$A"; else E="$B"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    env $E timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmcab_${TAG}_${k}_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-calib > $O/pmcab_${TAG}_${k}_$c.log 2>&1 || exit 1
  done
  f=$(find $O/pmcab_${TAG}_${k}_FETCH_SIZE -name "*counter_collection.csv" | head -1)
  w=$(find $O/pmcab_${TAG}_${k}_WRITE_SIZE -name "*counter_collection.csv" | head -1)
  python tools/pmc_summary.py $f $w $O/pmcab_${TAG}_${k}.json > /dev/null || exit 1
  python -c "
import json
d = json.load(open('$O/pmcab_${TAG}_${k}.json'))['kernels']
for n, v in d.items():
    if '$K' in n:
        print('$k', '$E', n, v)
"
  rm -rf $O/pmcab_${TAG}_${k}_FETCH_SIZE $O/pmcab_${TAG}_${k}_WRITE_SIZE
done

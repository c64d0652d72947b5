# Usage: bash tools/gpu_ab2.sh <tag> "<A: env or lib>" "<B: env or lib>" [bench args] -- A/B on one box of two builds
# (an argument ending in .so is a library under scdhip/, loaded through SCDHIP_LIB) or two environment settings
# ("X=1"), alternating A B A B (bench line: img/s, ms/step, heads GEMM live ms), then one rocprofv3 kernel trace of
# each with its kernel summary: gpurun_out/ab2_<tag>_{A,B}_kernel_summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; shift 3
O=gpurun_out
mkdir -p $O
envof() { case "$1" in *.so) echo "SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/$1" ;; *) echo "$1" ;; esac; }
for i in 1 2; do
  for k in A B; do
    if [ $k = A ]; then E=$(envof "$A"); else E=$(envof "$B"); fi
    env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > $O/ab2_${TAG}_${k}_$i.json 2>> $O/ab2_${TAG}.err || exit 1
    python -c "import json; d=json.load(open('$O/ab2_${TAG}_${k}_$i.json')); r=d.get('roofline') or {}; print('$k', d['value'], d['ms_per_step'], r.get('avg_launch_ms'), r.get('frac'))"
  done
done
for k in A B; do
  if [ $k = A ]; then E=$(envof "$A"); else E=$(envof "$B"); fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ab2_${TAG}_${k}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > /dev/null 2>> $O/ab2_${TAG}.err || exit 1
  python tools/prof_summary.py $O/ab2_${TAG}_${k}_prof/run_kernel_trace.csv $O/ab2_${TAG}_${k}_kernel_stats.csv > $O/ab2_${TAG}_${k}_kernel_summary.txt 2>&1
  python tools/step_timeline.py $O/ab2_${TAG}_${k}_prof/run_kernel_trace.csv > $O/ab2_${TAG}_${k}_step_timeline.txt 2>&1
  rm -rf $O/ab2_${TAG}_${k}_prof
done
echo ab2 done

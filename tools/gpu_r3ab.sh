# Usage: bash tools/gpu_r3ab.sh -- the round-3 HEAD (fe15776, its own tree and library in _r3/, built in the build
# container) against the current tree on one box: Res10 bench round-robin three times, then a kernel trace of the
# round-3 tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$PWD/gpurun_out
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/r3ab_cur_$i.json 2>> $O/r3ab.err || exit 1
  python -c "import json; d=json.load(open('$O/r3ab_cur_$i.json')); print('cur', d['value'], d['ms_per_step'])"
  (cd _r3 && timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/r3ab_r3_$i.json 2>> $O/r3ab.err) || exit 1
  python -c "import json; d=json.load(open('$O/r3ab_r3_$i.json')); print('r3 ', d['value'], d['ms_per_step'])"
done
(cd _r3 && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r3ab_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>> $O/r3ab.err) || exit 1
python tools/prof_summary.py $O/r3ab_prof/run_kernel_trace.csv $O/r3ab_r3_kernel_stats.csv > $O/r3ab_r3_kernel_summary.txt 2>&1
python tools/step_timeline.py $O/r3ab_prof/run_kernel_trace.csv > $O/r3ab_r3_step_timeline.txt 2>&1
rm -rf $O/r3ab_prof
echo r3ab done

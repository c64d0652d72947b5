# Usage: bash tools/gpu_r4.sh [tag] [pytest-args...] -- the GPU suite (or the given tests), the Res10 bench line, and a
# rocprofv3 kernel trace of the bench command with its kernel summary and step timeline, into gpurun_out/<tag>_*
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4}
shift
O=gpurun_out
mkdir -p $O
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf -s ${@:-tests} > $O/${T}_tests.log 2>&1
  rc=$?
  tail -3 $O/${T}_tests.log
  # a fault, abort or timeout ends the call here (a plain test failure does not)
  case $rc in 0|1) ;; *) echo "pytest rc $rc"; exit $rc ;; esac
fi
timeout -k 10 400 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
cut -c1-300 $O/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/${T}_profbench.json 2> $O/${T}_prof.err || exit 1
python tools/prof_summary.py $O/${T}_prof/run_kernel_trace.csv $O/${T}_kernel_stats.csv > $O/${T}_kernel_summary.txt 2>&1
python tools/step_timeline.py $O/${T}_prof/run_kernel_trace.csv > $O/${T}_step_timeline.txt 2>&1
echo all done

# Usage: bash tools/gpu_suite.sh [tag] -- the GPU suite, then the Res10 bench line and its rocprofv3 trace (kernel
# summary, step timeline, rocprofv3 --stats) and the host issue cost, into gpurun_out/<tag>_*; PMC passes and the
# other configs: tools/gpu_profiles.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r5}
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests > $O/${T}_tests.log 2>&1
rc=$?; tail -3 $O/${T}_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
cut -c1-300 $O/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-calib > $O/${T}_profbench.json 2> $O/${T}_prof.err || exit 1
python tools/prof_summary.py $O/${T}_prof/run_kernel_trace.csv $O/${T}_kernel_stats.csv > $O/${T}_kernel_summary.txt 2>&1
python tools/step_timeline.py $O/${T}_prof/run_kernel_trace.csv > $O/${T}_step_timeline.txt 2>&1
cp $O/${T}_prof/run_kernel_stats.csv $O/${T}_rocprof_kernel_stats.csv 2>/dev/null
rm -rf $O/${T}_prof
timeout -k 10 300 python tools/host_overhead.py --steps 30 > $O/${T}_host_overhead.txt 2>&1 || exit 1
cat $O/${T}_host_overhead.txt
echo final done

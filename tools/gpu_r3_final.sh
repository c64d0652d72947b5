# Usage: bash tools/gpu_r3_final.sh -- the GPU suite, then the Res10 bench line (reads the committed PMC summaries) and
# a rocprofv3 kernel trace of the bench command, into gpurun_out/r3_* (a shorter gpu_r3_profiles.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $O/tall_final.log 2>&1 || { tail -5 $O/tall_final.log; exit 1; }
tail -1 $O/tall_final.log
timeout -k 10 400 python bench.py > $O/r3_bench.json 2> $O/r3_bench.err || exit 1
cut -c1-200 $O/r3_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r3_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/r3_profbench.json 2> $O/r3_prof.err || exit 1
python tools/prof_summary.py $O/r3_prof/run_kernel_trace.csv $O/r3_kernel_stats.csv > $O/r3_kernel_summary.txt 2>&1
python tools/step_timeline.py $O/r3_prof/run_kernel_trace.csv > $O/r3_step_timeline.txt 2>&1
echo all done

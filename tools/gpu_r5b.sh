set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out; T=r5b
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf tests/test_kernels_gpu.py tests/test_corner_gpu.py -k "stem or cpool or corner" > $O/${T}_tests.log 2>&1; rc=$?; tail -4 $O/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 2 3; do SCD_CPOOL_BWD=$v timeout -k 10 120 python tools/hbm_bench.py --only cpool > $O/${T}_cpool$v.txt 2>&1 || exit 1; echo "variant $v"; grep bwd $O/${T}_cpool$v.txt; done
timeout -k 10 120 python tools/stem_bench.py > $O/${T}_stem.txt 2>&1 || exit 1; cat $O/${T}_stem.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
cut -c1-200 $O/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/${T}_profbench.json 2> $O/${T}_prof.err || exit 1
python tools/prof_summary.py $O/${T}_prof/run_kernel_trace.csv $O/${T}_kernel_stats.csv > $O/${T}_kernel_summary.txt 2>&1
python tools/step_timeline.py $O/${T}_prof/run_kernel_trace.csv > $O/${T}_step_timeline.txt 2>&1
rm -rf $O/${T}_prof
for c in FETCH_SIZE WRITE_SIZE; do timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${T}_pmc_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/${T}_pmc_$c.log 2>&1 || exit 1; done
f=$(find $O/${T}_pmc_FETCH_SIZE -name "*counter_collection.csv" | head -1); w=$(find $O/${T}_pmc_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python tools/pmc_summary.py $f $w $O/${T}_pmc_traffic.json 32 bf16 "python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline" centerOffsetRes10 512 > $O/${T}_pmc_traffic.txt
grep -i "stem\|cpool" $O/${T}_pmc_traffic.txt
rm -rf $O/${T}_pmc_FETCH_SIZE $O/${T}_pmc_WRITE_SIZE
echo done

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_model_gpu.py -x -q -m gpu > gpurun_out/t_model.log 2>&1; rc=$?
tail -40 gpurun_out/t_model.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?
cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
exit $rc

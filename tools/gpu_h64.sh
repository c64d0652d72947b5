set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "h64 or conv_fwd_dgrad" -v --timeout 120 --timeout-method thread > gpurun_out/tests_h64.log 2>&1; rc=$?
tail -5 gpurun_out/tests_h64.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/tests_h64.log | head -20; exit $rc; }
timeout -k 10 120 python tools/gemm_bench.py --only layer1 > gpurun_out/gemm_h64_on.log 2>&1 && cat gpurun_out/gemm_h64_on.log
SCD_GEMM_H64=0 timeout -k 10 120 python tools/gemm_bench.py --only layer1 > gpurun_out/gemm_h64_off.log 2>&1 && cat gpurun_out/gemm_h64_off.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_h64_on.json 2>/dev/null && cat gpurun_out/bench_h64_on.json | cut -c1-200
SCD_GEMM_H64=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_h64_off.json 2>/dev/null && cat gpurun_out/bench_h64_off.json | cut -c1-200

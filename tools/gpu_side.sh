# Usage: bash tools/gpu_side.sh <tag>  -- all GPU tests, step bench with the weight-gradient side stream off (A)
# and on (B), 2-rank shared-GPU rehearsal of the distributed bench path
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-s}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  SCD_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
  echo "side=$v $(python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['final_loss'])")"
done
SCD_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --batch 8 > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err; rc=$?
cat gpurun_out/bench2_$TAG.json
exit $rc

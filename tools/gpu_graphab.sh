# Usage: bash tools/gpu_graphab.sh <tag> -- graph replay vs eager under HIP runtime knobs, + a kernel trace of the graph run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-gab}
mkdir -p gpurun_out
run() {  # name, env...  (bench flags in $EXTRA)
    local name=$1; shift
    timeout -k 10 200 env "$@" python bench.py --no-cpu-baseline --steps 30 $EXTRA > gpurun_out/gab_${TAG}_$name.json 2> gpurun_out/gab_${TAG}_$name.err || return 1
    python -c "import json,sys; d=json.load(open('gpurun_out/gab_${TAG}_$name.json')); print('%-14s %8.2f img/s %7.3f ms heads %.4f ms' % ('$name', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']))"
}
EXTRA=--eager run eager A=1 && EXTRA=  run graph A=1 && run graph_q1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && run graph_q2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 \
  && run graph_q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 && run graph_pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gtrace_$TAG -o run -- python3 bench.py --steps 6 --warmup 4 --no-cpu-baseline > /dev/null 2> gpurun_out/gtrace_$TAG.err

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k stem --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
SCDHIP_LIB=$PWD/scd-resnet_amd/scdhip/libscdhip_base.so timeout -k 10 200 python tools/hbm_bench.py 2>&1 | grep stem_conv
timeout -k 10 200 python tools/hbm_bench.py 2>&1 | grep stem_conv

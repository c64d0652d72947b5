# Usage: bash tools/gpu_r4f.sh -- the GPU suite on the fence-free fused BN finalize, the fused finalize A/B (Res10 bench
# + kernel traces), and the host issue cost of a step (tools/host_overhead.py, tools/host_profile.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu -rf -s tests > $O/r4f_tests.log 2>&1
rc=$?; tail -3 $O/r4f_tests.log; case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_ab2.sh fin2 SCD_BN_FIN_FUSE=0 SCD_BN_FIN_FUSE=1 || exit 1
timeout -k 10 300 python tools/host_overhead.py --steps 30 > $O/r4f_host_overhead.txt 2>&1 || exit 1
cat $O/r4f_host_overhead.txt
timeout -k 10 300 python tools/host_profile.py --steps 20 --top 60 > $O/r4f_host_profile.txt 2>&1 || exit 1
echo r4f done

# Usage: bash tools/gpu_libab.sh <tag> "<tool command>" lib1.so lib2.so ... -- a standalone tool (e.g. tools/stem_bench.py)
# under each library build (scdhip/<lib>, through SCDHIP_LIB; "default" = scdhip/libscdhip.so), round-robin twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CMD=$2; shift 2
O=gpurun_out
mkdir -p $O
for i in 1 2; do
  for l in "$@"; do
    case "$l" in default) lib=$PWD/scd-resnet_amd/scdhip/libscdhip.so ;; *) lib=$PWD/scd-resnet_amd/scdhip/$l ;; esac
    echo "== $l ($i)"
    SCDHIP_LIB=$lib timeout -k 10 120 $CMD > $O/libab_${TAG}_${l}_$i.txt 2>&1 || exit 1
    grep -v amdgpu.ids $O/libab_${TAG}_${l}_$i.txt
  done
done

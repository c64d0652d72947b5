# Usage: bash tools/build_variant.sh <name> [SRC=<conv_gemm.hip path>] <hipcc -D flags...>
# builds scd-resnet_amd/scdhip/libscdhip_<name>.so with conv_gemm.hip (or SRC) compiled under the given macros
# (timing experiments only; load with SCDHIP_LIB=<path>)
set -e
cd "$(dirname "$0")/../scd-resnet_amd/csrc"
NAME=$1; shift
SRC=conv_gemm.hip
if [[ "$1" == SRC=* ]]; then SRC=${1#SRC=}; shift; fi
mkdir -p build/var_$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Wno-unused-function -I. "$@" -c $SRC -o build/var_$NAME/conv_gemm.o
OBJS="$(ls build/*.o | grep -v conv_gemm.o) $(ls build/f16/*.o)"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/var_$NAME/conv_gemm.o $OBJS -o ../scdhip/libscdhip_$NAME.so

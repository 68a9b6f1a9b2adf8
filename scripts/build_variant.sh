# build a profiling variant of libauthjx.so: scripts/build_variant.sh NAME -DFLAG ...
# (kernels recompiled with the extra flags, host objects reused; load it with AUTHJX_LIB)
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p scripts/bin scripts/var
B=authorino_amd/csrc/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function "$@" -c authorino_amd/csrc/ajx_kernels.hip -o scripts/bin/k_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/var/libauthjx_$NAME.so $B/*.cpp.o scripts/bin/k_$NAME.o
rm -f scripts/bin/k_$NAME.o
echo scripts/var/libauthjx_$NAME.so

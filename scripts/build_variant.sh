# build a profiling variant of libauthjx.so: scripts/build_variant.sh NAME -DFLAG ...
# (the lean kernel's translation unit, ajx_lean.hip, recompiled with the extra flags; every
# other object is the in-tree build's; load it with AUTHJX_LIB). AJX_KERNELS=1 recompiles
# ajx_kernels.hip with the flags instead.
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p scripts/bin scripts/var
B=authorino_amd/csrc/build
SRC=${AJX_KERNELS:+ajx_kernels.hip}
SRC=${SRC:-ajx_lean.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function "$@" -c authorino_amd/csrc/$SRC -o scripts/bin/k_$NAME.o
OBJS=$(for f in ajx_regex.cpp ajx_compiler.cpp ajx_api.cpp ajx_index.cpp ajx_producer.cpp ajx_kernels.hip ajx_lean.hip; do [ $f = $SRC ] || echo $B/$f.o; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/var/libauthjx_$NAME.so $OBJS scripts/bin/k_$NAME.o
rm -f scripts/bin/k_$NAME.o
echo scripts/var/libauthjx_$NAME.so

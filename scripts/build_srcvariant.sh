# build a profiling variant of libauthjx.so with a replacement header:
#   scripts/build_srcvariant.sh NAME HEADER_FILE TARGET_NAME [-DFLAG ...]
# (the kernels recompiled from a copy of csrc/ with TARGET_NAME replaced; host objects reused)
set -e
cd "$(dirname "$0")/.."
NAME=$1; HDR=$2; TGT=$3; shift 3
T=$(mktemp -d)
cp authorino_amd/csrc/*.h authorino_amd/csrc/*.hip "$T"/
cp "$HDR" "$T/$TGT"
mkdir -p scripts/bin scripts/var
B=authorino_amd/csrc/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function "$@" -c "$T/ajx_kernels.hip" -o scripts/bin/k_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/var/libauthjx_$NAME.so $B/*.cpp.o scripts/bin/k_$NAME.o
rm -rf "$T" scripts/bin/k_$NAME.o
echo scripts/var/libauthjx_$NAME.so

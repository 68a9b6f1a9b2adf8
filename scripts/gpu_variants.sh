# timing of profiling / occupancy variants of libauthjx.so (scripts/build_variant.sh) on c2 and c3
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/variants.log
for v in "$@"; do
  lib=scripts/bin/libauthjx_$v.so
  [ "$v" = base ] && lib=authorino_amd/libauthjx.so
  for w in c2 c3; do
    echo "== $v $w" >> gpurun_out/variants.log
    AUTHJX_LIB=$PWD/$lib timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0 >> gpurun_out/variants.log 2>&1 || exit $?
  done
done

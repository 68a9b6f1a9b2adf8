# event scanner (31) vs token scanner (0), default build and a 3-waves/SIMD build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ev2 && export TMPDIR=/tmp
for w in c2 c3; do
  timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0,31 > gpurun_out/ev2/ab_$w.log 2>&1 || exit $?
  AUTHJX_LIB=$PWD/scripts/bin/libauthjx_w3.so timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0,31 > gpurun_out/ev2/ab_w3_$w.log 2>&1 || exit $?
done

# register budget experiments: the default kernel at 3 and 2 waves/SIMD, and the
# unrolled key lookup at 3 waves/SIMD, against the default build (c2, c3)
cd $GRAFT_REPO_ROOT && O=gpurun_out/waves && mkdir -p $O && export TMPDIR=/tmp
for w in c2 c3; do
  timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0 > $O/base_$w.log 2>&1 || exit $?
  for v in w3 w3u w2; do
    AUTHJX_LIB=$PWD/scripts/var/libauthjx_$v.so timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0 > $O/${v}_$w.log 2>&1 || exit $?
  done
done

# time split of the single-pass kernel on c2 / c3: modes 0 full, 1 loads, 2 + classification,
# 3 stage A / stage B split; build variants: walk (token loop skeleton), nokeys, noscalar
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abl && export TMPDIR=/tmp
for w in c2; do
  timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0 > gpurun_out/abl/base_$w.log 2>&1 || exit $?
  for v in walk nokeys noscalar; do
    AUTHJX_LIB=$PWD/scripts/bin/libauthjx_$v.so timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0 > gpurun_out/abl/${v}_$w.log 2>&1 || exit $?
  done
done

# key lookup ablations of the token scanner on c2 (profiling variants in scripts/var)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/keyabl && export TMPDIR=/tmp
timeout -k 10 200 python scripts/ablate_scan.py c2 1048576 0 > gpurun_out/keyabl/base.log 2>&1 || exit $?
for v in noesc nosig nocmp probe1 nokeys; do
  AUTHJX_LIB=$PWD/scripts/var/libauthjx_$v.so timeout -k 10 200 python scripts/ablate_scan.py c2 1048576 0 > gpurun_out/keyabl/$v.log 2>&1 || exit $?
done

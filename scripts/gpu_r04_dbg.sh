# round 4: run named GPU tests with full tracebacks (debugging)
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04d} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $TESTS -v --tb=long --timeout 100 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "Error|error|assert|FAILED|PASSED" $O/pytest.log | head -60
exit 0

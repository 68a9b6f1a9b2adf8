# round 4: one staging copy per serving batch, results written to mapped host memory, no
# counter fill; stream / batcher GPU tests, then the serving sweep over worker counts
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04s2} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_chain.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 600 python -u scripts/serve_sweep.py > $O/sweep.log 2>&1; rc=$?
cat $O/sweep.log | tail -12
[ $rc -eq 0 ] || exit 1
echo done

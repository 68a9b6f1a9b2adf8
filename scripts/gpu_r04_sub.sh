# round 4: sub-phase clocks of the small-batch stream kernel (kernel mode 53), stream tests
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04sub} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/lat_phases.py > $O/phases.log 2>&1 || { tail -5 $O/phases.log; exit 1; }
cat $O/phases.log | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
echo done

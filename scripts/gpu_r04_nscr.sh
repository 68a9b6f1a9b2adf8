# round 4: stage-B list as a call (not inlined), blob copy and phase clocks out of scratch:
# parity, phases, serving, c2 / c3 kernel times and scratch
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04nscr} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_chain.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/lat_phases.py > $O/phases.log 2>&1 || { tail -5 $O/phases.log; exit 1; }
grep -v amdgpu.ids $O/phases.log
SWEEP_WORKERS=2 timeout -k 10 300 python -u scripts/serve_sweep.py > $O/sweep.log 2>&1 || { tail -5 $O/sweep.log; exit 1; }
grep workers $O/sweep.log
OUT=${OUT:-r04nscr} bash scripts/gpu_r04_pack.sh 2>&1 | grep -v "passed"

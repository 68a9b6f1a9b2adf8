# round 4: bench lines of the streaming kernel and the lean kernel, then the GPU test suite
cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r04c} && mkdir -p $O && export TMPDIR=/tmp
MODES="${MODES:-0 41 50}" WLS="${WLS:-c2}" OUT=${OUT:-r04c} bash scripts/gpu_r04_stream.sh &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${TESTS:-} > $O/pytest.log 2>&1
rc=$?; tail -40 $O/pytest.log; exit $rc

# ablation / fused-vs-split timing on c2 and c3, then the GPU parity tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python scripts/ablate_scan.py c2 > gpurun_out/ablate.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ablate_scan.py c3 >> gpurun_out/ablate.log 2>&1 || exit $?
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1

# multi-tenant (c4) single-pass kernel: workgroup-uniform LDS staging of the ruleset (0)
# vs every table read from global memory (300), on the bucketed c4 batch
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python scripts/ablate_scan.py c4 2097152 0,300 > gpurun_out/tenant_ab.log 2>&1 || exit $?

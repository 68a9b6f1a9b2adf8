# wave kernel: time split by ablation (c2), kernel stats and SQ instruction counters
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wprof && export TMPDIR=/tmp
for m in 0 14 11 12 6; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --steps 10 --kernel-mode $m > gpurun_out/wprof/c2_m$m.log 2>&1 || exit $?
done
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_BRANCH --output-format csv -d gpurun_out/wprof/pmc_sq -o sq -- python -u bench.py --no-cpu --no-pcie --steps 2 --warmup 1 > gpurun_out/wprof/pmc_sq.log 2>&1 || exit $?

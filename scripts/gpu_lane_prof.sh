# lane kernel (c2): time split by ablation, occupancy variants, SQ instruction counters
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/lprof && export TMPDIR=/tmp
for m in 0 24 23 22 21; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --steps 10 --kernel-mode $m > gpurun_out/lprof/c2_m$m.log 2>&1 || exit $?
done
for v in w2 w3; do
  AUTHJX_LIB=$PWD/scripts/bin/libauthjx_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --steps 10 > gpurun_out/lprof/c2_$v.log 2>&1 || exit $?
done
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_BRANCH --output-format csv -d gpurun_out/lprof/pmc_sq -o sq -- python -u bench.py --no-cpu --no-pcie --steps 2 --warmup 1 > gpurun_out/lprof/pmc_sq.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SCRATCH SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/lprof/pmc_sq2 -o sq2 -- python -u bench.py --no-cpu --no-pcie --steps 2 --warmup 1 > gpurun_out/lprof/pmc_sq2.log 2>&1 || true

# round 4: GPU parity file first (error detail), then SQ instruction-mix passes of the
# streaming kernel (kernel mode 0 full, 50 structural pass alone) on c2
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04p} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -30 $O/pytest.log
[ $rc -le 1 ] || exit 1
for m in ${MODES:-50 0}; do
  (cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/pmc1_m$m -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --steps 2 --warmup 1 --kernel-mode $m > $R/$O/pmc1_m$m.log 2>&1) || { echo "pmc1 $m failed"; exit 1; }
  (cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA --output-format csv -d $R/$O/pmc2_m$m -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --steps 2 --warmup 1 --kernel-mode $m > $R/$O/pmc2_m$m.log 2>&1) || { echo "pmc2 $m failed"; exit 1; }
done
echo done

# round 3: where the lean kernel's time goes (c2): ablation builds (scripts/var) and the
# SQ instruction mix of the default build (two PMC passes)
cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r03g} && mkdir -p $O && export TMPDIR=/tmp
W=${W:-c2}
for v in abl1 abl2 nob; do
  AUTHJX_LIB=scripts/var/libauthjx_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload $W --steps 10 > $O/abl_${W}_$v.log 2>&1 || { echo "$v failed"; tail -5 $O/abl_${W}_$v.log; exit 1; }
done
timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload $W --steps 10 > $O/abl_${W}_full.log 2>&1 || exit 1
for v in abl1 abl2 nob full; do python3 -c "
import json
for l in open('$O/abl_${W}_$v.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', round(d['ms_per_step'],3), 'ms', d['roofline']['kernel_ms'])"; done
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $GRAFT_REPO_ROOT/$O/pmcq1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pcie --workload $W --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$O/pmcq1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --output-format csv -d $GRAFT_REPO_ROOT/$O/pmcq2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pcie --workload $W --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$O/pmcq2.log 2>&1 || exit $?
echo done

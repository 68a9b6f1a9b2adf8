# round 3: lean kernel c2 ablations (classification, stage A only, full) + SQ mix of the
# stage-A-only and the full build
cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r03h} && mkdir -p $O && export TMPDIR=/tmp
W=${W:-c2}
for v in abl2 nob; do
  AUTHJX_LIB=scripts/var/libauthjx_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload $W --steps 10 > $O/abl_${W}_$v.log 2>&1 || { echo "$v failed"; tail -5 $O/abl_${W}_$v.log; exit 1; }
done
timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload $W --steps 10 > $O/abl_${W}_full.log 2>&1 || exit 1
for v in abl2 nob full; do python3 -c "
import json
for l in open('$O/abl_${W}_$v.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', round(d['ms_per_step'],3), 'ms', d['roofline']['kernel_ms'], d.get('parity'))"; done
cd /tmp
for v in nob full; do
  L=$GRAFT_REPO_ROOT/scripts/var/libauthjx_$v.so; [ $v = full ] && L=$GRAFT_REPO_ROOT/authorino_amd/libauthjx.so
  AUTHJX_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pcie --workload $W --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$O/pmc_$v.log 2>&1 || exit $?
done
echo done

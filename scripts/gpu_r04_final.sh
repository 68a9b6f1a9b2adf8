# round 4 evidence, part 1: HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one counter per
# pass) of the dominant kernel per workload -> pmc_traffic.json, the SQ mix of c2 and c3,
# the streaming kernel's SQ mix on c2 (kernel modes 50 / 52); part 2: gpu_r04_final2.sh
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04final} && mkdir -p $O && export TMPDIR=/tmp
ns() { case $1 in c4|c5) echo 2097152;; *) echo 1048576;; esac; }
for w in ${WLS:-c2 c3 c4 c5}; do
  k=ajx_scan_lean; [ $w = c4 ] && k=ajx_scan_fused_tenant
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_f_$w -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $w --steps 2 --warmup 1 > $R/$O/pmc_f_$w.log 2>&1) || { echo "pmc fetch $w failed"; exit 1; }
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_w_$w -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $w --steps 2 --warmup 1 > $R/$O/pmc_w_$w.log 2>&1) || { echo "pmc write $w failed"; exit 1; }
  python3 scripts/pmc_traffic.py $O/pmc_f_$w $O/pmc_w_$w $w $(ns $w) pmc_traffic.json $k > $O/pmc_$w.txt || exit 1
  echo "traffic $w: $(tail -1 $O/pmc_$w.txt)"
done
for w in c2 c3; do
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/pmc_sq_$w -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $w --steps 2 --warmup 1 > $R/$O/pmc_sq_$w.log 2>&1) || { echo "pmc sq $w failed"; exit 1; }
done
for m in 50 52; do
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/pmc_sq_stream_m$m -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --steps 2 --warmup 1 --kernel-mode $m > $R/$O/pmc_sq_stream_m$m.log 2>&1) || { echo "pmc sq stream $m failed"; exit 1; }
done
python3 scripts/pmc_summary.py $O/pmc_sq_c2 $O/pmc_sq_c3 $O/pmc_sq_stream_m50 $O/pmc_sq_stream_m52 > $O/pmc_sq.txt 2>&1
cp pmc_traffic.json $O/pmc_traffic.json
echo done

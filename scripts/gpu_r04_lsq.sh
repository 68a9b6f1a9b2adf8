# round 4: SQ instruction mix of the small-batch streaming kernel (64 c2 requests, one
# request per wave): is the latency path instruction-bound?
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04lsq} && mkdir -p $O && export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/sq_n64 -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --n 64 --steps 20 --warmup 2 > $R/$O/sq_n64.log 2>&1) || { echo "pmc failed"; tail -5 $O/sq_n64.log; exit 1; }
python3 - $O/sq_n64 <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "scan_stream" not in r["Kernel_Name"]:
        continue
    acc[r["Counter_Name"]][r["Dispatch_Id"]].append(float(r["Counter_Value"]))
for c, d in sorted(acc.items()):
    per = [sum(v) for v in d.values()]
    print("%-18s per dispatch (median over %d): %.0f" % (c, len(per), sorted(per)[len(per) // 2]))
PY
echo done

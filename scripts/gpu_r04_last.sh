# round 4, last evidence pass on the final tree: GPU suite, bench lines c2..c5 with
# rocprofv3 stats, the 64-request batch, HBM traffic passes, phase clocks, smoke
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04last} && mkdir -p $O && export TMPDIR=/tmp
WLS="c2 c3 c4 c5" OUT=${OUT:-r04last}/f2 bash scripts/gpu_r04_final2.sh || exit 1
timeout -k 10 300 python -u scripts/lat_phases.py > $O/phases.log 2>&1 || { tail -5 $O/phases.log; exit 1; }
grep -v amdgpu.ids $O/phases.log
WLS="c2 c3 c4 c5" OUT=${OUT:-r04last}/f1 bash scripts/gpu_r04_final.sh 2>&1 | grep -v "^  *$" | cut -c1-260

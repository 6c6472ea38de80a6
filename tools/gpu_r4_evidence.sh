# GPU box, round 4 evidence: the ICP timeline (debug build), the C2 PMC passes per kernel (incl. the
# ICP's LDS counters), a rocprofv3 kernel trace + stats of the default bench command, and the
# secondary bench lines (C2 colour, C3, C3I, C3R, C5, C5E, C5E swapping).  Outputs: gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_r4_evidence.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-ev}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 \
  || { tail -20 $O/icp_timeline.txt; exit 1; }
tail -4 $O/icp_timeline.txt | cut -c1-250
for cfg in "--colour" "--config C3" "--config C3I" "--config C3R" "--config C5" "--config C5E" "--config C5E --swapping"; do
  name=$(echo "$cfg" | tr -d ' -')
  timeout -k 10 400 python bench.py $cfg --no-cpu-baseline > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; exit 1; }
  tail -1 $O/bench_$name.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv > $O/kernel_trace_summary.txt 2>&1 || true
head -12 $O/kernel_trace_summary.txt | cut -c1-200
cd /tmp
P=$O/pmck
mkdir -p $P
ARGS="--steps 2 --warmup 1 --per-call-frames 0 --no-cpu-baseline --no-profile"
run() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $P/$name -o run -- \
    python3 $R/bench.py $ARGS > $P/$name.log 2>&1 || { tail -20 $P/$name.log; exit 1; }
  echo "pass $name ok"
}
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run write WRITE_SIZE
run occ SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM
run lds SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE
cd $R
for k in k_icp_frame k_raycast_pair k_integrate k_alloc_requests k_alloc_apply k_icp_maps_end; do
  extra=""; [ "$k" = "k_icp_frame" ] && extra="--full"
  python3 tools/pmc_kernel_summary.py $P $k $extra -o $O/pmc_kernel_c2_$k.json \
    --source "tools/gpu_r4_evidence.sh: rocprofv3 --pmc passes (fetch, write, occ, inst, lds, tcc) over bench.py $ARGS (C2), averaged per dispatch by tools/pmc_kernel_summary.py" > /dev/null
done
python3 -c "
import json
for k in ['k_icp_frame','k_raycast_pair','k_integrate']:
    d=json.load(open('$O/pmc_kernel_c2_'+k+'.json')); print(k, {x: d.get(x) for x in ('waves_per_cu','wave_lifetime_us','wait_any_frac','issue_stall_frac','valu_issue_frac','lds_bank_conflict_ratio')})"

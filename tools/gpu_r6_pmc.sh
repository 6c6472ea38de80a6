# GPU box, round 6: the C2 PMC passes per kernel at the current code (the default algebra, the
# reference's OpenCV 4; k_icp_frame<4>): occupancy / wait / VALU / LDS / L2 per kernel, then the
# frame-typed HBM traffic (tools/pmc_frames.py).  One counter group per pass, kernel trace only.
#   gpurun -- bash tools/gpu_r6_pmc.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc}
O=$R/gpurun_out/$TAG
P=$O/pmck
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --per-call-frames 0 --no-cpu-baseline --no-profile --no-other-algebra"
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
for k in k_icp_frame k_raycast_pair k_integrate; do
  extra=""; [ "$k" = "k_icp_frame" ] && extra="--full"
  python3 tools/pmc_kernel_summary.py $P $k $extra -o $O/pmc_kernel_c2_$k.json \
    --source "tools/gpu_r6_pmc.sh: rocprofv3 --pmc passes (fetch, write, occ, inst, lds, tcc) over bench.py $ARGS (C2, the default OpenCV 4 algebra), averaged per dispatch by tools/pmc_kernel_summary.py" > /dev/null
done
python3 -c "
import json
for k in ['k_icp_frame','k_raycast_pair','k_integrate']:
    d=json.load(open('$O/pmc_kernel_c2_'+k+'.json')); print(k, {x: d.get(x) for x in ('waves_per_cu','wave_lifetime_us','wait_any_frac','issue_stall_frac','valu_issue_frac','lds_bank_conflict_ratio','lds_util_frac')})"
cd /tmp
for pass in fetch write; do
  if [ $pass = fetch ]; then C="FETCH_SIZE"; else C="WRITE_SIZE"; fi
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/frames_$pass -o run -- \
    python3 $R/tools/pmc_frames.py $O/frames_$pass.json > $O/frames_$pass.log 2>&1 || { tail -20 $O/frames_$pass.log; exit 1; }
  echo "frames pass $pass ok"
done
cd $R
python3 tools/pmc_frames_summary.py $O/frames_fetch $O/frames_write $O/frames_fetch.json $O/pmc_traffic.json > $O/traffic_summary.json
head -40 $O/traffic_summary.json

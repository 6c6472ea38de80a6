# GPU box recipe: SQ / occupancy / memory PMC passes (one counter group per pass, kernel trace
# only) over one bench configuration, for the per-kernel instruction mix and wait breakdown.
# Usage: gpurun -- bash tools/gpu_pmc_kernel.sh TAG CONFIG   (CONFIG: C2 | C3I | C3R)
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-k}
CFG=${2:-C3I}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmck_$TAG
mkdir -p $O
if [ "$CFG" = "C3I" ] || [ "$CFG" = "C3R" ]; then ARGS="--config $CFG --steps 4"; else
  ARGS="--config $CFG --steps 2 --warmup 1 --per-call-frames 0 --no-cpu-baseline --no-profile"; fi
run() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- \
    python3 $R/bench.py $ARGS > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "pass $name ok"
}
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run write WRITE_SIZE
run occ SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE

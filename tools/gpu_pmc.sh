# GPU box recipe: rocprofv3 PMC passes (one counter group per pass, kernel trace only, no
# sys/runtime traces) over a short bench run.  Usage: gpurun -- bash tools/gpu_pmc.sh TAG [C2|C3|C3I|C3R]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc}
CFG=${2:-C2}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_$TAG
if [ "$CFG" = "C3I" ] || [ "$CFG" = "C3R" ]; then ARGS="--config $CFG --steps 4"; else
  ARGS="--config $CFG --steps 2 --warmup 1 --per-call-frames 0 --no-cpu-baseline --no-profile"; fi
run() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_$TAG/$name -o run -- \
    python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_$TAG/$name.log 2>&1 \
    || { tail -20 $R/gpurun_out/pmc_$TAG/$name.log; exit 1; }
  echo "pass $name ok"
}
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run write WRITE_SIZE
if [ "$CFG" = "C2" ]; then
  run occ SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
fi

# GPU box recipe: rocprofv3 PMC passes (one counter group per pass, kernel trace only, no
# sys/runtime traces) over a short bench run.  Usage: gpurun -- bash tools/gpu_pmc.sh TAG [C2|C3]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc}
CFG=${2:-C2}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_$TAG
run() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_$TAG/$name -o run -- \
    python $R/bench.py --config $CFG --steps 30 --warmup 5 --no-cpu-baseline --no-profile > $R/gpurun_out/pmc_$TAG/$name.log 2>&1 \
    || { tail -20 $R/gpurun_out/pmc_$TAG/$name.log; exit 1; }
  echo "pass $name ok"
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run write WRITE_SIZE
run l2 TCC_HIT_sum TCC_MISS_sum

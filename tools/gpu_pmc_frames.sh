# GPU box: PMC traffic of the frame kernels on the C2 bench's timed frames, per frame type
# (tools/pmc_frames.py under two rocprofv3 --pmc passes; summary by tools/pmc_frames_summary.py).
#   gpurun -- bash tools/gpu_pmc_frames.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-pf}
O=$R/gpurun_out/pmcf_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pass in fetch write; do
  if [ $pass = fetch ]; then C="FETCH_SIZE"; else C="WRITE_SIZE"; fi
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/$pass -o run -- \
    python3 $R/tools/pmc_frames.py $O/frames_$pass.json > $O/$pass.log 2>&1 || { tail -20 $O/$pass.log; exit 1; }
  echo "pass $pass ok"
done
cd $R
python3 tools/pmc_frames_summary.py $O/fetch $O/write $O/frames_fetch.json $O/pmc_traffic.json > $O/summary.json
cat $O/summary.json | head -80

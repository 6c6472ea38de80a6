set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof2 -o run -- python $R/bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-profile > $R/gpurun_out/prof2.log 2>&1
tail -1 $R/gpurun_out/prof2.log

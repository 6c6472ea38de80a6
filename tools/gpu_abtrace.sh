# GPU box: rocprofv3 kernel traces of the default bench with two builds of libtfusion_hip.so
# (A/B of a kernel change).  Usage: gpurun -- bash tools/gpu_abtrace.sh LIB_A LIB_B
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  TFUSION_HIP_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abt$i -o run -- \
    python $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-profile > $R/gpurun_out/abt$i.log 2>&1 \
    || { tail -20 $R/gpurun_out/abt$i.log; exit 1; }
  echo "== $lib: $(tail -1 $R/gpurun_out/abt$i.log | cut -c1-120)"
  (cd $R && python tools/trace_summary.py gpurun_out/abt$i/run_kernel_trace.csv | head -12)
done

# GPU box, round 5: where C3I's reads come from.  Per library (tree; diagnostic builds
# -DTF_C3X=1 no depth-image traffic, =2 no voxel loads, =3 neither): the C3I pass time, and
# rocprofv3 PMC passes FETCH_SIZE and TCC_EA0_RDREQ / TCC_EA0_RDREQ_32B (request counts by size).
#   gpurun -- bash tools/gpu_c3x.sh TAG tree c3x1 c3x2 c3x3
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
for v in "$@"; do
  if [ $v = tree ]; then L=$R/topfusion_amd/libtfusion_hip.so; else L=$R/tools/_build/$v/libtfusion_hip.so; fi
  export TFUSION_HIP_LIB=$L
  timeout -k 10 200 python3 $R/bench.py --config C3I > $O/c3i_$v.log 2>&1 || { tail -20 $O/c3i_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3i_$v.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$v C3I ms', d['ms_per_step'], 'lanes read', r['voxel_lanes_read'], 'written', r['voxel_lanes_written'])"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$v/fetch -o run -- \
    python3 $R/bench.py --config C3I --steps 4 > $O/pmc_$v.fetch.log 2>&1 || { tail -20 $O/pmc_$v.fetch.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_$v/write -o run -- \
    python3 $R/bench.py --config C3I --steps 4 > $O/pmc_$v.write.log 2>&1 || { tail -20 $O/pmc_$v.write.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/pmc_$v/req -o run -- \
    python3 $R/bench.py --config C3I --steps 4 > $O/pmc_$v.req.log 2>&1 || echo "request-size pass failed (see pmc_$v.req.log)"
  python3 $R/tools/pmc_traffic.py $O/pmc_$v C3I $O/traffic.json > /dev/null
  python3 -c "
import json; t=json.load(open('$O/traffic.json'))['C3I'].get('integrate', {}); print('$v', t)"
  cp $O/traffic.json $O/traffic_$v.json
done

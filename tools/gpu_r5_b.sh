# GPU box, round 5: ICP-tail micro-benchmark, a pytest selection, then the C5E engine batch in its
# four-launch (default) and seven-launch (TFUSION_FUSE_TAIL=0) forms, alternated.
#   gpurun -- bash tools/gpu_r5_b.sh TAG [pytest selection...]
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r5b}; shift || true
SEL=${@:-tests/test_gpu_hash_stress.py}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 60 ./tools/micro/icp_tail > $O/icp_tail.txt 2>&1 || { cat $O/icp_tail.txt; exit 1; }
cat $O/icp_tail.txt
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q -rs --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0 1 0; do
  TFUSION_FUSE_TAIL=$v timeout -k 10 300 python bench.py --config C5E --steps 20 > $O/c5e_$v.json 2> $O/c5e_$v.err || { tail -20 $O/c5e_$v.err; exit 1; }
  python -c "import json; e=json.loads(open('$O/c5e_$v.json').read().strip().splitlines()[-1]); print('C5E fuse_tail=$v', e['value'], 'sat', e['saturated_frames_per_sec'], 'first_fail', e['first_failure_frame'])"
done

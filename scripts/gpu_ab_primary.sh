# k_primary A/B: the wide-packet primary walk at 1 / 2 / 4 rays per lane (RTBVH_PRIMARY_RAYS),
# after the parity tests of the wide modes; C5 bench lines (no CPU baseline, no extras).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${TESTK:-wide or auto or c5 or containment or general or tiles or band or flight}" > gpurun_out/ab_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in ${RAYS:-1 4 2 1 4}; do
  RTBVH_PRIMARY_RAYS=$r timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/ab_r$r.json 2> gpurun_out/ab_r$r.err || { echo "BENCH r=$r FAILED"; tail -20 gpurun_out/ab_r$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_r$r.json'));k=d['kernels'];print('R=$r', 'value',d['value'],'step',d['ms_per_step'],'primary',k['k_primary']['ms'],'bounce',k['k_bounce_trav']['ms'],'lat',d['traversal']['one_frame_latency_ms'],'steps',d['visits']['primary_packet_steps'],'ident',d['traversal']['frames_identical'])"
done

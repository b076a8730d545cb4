# A/B runs of round 4 (one GPU call): the certified walks against the same walks unchecked (visit and
# re-trace counts), then library builds on the certified mode (ab_libs.sh; AB_LIBS: the .so files)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-ab}
if [ "${CERT_AB:-1}" = 1 ]; then
  AB_SET=certified AB_COUNTS=1 AB_ROUNDS=${AB_ROUNDS:-5} timeout -k 10 400 python -u scripts/ab_trace.py > gpurun_out/${T}_cert.log 2>&1 || { echo "CERT AB FAILED"; tail -20 gpurun_out/${T}_cert.log; exit 1; }
  cat gpurun_out/${T}_cert.log
fi
if [ -n "${AB_LIBS:-}" ]; then
  AB_SET=${LIB_SET:-certbase} ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash scripts/ab_libs.sh $AB_LIBS > gpurun_out/${T}_libs.log 2>&1 || { echo "LIB AB FAILED"; tail -20 gpurun_out/${T}_libs.log; exit 1; }
  cat gpurun_out/${T}_libs.log
fi
if [ "${PB_PHASES:-0}" = 1 ]; then   # k_primary_binned's phase split (RTBVH_PB_PROF builds)
  for lib in raytracebvh_amd/librtbvh_prof.so raytracebvh_amd/librtbvh_rmprof.so; do
    RTBVH_LIB=$(realpath $lib) timeout -k 10 300 python -u scripts/pb_phases.py > gpurun_out/${T}_phases_$(basename $lib .so).log 2>&1 || { echo "PHASES FAILED"; tail -10 gpurun_out/${T}_phases_$(basename $lib .so).log; exit 1; }
    echo "$lib: $(cat gpurun_out/${T}_phases_$(basename $lib .so).log)"
  done
fi

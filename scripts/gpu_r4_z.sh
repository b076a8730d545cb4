# Round 4, call z: the C3 bounce walks counted (scripts/c3_census.py), and the bounce queue sorted
# for coherence (RTBVH_FLAG_SORT_BOUNCE) beside AUTO's plain kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04_z}
timeout -k 10 120 python -u scripts/c3_census.py > gpurun_out/${T}_c3_census.log 2>&1 || { echo "census FAILED"; tail -5 gpurun_out/${T}_c3_census.log; exit 1; }
tail -1 gpurun_out/${T}_c3_census.log
for r in 1 2; do
  for m in auto sort packet+sort; do
    C3_MODE=$m timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_c3_modes.log || { echo "C3 $m FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_c3_modes.log
echo "call ok"

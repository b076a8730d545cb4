# Round 4, call cc: what the C3 bounce pass spends its time on -- probe builds (wrong frames, timing
# only): RTBVH_BOUNCE_PROBE=1 no walk (every bounce ray misses), =2 the walk without the hit's shading.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04_cc}
for r in 1 2; do
  for lib in new librtbvh_bprobe1.so librtbvh_bprobe2.so; do
    L=$PWD/ablib/$lib; [ $lib = new ] && L=$PWD/raytracebvh_amd/librtbvh.so
    echo -n "$lib " >> gpurun_out/${T}_bounce_probes.log
    RTBVH_LIB=$L C3_GRAPH=0 timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_bounce_probes.log || { echo "C3 $lib FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_bounce_probes.log
echo "call ok"

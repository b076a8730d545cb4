# Round 5, call y: A/B of the certified walk's wave-uniform bounded box test (RTBVH_CERT_UNIFORM 0 / 1), C5 certified mode
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_SET=certbase ROUNDS=3 AB_ROUNDS=3 timeout -k 10 900 bash scripts/ab_libs.sh ablib/librtbvh_unif0.so ablib/librtbvh_unif1.so > gpurun_out/r05_y_cert_uniform_ab.log 2>&1
rc=$?; cat gpurun_out/r05_y_cert_uniform_ab.log | cut -c1-400; exit $rc

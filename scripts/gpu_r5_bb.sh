# Round 5, call bb: A/B of the certified box test as packed FMA pairs (RTBVH_PK_BOX 0 / 1), C5 certified mode
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_SET=certbase ROUNDS=3 AB_ROUNDS=3 timeout -k 10 900 bash scripts/ab_libs.sh ablib/librtbvh_pk0.so ablib/librtbvh_pk1.so > gpurun_out/r05_bb_pk_box_ab.log 2>&1
rc=$?; grep -o 'librtbvh_pk[01].so\|"bounce_trav_ms_med": [0-9.]*\|"trace_ms_med": [0-9.]*\|frame_sha1": "[0-9a-f]*"' gpurun_out/r05_bb_pk_box_ab.log | paste -sd' ' | sed 's/librtbvh/\nlibrtbvh/g'; exit $rc

#!/bin/bash
# A/B of library builds (RTBVH_LIB) on the bench's mode: rounds x libs, interleaved.
# usage: scripts/ab_libs.sh lib1.so lib2.so ...   (env AB_SET, AB_ROUNDS, ROUNDS;
# AB_SCRIPT=ab_build.py for build-stage times)
set -o pipefail
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    out=$(RTBVH_LIB=$(realpath "$lib") AB_SET=${AB_SET:-base} AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 300 python scripts/${AB_SCRIPT:-ab_trace.py} 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "$(basename $lib) $(echo "$out" | grep -E "ms_med|stages_ms|frame_sha1|packet_steps")"
  done
done

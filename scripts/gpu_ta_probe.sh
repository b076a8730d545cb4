# Vector-memory pipeline counters of the bounce walk (TA / TCP busy) and the counter list of the box
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_avail.txt 2>&1 || true
grep -oE "\b(TA|TD|TCP)_[A-Z0-9_]+" $R/gpurun_out/counters_avail.txt | sort -u > $R/gpurun_out/counters_ta.txt || true
PMC_OUT=pmc_ta MODES="nearest+packet+refill+wide+binned" SETS="${TA_SETS:-TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE;TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum}" bash $R/scripts/gpu_pmc.sh

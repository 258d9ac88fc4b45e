# PMC counters of config 3's fp6 K-group main kernel alone (tools/prep_probe gemm_<kg|kv>main_N512:
# 4096x512x4096 q4_0 x q8_0, stationary weights, hipGraph replays), one --pmc pass per run.
# Usage (via gpurun): bash tools/pmc_fp6_main.sh gpurun_out/<dir> [kg|kv]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_fp6}
K=${2:-kv}
mkdir -p "$OUT"
pass() {
  timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o p -- tools/prep_probe gemm_${K}main_N512 > "$OUT/$1.log" 2>&1
}
pass fetch "FETCH_SIZE"
pass write "WRITE_SIZE"
pass tcp "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
pass tcc "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
pass sq1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
pass sq2 "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"

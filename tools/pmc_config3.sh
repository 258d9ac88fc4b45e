# PMC counters of config 3 (tools/pmc_config3.py: 30 stationary-weight q4_0 4096x512x4096 calls =
# prep_b_fp6_tile + gemm_fp6_kv_kernel each), one --pmc pass per run (gfx950 block limits), plus a
# kernel trace.  Usage (via gpurun): bash tools/pmc_config3.sh gpurun_out/<dir> [fmt]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_config3}
F=${2:-q4_0}
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- python3 tools/pmc_config3.py $F > "$OUT/trace.log" 2>&1
pass() {
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o p -- python3 tools/pmc_config3.py $F > "$OUT/$1.log" 2>&1
}
pass fetch "FETCH_SIZE"
pass write "WRITE_SIZE"
pass tcp "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
pass tcc "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
pass sq1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
pass sq2 "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"

# GPU step (via gpurun): SQ counters of the reference-order prefill GEMM and F16 kernel, one pass each
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_ref}
mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$OUT/p1" -o run -- python3 -u tools/ref_gemm_pmc.py > "$OUT/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 -u tools/ref_gemm_pmc.py > "$OUT/p2.log" 2>&1

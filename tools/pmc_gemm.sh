# SQ counters of the GEMM main kernels (fp6 q4_0 and super-block q4_K, 4 slices, stationary
# weights): two --pmc passes per format, each its own run.  Run via gpurun.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F6F4 SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_VALU_MFMA_I8 SQ_CYCLES GRBM_GUI_ACTIVE"
for F in q4_0 q4_k; do
  for k in 1 2; do
    eval "C=\$P$k"
    rm -rf gpurun_out/pmcg_${F}_$k
    FMT=$F SLICES=4 STATIONARY=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcg_${F}_$k -o p -- python3 tools/ab_gemm.py fp6 > gpurun_out/pmcg_${F}_$k.log 2>&1
  done
done

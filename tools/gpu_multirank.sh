# The bench's N>1 code paths on a one-GPU box: a one-rank RCCL communicator inside the
# captured graph (LAMM_BENCH_COMM1), then 2, 4 and 8 torchrun ranks sharing cuda:0 with the
# all-gather through gloo (LAMM_BENCH_REHEARSE).  Rank 0 checks the gathered C bit-exact.
# Usage (via gpurun): bash tools/gpu_multirank.sh gpurun_out/<dir>
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/multirank}
mkdir -p "$OUT"
LAMM_BENCH_COMM1=1 timeout -k 10 400 python -u bench.py --no-cpu --steps 200 > "$OUT/comm1.json" 2> "$OUT/comm1.err"
for n in 2 4 8; do
  LAMM_BENCH_REHEARSE=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29610 + n)) bench.py --gpus $n --no-cpu --no-llama --steps 50 \
    > "$OUT/rehearse_$n.json" 2> "$OUT/rehearse_$n.err"
done

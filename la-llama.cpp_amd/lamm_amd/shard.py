"""Row sharding of the lamm mul_mat across ranks -- host-side helpers.

Output rows are independent (``C[i, :]`` needs row i of A and all of B,
src/lamm_impl.hpp:50-53 -- the same contiguous row split ggml hands its threads,
src/lamm_impl.hpp:38-43), so each rank owns a contiguous slab of weight rows, computes
``C[:, r0:r1]`` and the slabs meet in one all-gather of C.  The split itself is the library's
(lamm_hip_shard_rows: every row exactly once -- the reference's ``job_size = M / nth`` drops
the remainder rows, SURVEY §8a defect 1); on GPUs the all-gather is the library's RCCL one
(lamm_amd.Comm.allgather_rows).  ``gather_rows`` is the same exchange through any
torch.distributed backend on host tensors: the CPU (gloo) tests and bench.py's one-GPU
rehearsal of the multi-rank path use it.
"""
import lamm_amd as la


def row_shard(M, world, rank, align=1):
    """Contiguous [r0, r1) of the M weight rows owned by ``rank`` (lamm_hip_shard_rows)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    r0, rows = la.shard_rows(M, world, rank, align)
    return r0, r0 + rows


def shard_rows_max(M, world, align=1):
    """Largest shard height (the all-gather's per-rank row count)."""
    return max(r1 - r0 for r0, r1 in (row_shard(M, world, r, align) for r in range(world)))


def gather_rows(dist, c_shard, M, N, world, rank, align=1, out=None):
    """All-gather the ranks' C slabs into the full ``C[N][M]`` (lamm layout, C[j*M + i]).

    ``c_shard``: this rank's ``[N][r1 - r0]`` block (torch tensor, contiguous).  Every
    rank sends a ``[N][mmax]`` block (zero-padded), one ``all_gather_into_tensor`` moves
    them, and one strided copy per rank interleaves the row slabs into ``[N][M]``."""
    import torch

    mmax = shard_rows_max(M, world, align)
    r0, r1 = row_shard(M, world, rank, align)
    send = torch.zeros((N, mmax), dtype=c_shard.dtype, device=c_shard.device)
    send[:, :r1 - r0] = c_shard.view(N, r1 - r0)
    recv = torch.empty((world, N, mmax), dtype=c_shard.dtype, device=c_shard.device)
    if world > 1:
        dist.all_gather_into_tensor(recv.view(-1), send.view(-1))
    else:
        recv[0] = send
    if out is None:
        out = torch.empty((N, M), dtype=c_shard.dtype, device=c_shard.device)
    for r in range(world):
        a0, a1 = row_shard(M, world, r, align)
        out[:, a0:a1] = recv[r, :, :a1 - a0]
    return out

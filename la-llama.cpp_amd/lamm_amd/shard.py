"""Row sharding of the lamm mul_mat across ranks.

Output rows are independent (``C[i, :]`` needs row i of A and all of B,
src/lamm_impl.hpp:50-53 -- the same contiguous row split ggml hands its threads,
src/lamm_impl.hpp:38-43), so one process per GPU owns a contiguous slab of weight rows,
computes ``C[:, r0:r1]`` and the slabs meet in one all-gather of C (RCCL over xGMI with the
``nccl`` backend, gloo in the CPU tests).  Unlike the reference's ``job_size = M / nth``
split, the remainder rows are not dropped (SURVEY §8a defect 1).
"""


def row_shard(M, world, rank, align=1):
    """Contiguous [r0, r1) of the M weight rows owned by ``rank``.

    Shards are whole multiples of ``align`` rows (the GEMM tile height) except the last
    one; the ``ceil(M / align)`` tiles are spread as evenly as possible, earlier ranks
    taking the extra tile."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    tiles = -(-M // align)
    base, extra = divmod(tiles, world)
    t0 = rank * base + min(rank, extra)
    t1 = t0 + base + (1 if rank < extra else 0)
    return min(M, t0 * align), min(M, t1 * align)


def shard_rows_max(M, world, align=1):
    """Largest shard height (the all-gather's per-rank row count)."""
    return max(r1 - r0 for r0, r1 in (row_shard(M, world, r, align) for r in range(world)))


def gather_rows(dist, c_shard, M, N, world, rank, align=1, out=None):
    """All-gather the ranks' C slabs into the full ``C[N][M]`` (lamm layout, C[j*M + i]).

    ``c_shard``: this rank's ``[N][r1 - r0]`` block (torch tensor, contiguous).  Every
    rank sends a ``[N][mmax]`` block (zero-padded), one ``all_gather_into_tensor`` moves
    them, and a single strided copy interleaves the row slabs into ``[N][M]``."""
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


class RowGather:
    """Preallocated all-gather of equal row slabs (every rank owns ``m`` rows; the bench's
    weak-scaling case): ``C_shard [R][m]`` (R = slices x N activation rows) -> ``C [R][world*m]``
    with one ``all_gather_into_tensor`` and one strided copy, no per-step allocation."""

    def __init__(self, dist, R, m, world, dtype, device):
        import torch

        self.dist, self.R, self.m, self.world = dist, R, m, world
        self.recv = torch.empty((world, R, m), dtype=dtype, device=device)
        self.out = torch.empty((R, world * m), dtype=dtype, device=device)

    def __call__(self, c_shard):
        if self.world > 1 and self.recv.is_cuda and self.dist.get_backend() == "gloo":
            # gloo is a host backend: stage device slabs through host memory (bench rehearsal)
            recv = self.recv.cpu()
            self.dist.all_gather_into_tensor(recv.view(-1), c_shard.reshape(-1).cpu())
            self.recv.copy_(recv)
        elif self.world > 1:
            self.dist.all_gather_into_tensor(self.recv.view(-1), c_shard.reshape(-1))
        else:
            self.recv[0].copy_(c_shard.view(self.R, self.m))
        self.out.view(self.R, self.world, self.m).copy_(self.recv.permute(1, 0, 2))
        return self.out

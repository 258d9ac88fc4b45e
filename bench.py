#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric for the MI355X lamm backend.

metric: "Q4_0xQ8_0 GEMM effective GFLOPS @ K=4096; achieved HBM GB/s (GEMV)"

Headline (`value`): BASELINE config 2 as the survey states it -- ONE Q4_0 x Q8_0
GEMV, M = 4096, N = 1, K = 4096, per step, the steps rotating over enough distinct weight copies
that every byte comes from HBM (> the 256 MiB Infinity Cache).  With N GPUs the ONE weight's rows
are split over the ranks (strong scaling, lamm_hip_shard_rows) and every step ends with the
library's RCCL all-gather of C (lamm_hip_allgather_rows), so each rank holds the whole C.
  value    = algorithmic bytes of one GEMV (A + B + C = 9,457,920 B) x steps / max-over-ranks time
  roofline = the rank's GEMV kernel alone: its slab's algorithmic bytes / its per-launch time
             (HIP events on the stream it runs on), vs 8 TB/s HBM3E
The K steps are captured once as a hipGraph and replayed (per-launch host submission through
Python/ctypes costs ~5 us, more than the kernel; bench measures the GPU).

Beside it (same JSON line):
  gemv_stacked  : 33 4096x4096 slices in ONE launch (steady-state streaming rate), N = 1
  gemm          : BASELINE config 3 (M=4096 N=512 K=4096, stationary weights): one slice and
                  a 4-slice batch; roofline = the WHOLE launch (activation prep + main loop +
                  split-K reduce).  N > 1: the slice's rows split over the ranks + the RCCL
                  all-gather of C (8 MiB)
  config1       : BASELINE config 1 (F32 M=N=K=512, la-benchmark-matmult's plumbing shape): the
                  GPU's F32 path and the reference's CPU path side by side
  sweep         : BASELINE config 4 (Q4_1 / Q5_0 / Q5_1 / Q8_0 / Q2_K at K=4096): per format the
                  single-call GEMV (config 2's measurement) and the config-3-shaped GEMM
  llama7b_e2e   : BASELINE config 5 through the unchanged caller -- llama.cpp-b2430's own
                  llama_decode (integration/_build/llama_e2e_hip: the reference's llama.cpp and
                  ggml with the LA_LLAMA hook linked to liblamm_hip.so), synthetic Llama-7B Q4_0
                  GGUF, pp512 / tg128; with N GPUs the boundary splits every weight's rows over
                  all N (LAMM_HIP_DEVICES)
  llama7b_matmul_step : the same model's weight matmuls through the device API (hipGraph) --
                  the ceiling without the ggml boundary's host round trips; with N GPUs every
                  weight's rows sharded over the N ranks (one llama-matmul-bench process per GPU,
                  RCCL all-gather after every projection, hipGraph-captured)
  cpu_baseline  : the reference itself (oracle/_ref: la-llama.cpp lamm opt-3 AVX2 build) on this
                  host's cores (the CPUs this process may use: affinity, cgroup quota,
                  OMP_NUM_THREADS -- the GPU box's share), rank 0, N = 1; the same leg checks a
                  sample of the GPU outputs above against the oracle (`parity_sample`) and runs
                  config 5's greedy-token parity (GPU build vs the reference, pp64 / tg16)

Synthetic data: A bytes random with valid fp16 scales; B = the GPU activation quantizer applied
to N(0,1) floats.  Inputs are resident in HBM before the timed region.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
I8_DENSE_PEAK_TOPS = 5000.0    # dense MFMA-i8 = 2x the 2.5 PF dense bf16 rate (MI355X_MICROARCH.md)
F32_VALU_PEAK_TFLOPS = 157.3   # f32 vector peak (v_pk_fma_f32; MI355X_MICROARCH.md F32 row)
MALL_BYTES = 256 << 20
ALIGN = 16                     # row-slab granularity of the GEMV split (one wave-group row tile)
GEMM_ALIGN = 256               # fp6 GEMM row tile

FP16_FIELDS = {  # byte offsets of fp16 scale fields inside one block (lamm_formats.h)
    "q4_0": [0], "q4_1": [0, 2], "q5_0": [0], "q5_1": [0, 2], "q8_0": [0], "q2_k": [80, 82],
    "q4_k": [0, 2], "q5_k": [0, 2], "q6_k": [208]}


GEMM_KERNELS = {"dq16": "lamm::gemm_dq2_kernel (csrc/lamm_gemm_dq.hip; f16 MFMA, block scales folded into the "
                        "operands, 1e-3 bar)",
                "fp6": "lamm::gemm_fp6_kv_kernel (csrc/lamm_gemm_fp6.hip; exact block dots)",
                "i8": "lamm::gemm3_kernel (csrc/lamm_gemm.hip; exact block dots)"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota and by
    OMP_NUM_THREADS (the GPU box exports its CPU share there: its nproc shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    src = f"affinity {n}"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            if q < n:
                n, src = q, f"cgroup cpu.max {q}"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < n:
        n, src = int(omp), f"OMP_NUM_THREADS={omp} (the box's CPU share)"
    return n, src


def make_weights(torch, la, fmt, slices, M, K, gen):
    t = la.BY_NAME[fmt]
    rb = la.row_bytes(t, K)
    assert rb % 16 == 0
    if fmt == "f32":
        return torch.randn(slices * M * K, device="cuda", generator=gen).view(torch.uint8), rb
    if fmt == "f16":
        return torch.randn(slices * M * K, device="cuda", generator=gen).half().view(torch.uint8), rb
    w = torch.randint(0, 256, (slices * M * rb,), dtype=torch.uint8, device="cuda", generator=gen)
    blocks = w.view(-1, la.type_size(t))
    for off in FP16_FIELDS[fmt]:
        d = (torch.rand(blocks.shape[0], device="cuda", generator=gen) * 0.02 + 1e-3).half()
        blocks[:, off:off + 2].view(torch.float16)[:, 0] = d
    return w, rb


def make_activations(torch, la, fmt, rows, K, gen):
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    x = torch.randn(rows, K, device="cuda", generator=gen)
    if vt == la.F32:
        return x.view(torch.uint8).reshape(-1).clone()
    y = torch.zeros(rows * la.row_bytes(vt, K) + 16, dtype=torch.uint8, device="cuda")
    la.quantize_torch(vt, x, y, flavour=1)
    return y


def gemv_bytes(la, fmt, M, K, N=1):
    t = la.BY_NAME[fmt]
    return M * la.row_bytes(t, K) + N * la.row_bytes(la.vec_dot_type(t), K) + 4 * M * N


class Ctx:
    """Ranks, devices and the communicators: gloo for control (barriers, the RCCL id, the
    max-over-ranks timing, on host tensors), the library's RCCL communicator for data."""

    def __init__(self, torch, la):
        import torch.distributed as dist
        self.torch, self.la, self.dist = torch, la, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # LAMM_BENCH_REHEARSE=1: the N>1 code path on a one-GPU box (every rank on cuda:0, the
        # all-gather through gloo on host copies -- RCCL refuses ranks sharing a device)
        self.rehearse = self.world > 1 and os.environ.get("LAMM_BENCH_REHEARSE") == "1"
        self.device = 0 if self.rehearse else local
        torch.cuda.set_device(self.device)
        self.comm = None
        if self.world > 1:
            dist.init_process_group("gloo")
            if not self.rehearse:
                uid = [la.comm_unique_id() if self.rank == 0 else None]
                dist.broadcast_object_list(uid, src=0)
                self.comm = la.Comm.rank(self.world, self.rank, uid[0], self.device)
        elif os.environ.get("LAMM_BENCH_COMM1") == "1":
            # the RCCL path on one GPU: a one-rank communicator, every step's all-gather through
            # RCCL (in the captured hipGraph) -- exercises what the multi-GPU run uses
            self.comm = la.Comm.rank(1, 0, la.comm_unique_id(), self.device)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, *vals):
        v = self.torch.tensor(vals, dtype=self.torch.float64)
        if self.world > 1:
            self.dist.all_reduce(v, op=self.dist.ReduceOp.MAX)
        return v.tolist()

    def allgather_rows(self, C, M, N, align, stream):
        """C (device tensor, [N][M]) holds this rank's rows at their place; gather the rest."""
        if self.world == 1 and self.comm is None:
            return
        if self.comm is not None:
            r0, rows = self.la.shard_rows(M, self.world, self.rank, align)
            self.comm.allgather_rows([C.data_ptr() + 4 * r0], [M], [C.data_ptr()], M, M, N, align, [stream])
        else:   # rehearsal: gloo on host copies
            from lamm_amd.shard import gather_rows
            r0, rows = self.la.shard_rows(M, self.world, self.rank, align)
            slab = C.view(N, M)[:, r0:r0 + rows].contiguous().cpu()
            C.copy_(gather_rows(self.dist, slab, M, N, self.world, self.rank, align).reshape(-1).to(C.device))

    def close(self):
        if self.comm is not None:
            self.comm.close()
        if self.world > 1:
            self.dist.destroy_process_group()


_SCRATCH = None


def flush_caches(torch):
    """Write a 512 MiB scratch buffer (2x the 256 MiB MALL, 128x an XCD's L2) so that weights an
    untimed pass touched are not still cached when the timed pass starts."""
    global _SCRATCH
    if _SCRATCH is None:
        _SCRATCH = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    _SCRATCH.fill_(1)


def time_steps(ctx, step, steps, warmup, graph=True, flush=False):
    """Warm-up, then EXACTLY `steps` steps bracketed by barrier + synchronize on both sides;
    returns (wall seconds per step, event-timed seconds per step -- both max over ranks --,
    graph used).  graph: the steps are captured once as a hipGraph and replayed in the timed
    region.  Everything runs on one side stream, the warm-up included, so the library's
    per-stream workspaces exist before the capture (nothing allocates while capturing)."""
    torch = ctx.torch
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        for i in range(warmup):
            step(i)
    torch.cuda.synchronize()
    g = None
    if graph:
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for s in range(steps):
                    step(warmup + s)
            g.replay()                      # one untimed replay (first-replay setup)
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 -- eager fallback, reported
            log("graph capture failed, eager steps:", str(e)[:200])
            g = None
            torch.cuda.synchronize()
    def run():
        if g is not None:
            g.replay()
        else:
            for s in range(steps):
                step(warmup + s)

    # the timed region: nothing but the K steps between the barrier + synchronize brackets (the
    # events of the second pass cost host calls of their own: profiles/r04/roofline/)
    with torch.cuda.stream(st):
        if flush:
            flush_caches(torch)
        ctx.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        ctx.barrier()
        wall = time.perf_counter() - t0
        # the same K steps again, timed by HIP events on the stream they run on
        if flush:
            flush_caches(torch)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        run()
        e1.record(st)
    torch.cuda.synchronize()
    ev = e0.elapsed_time(e1) / 1e3
    wmax, emax = ctx.max(wall / steps, ev / steps)
    return wmax, emax, g is not None


_STEPS_LIB = None


def isolated_launches(la, mats, R, Bm, Cm, n, sync_each=1, flags=0):
    """median duration (s) of n lamm_hip_matmul_ex dispatches from their own timestamps
    (lamm_hip_profile_next, tools/steps_loop.hip), each launched alone (sync_each) or back to back;
    None when the helper is not built or the kernel took no timestamps"""
    import ctypes
    if steps_lib(la) is None:
        return None
    import torch
    arr = (la.Matrix * R)(*mats)
    out = (ctypes.c_float * n)()
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    rc = _STEPS_LIB.lamm_steps_isolated_ex(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm),
                                           0, n, ctypes.c_void_p(st.cuda_stream), out, sync_each, flags)
    torch.cuda.synchronize()
    v = sorted(out)
    if rc != 0 or v[0] <= 0.0:
        log("lamm_steps_isolated failed:", rc, v[:3])
        return None
    return v[n // 2] * 1e-6


def steps_lib(la):
    """tools/libsteps_loop.so (the C caller of the plug-in API), or None when it is not built"""
    global _STEPS_LIB
    import ctypes
    path = os.path.join(ROOT, "tools", "libsteps_loop.so")
    if _STEPS_LIB is None and os.path.exists(path):
        _STEPS_LIB = ctypes.CDLL(path)
        _STEPS_LIB.lamm_steps_isolated_ex.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(la.Matrix),
                                                      ctypes.POINTER(la.Matrix), ctypes.c_int, ctypes.c_int,
                                                      ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                                      ctypes.c_int]
        _STEPS_LIB.lamm_read_floor.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_size_t,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                               ctypes.POINTER(ctypes.c_float)]
        _STEPS_LIB.lamm_empty_floor.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.POINTER(ctypes.c_float)]
        _STEPS_LIB.lamm_steps_direct.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(la.Matrix),
                                                 ctypes.POINTER(la.Matrix), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    return _STEPS_LIB


def read_floor(la, base_ptr, stride, R, nbytes, n):
    """median duration (s) of n isolated launches of a read-only kernel on the config-2 GEMV's grid over
    the same rotated weight bytes (tools/steps_loop.hip lamm_read_floor, timed like isolated_launches):
    what one launch of that size costs before any GEMV work -- the single-launch ceiling of DESIGN §3.1,
    measured in the driver's own run"""
    import ctypes
    if steps_lib(la) is None:
        return None
    import torch
    out = (ctypes.c_float * n)()
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    rc = _STEPS_LIB.lamm_read_floor(ctypes.c_void_p(base_ptr), stride, R, nbytes, 0, n, ctypes.c_void_p(st.cuda_stream),
                                    out)
    torch.cuda.synchronize()
    v = sorted(out)
    if rc != 0 or v[0] <= 0.0:
        log("lamm_read_floor failed:", rc, v[:3])
        return None
    return v[n // 2] * 1e-6


def empty_floor(la, grid, n):
    """median duration (s) of n isolated launches of an EMPTY kernel on `grid` workgroups of 512 threads,
    timed like isolated_launches: the dispatch's own cost, which every per-launch time above includes"""
    import ctypes
    if steps_lib(la) is None:
        return None
    import torch
    out = (ctypes.c_float * n)()
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    rc = _STEPS_LIB.lamm_empty_floor(grid, n, ctypes.c_void_p(st.cuda_stream), out)
    torch.cuda.synchronize()
    v = sorted(out)
    return v[n // 2] * 1e-6 if rc == 0 and v[0] > 0.0 else None


def time_direct(ctx, mats, R, Bm, Cm, steps, warmup, flags=0):
    """The K steps on the library's own AQL queue (lamm_hip_direct_begin / end, tools/steps_loop.hip
    lamm_steps_direct: K lamm_hip_matmul_ex calls from C in one direct region, returning once the
    last kernel completed), between the same barrier + synchronize brackets as time_steps.  Returns
    wall seconds per step (max over ranks), or None when a call did not dispatch directly."""
    import ctypes
    torch, la = ctx.torch, ctx.la
    lib = steps_lib(la)
    if lib is None:
        return None
    arr = (la.Matrix * R)(*mats)
    dev = torch.cuda.current_device()
    wall_us = ctypes.c_double()
    torch.cuda.synchronize()
    # untimed: the warm-up calls, then the timed region's own K calls once (as time_steps replays its
    # graph once untimed: the queue's cached kernarg slots then hold them, as in a decode loop's steady
    # state); the caches are flushed before the timed pass, so the weights come from HBM
    first = max(warmup, 1)
    for f0, n0 in ((0, first), (first, steps)):
        n = lib.lamm_steps_direct(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), f0,
                                  n0, dev, flags, ctypes.byref(wall_us))
        if n != n0:   # e.g. config 4's q2_K GEMV: only the flat GEMV kernels have a direct form
            log(f"direct dispatch not taken ({n} of {n0} calls direct):", la.last_error())
            return None
    flush_caches(torch)
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = lib.lamm_steps_direct(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm),
                              max(warmup, 1), steps, dev, flags, ctypes.byref(wall_us))
    torch.cuda.synchronize()
    ctx.barrier()
    wall = time.perf_counter() - t0
    if n != steps:
        log("direct dispatch: only", n, "of", steps, "steps dispatched directly")
        return None
    return ctx.max(wall / steps, 0.0)[0]


def config2_gemv(ctx, fmt, M, K, steps, warmup):
    """BASELINE config 2, strong-scaled: rank r owns rows [r0, r0 + rows) of ONE M x K weight;
    a step = its slab's GEMV on the next of R rotated weight copies + the RCCL all-gather of C."""
    torch, la = ctx.torch, ctx.la
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    kb = K // la.blck_size(t)
    arow = la.row_bytes(t, K)
    r0, rows = la.shard_rows(M, ctx.world, ctx.rank, ALIGN)
    slab_bytes = rows * arow
    R = max(8, min(4096, -(-int(1.15 * MALL_BYTES) // max(slab_bytes, 1))))
    # copy c = rows [r0, r0+rows) of the full weight made from seed c (every rank can rebuild
    # any full copy, so rank 0 can check the gathered C against one GPU computing all rows)
    A = torch.empty(R * slab_bytes + 64, dtype=torch.uint8, device="cuda")
    for c in range(R):
        gen = torch.Generator(device="cuda")
        gen.manual_seed(1000 + c)
        full, _ = make_weights(torch, la, fmt, 1, M, K, gen)
        A[c * slab_bytes:(c + 1) * slab_bytes] = full[r0 * arow:(r0 + rows) * arow]
        del full
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    B = make_activations(torch, la, fmt, 1, K, gen)
    C = torch.zeros(M, dtype=torch.float32, device="cuda")
    mats = [la.Matrix(A.data_ptr() + c * slab_bytes, t, rows, kb, kb) for c in range(R)]
    Bm = la.Matrix(B.data_ptr(), vt, kb, 1, kb)
    Cm = la.Matrix(C.data_ptr() + 4 * r0, la.F32, rows, 1, rows)

    def gemv(i):
        la.matmul(mats[i % R], Bm, Cm, torch.cuda.current_stream().cuda_stream)

    def step(i):
        gemv(i)
        ctx.allgather_rows(C, M, 1, ALIGN, torch.cuda.current_stream().cuda_stream)

    per_step, ev_step, graphed = time_steps(ctx, step, steps, warmup, graph=not ctx.rehearse, flush=True)
    # one GPU: the same K steps dispatched on the library's own AQL queue (no collective to order
    # against), reported beside the graph replay as value_direct
    direct = time_direct(ctx, mats, R, Bm, Cm, steps, warmup) if ctx.world == 1 else None
    last = warmup + steps - 1
    torch.cuda.synchronize()
    gathered = C.clone()      # C after the last timed step (copy last % R)
    check = None
    if ctx.world > 1:
        # rank 0: the gathered C of the last step vs one GPU computing all rows of that copy
        if ctx.rank == 0:
            g2 = torch.Generator(device="cuda")
            g2.manual_seed(1000 + last % R)
            full, _ = make_weights(torch, la, fmt, 1, M, K, g2)
            Cf = torch.zeros(M, dtype=torch.float32, device="cuda")
            la.matmul(la.Matrix(full.data_ptr(), t, M, kb, kb), Bm, la.Matrix(Cf.data_ptr(), la.F32, M, 1, M),
                      torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            check = "bit-exact" if torch.equal(gathered, Cf) else \
                f"MISMATCH max abs {float((gathered - Cf).abs().max()):.3e}"
    sample = {"fmt": fmt, "M": M, "N": 1, "K": K, "rows": [0, 1, M // 2, M - 1]} if ctx.world == 1 else None
    if sample is not None:   # the last step's copy: weight rows + C for the cpu_baseline leg's parity check
        a = A[(last % R) * slab_bytes:(last % R + 1) * slab_bytes].view(M, arow)
        sample.update(A=a[sample["rows"]].cpu().numpy(), B=B[:la.row_bytes(vt, K)].cpu().numpy(),
                      C=gathered[sample["rows"]].cpu().numpy())
    # the rank's kernel alone (no collective): the roofline's per-launch time.  Each launch timed
    # on its own by HIP events, the stream held until the events and the launch are all enqueued
    # (tools/steps_loop.hip lamm_steps_isolated): the device's time for one dispatch with nothing
    # queued behind it -- the duration rocprofv3's kernel trace reports for the same dispatch
    # (back-to-back launches overlap a dispatch's start with the previous one's tail, and under the
    # tracer are stretched by its own per-dispatch cost instead)
    iso = isolated_launches(la, mats, R, Bm, Cm, 300)
    b2b = isolated_launches(la, mats, R, Bm, Cm, 300, sync_each=0)
    floor = read_floor(la, A.data_ptr(), slab_bytes, R, slab_bytes, 300)
    empty = empty_floor(la, (rows + 7) // 8, 300)   # the GEMV's grid: 8 rows per 512-thread workgroup
    if iso is not None:
        kern = iso
        kern_method = ("median of 300 single launches, each completed before the next, timed by the dispatch's "
                       "own start / end timestamps (lamm_hip_profile_next -> hipExtLaunchKernel events)")
    else:
        _, kern, _ = time_steps(ctx, gemv, max(steps, 1000), 3)
        kern_method = "HIP events over 1000 back-to-back hipGraph-replayed launches on their stream"
    res = dict(per_step=per_step, direct_step=direct, ev_step=ev_step, kern=kern,
               kern_method=kern_method, kern_b2b=b2b, floor=floor, empty=empty, graphed=graphed,
               R=R, rows=rows,
               slab_bytes=slab_bytes + la.row_bytes(vt, K) + 4 * rows, gather_check=check, sample=sample)
    del A, B, C
    torch.cuda.empty_cache()
    return res


def stacked_gemv(ctx, fmt, M, K, steps):
    """33 distinct M x K slices in one launch (> MALL): the steady-state streaming rate."""
    torch, la = ctx.torch, ctx.la
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    kb = K // la.blck_size(t)
    u = gemv_bytes(la, fmt, M, K)
    sl = max(8, -(-int(1.15 * MALL_BYTES) // u))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11)
    A, arow = make_weights(torch, la, fmt, sl, M, K, gen)
    B = make_activations(torch, la, fmt, sl, K, gen)
    C = torch.zeros(sl * M, dtype=torch.float32, device="cuda")
    brow = la.row_bytes(vt, K)
    Am, Bm, Cm = la.Matrix(A.data_ptr(), t, M, kb, kb), la.Matrix(B.data_ptr(), vt, kb, 1, kb), \
        la.Matrix(C.data_ptr(), la.F32, M, 1, M)
    bt = la.Batch(sl, 1, sl, 1, M * arow, sl * M * arow, brow, sl * brow, 4 * M, 4 * M * sl)
    _, kern, _ = time_steps(ctx, lambda i: la.matmul_batched(Am, Bm, Cm, bt, torch.cuda.current_stream().cuda_stream),
                            steps, 3)
    del A, B, C
    torch.cuda.empty_cache()
    return {"workload": f"{fmt.upper()}xQ8 GEMV M={M} N=1 K={K}, {sl} distinct slices in ONE launch "
                        f"(ggml ne02=ne12={sl}, {sl * u / 1e6:.1f} MB > MALL): steady-state streaming",
            "kernel": "lamm::gemv_stream_dma_kernel (csrc/lamm_gemv.hip)", "per_launch_us": round(kern * 1e6, 3),
            "achieved_GBs": round(sl * u / kern / 1e9, 1), "frac": round(sl * u / kern / 1e9 / HBM_PEAK_GBS, 4)}


def group3_fast(ctx, fmt, M, K, steps):
    """wq|wk|wv of a decode step as the ggml boundary's sibling calls run them in the default (fast)
    order: three config-2 weights times one activation in ONE launch (lamm_hip_matmul_group ->
    gemv_flat_group_kernel), weights rotated > MALL, graph-replayed, against three single calls."""
    torch, la = ctx.torch, ctx.la
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    kb = K // la.blck_size(t)
    arow = la.row_bytes(t, K)
    R = max(9, -(-int(1.15 * MALL_BYTES) // (M * arow)))
    R -= R % 3
    gen = torch.Generator(device="cuda")
    gen.manual_seed(41)
    A, _ = make_weights(torch, la, fmt, R, M, K, gen)
    B = make_activations(torch, la, fmt, 1, K, gen)
    C3 = torch.zeros(3 * M, dtype=torch.float32, device="cuda")
    mats = [la.Matrix(A.data_ptr() + c * M * arow, t, M, kb, kb) for c in range(R)]
    Bm = la.Matrix(B.data_ptr(), vt, kb, 1, kb)
    Cs = [la.Matrix(C3.data_ptr() + 4 * M * j, la.F32, M, 1, M) for j in range(3)]
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    _, kg, _ = time_steps(ctx, lambda i: la.matmul_group([mats[(3 * i + j) % R] for j in range(3)], Bm, Cs, 0, st()),
                          max(steps, 100), 2, flush=True)

    def three(i):
        for j in range(3):
            la.matmul(mats[(3 * i + j) % R], Bm, Cs[j], st())
    _, k3, _ = time_steps(ctx, three, max(steps, 100), 2, flush=True)
    u = gemv_bytes(la, fmt, M, K)
    del A, B, C3
    torch.cuda.empty_cache()
    return {"workload": f"3 x {fmt.upper()}xQ8 GEMV M={M} N=1 K={K} per step (wq|wk|wv of a decode step), {R} weight "
                        "copies rotated, graph-replayed",
            "kernel": "lamm::gemv_flat_group_kernel (csrc/lamm_gemv_rpw.hip)", "bound": "hbm",
            "per_launch_us": round(kg * 1e6, 3), "achieved_GBs": round(3 * u / kg / 1e9, 1),
            "frac": round(3 * u / kg / 1e9 / HBM_PEAK_GBS, 4),
            "three_single_calls_us": round(k3 * 1e6, 3)}


def config3_gemm(ctx, fmt, M, N, K, slices, steps):
    """BASELINE config 3 with stationary weights: `slices` independent M x K weight slices, each
    against its own N activation rows, per launch.  N GPUs: each slice's rows split over the
    ranks + the RCCL all-gather of C (only for slices == 1).  Returns whole-launch seconds."""
    torch, la = ctx.torch, ctx.la
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    kb = K // la.blck_size(t)
    arow, brow = la.row_bytes(t, K), la.row_bytes(vt, K)
    world = ctx.world if slices == 1 else 1
    rank = ctx.rank if slices == 1 else 0
    r0, rows = la.shard_rows(M, world, rank, GEMM_ALIGN)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(21)
    full, _ = make_weights(torch, la, fmt, slices, M, K, gen)
    if world > 1:
        A = full[r0 * arow:(r0 + rows) * arow].clone()
        del full
    else:
        A = full
    B = make_activations(torch, la, fmt, slices * N, K, gen)
    C = torch.zeros(slices * N * M, dtype=torch.float32, device="cuda")
    slab = torch.zeros(max(rows, 1) * N, dtype=torch.float32, device="cuda") if world > 1 else C
    ld = rows if world > 1 else M
    bt = la.Batch(slices, 1, slices, 1, rows * arow, slices * rows * arow, N * brow, slices * N * brow, 4 * ld * N,
                  4 * ld * N * slices)
    W = la.Weights(t, A, rows, K, ne02=slices, ne03=1, nba2=rows * arow, nba3=slices * rows * arow)

    def gemm(i):
        W.matmul_torch(B, slab, N, ldc=ld, batch=bt, stream=torch.cuda.current_stream().cuda_stream)

    def step(i):
        gemm(i)
        if world > 1 and ctx.comm is not None:   # (a rehearsal times the slab alone)
            ctx.comm.allgather_rows([slab.data_ptr()], [rows], [C.data_ptr()], M, M, N, GEMM_ALIGN,
                                    [torch.cuda.current_stream().cuda_stream])

    per_step, _, _ = time_steps(ctx, step, steps, 2, graph=not ctx.rehearse)
    _, kern, _ = time_steps(ctx, gemm, max(steps, 200), 2)   # (graph start-up amortized, as for config 2)
    torch.cuda.synchronize()
    sample = None
    if world == 1 and slices == 1:
        rws = [0, 255, 2048, M - 1]
        sample = {"fmt": fmt, "M": M, "N": N, "K": K, "rows": rws,
                  "A": A.view(M, arow)[rws].cpu().numpy(), "B": B[:N * brow].cpu().numpy(),
                  "C": C.view(N, M)[:, rws].cpu().numpy()}
    W.close()
    del A, B, C, slab, W
    torch.cuda.empty_cache()
    return per_step, kern, rows, sample


def ref_order_kernels(ctx, fmt, M, N, K, steps):
    """The kernels the ggml boundary runs under LAMM_HIP_ORDER=reference (its default until round 5: the
    reference's own AVX2 float order, bit for bit), at config 2 and config 3, each against
    its own bound:
    ref_gemv_kernel against HBM (config 2's bytes, weights rotated > MALL, the dispatch's own
    timestamps); the prefill kernel against the fp32 FMA-chain floor of that order -- per output and
    32-element block 8 dependent lane FMAs, M*N*K/4 FMAs at the 157.3 TFLOP/s f32 VALU peak -- and,
    for comparison with config 3, against the i8 MFMA peak."""
    torch, la = ctx.torch, ctx.la
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    kb = K // la.blck_size(t)
    arow, brow = la.row_bytes(t, K), la.row_bytes(vt, K)
    out = {}
    R = max(8, -(-int(1.15 * MALL_BYTES) // (M * arow)))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(31)
    A, _ = make_weights(torch, la, fmt, R, M, K, gen)
    B = make_activations(torch, la, fmt, N, K, gen)
    C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
    mats = [la.Matrix(A.data_ptr() + c * M * arow, t, M, kb, kb) for c in range(R)]
    Bm1 = la.Matrix(B.data_ptr(), vt, kb, 1, kb)
    Cm1 = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
    iso = isolated_launches(la, mats, R, Bm1, Cm1, 300, flags=la.ORDER_REFERENCE)
    u = gemv_bytes(la, fmt, M, K)
    if iso:
        out["gemv"] = {"workload": f"{fmt.upper()}xQ8 GEMV M={M} N=1 K={K} (config 2), {R} weight copies rotated",
                       "kernel": "lamm::ref_gemv_kernel (csrc/lamm_ref.hip)", "bound": "hbm",
                       "per_launch_us": round(iso * 1e6, 3), "achieved_GBs": round(u / iso / 1e9, 1),
                       "frac": round(u / iso / 1e9 / HBM_PEAK_GBS, 4)}
    # llama.cpp's decode through the boundary runs wq / wk / wv as ONE grouped launch (sibling calls,
    # lamm_hip_matmul_group -> ref_gemv_group_kernel): three config-2 weights per step,
    # rotated over the copies, graph-replayed
    if R >= 3 and t in (la.Q4_0, la.Q4_1, la.Q5_0, la.Q5_1):
        C3 = torch.zeros(3 * M, dtype=torch.float32, device="cuda")
        Cs3 = [la.Matrix(C3.data_ptr() + 4 * M * j, la.F32, M, 1, M) for j in range(3)]
        _, kg, _ = time_steps(ctx, lambda i: la.matmul_group([mats[(3 * i + j) % R] for j in range(3)], Bm1, Cs3,
                                                             la.ORDER_REFERENCE, torch.cuda.current_stream().cuda_stream),
                              max(steps, 100), 2)
        out["gemv_group3"] = {"workload": f"3 x {fmt.upper()}xQ8 GEMV M={M} N=1 K={K} in one launch (wq|wk|wv of a decode "
                                          f"step), {R} weight copies rotated",
                              "kernel": "lamm::ref_gemv_group_kernel (csrc/lamm_ref.hip)", "bound": "hbm",
                              "per_launch_us": round(kg * 1e6, 3), "achieved_GBs": round(3 * u / kg / 1e9, 1),
                              "frac": round(3 * u / kg / 1e9 / HBM_PEAK_GBS, 4)}
        del C3
    BmN = la.Matrix(B.data_ptr(), vt, kb, N, kb)
    CmN = la.Matrix(C.data_ptr(), la.F32, M, N, M)
    _, kern, _ = time_steps(ctx, lambda i: la.matmul_ex(mats[0], BmN, CmN, flags=la.ORDER_REFERENCE,
                                                        stream=torch.cuda.current_stream().cuda_stream),
                            max(steps, 100), 2)
    floor = M * N * K / 4 * 2 / (F32_VALU_PEAK_TFLOPS * 1e12)
    out["gemm"] = {"workload": f"{fmt.upper()}xQ8 GEMM M={M} N={N} K={K} (config 3), stationary weights",
                   "kernel": "lamm::ref_mfma2_kernel<swizzled, interleaved> (csrc/lamm_ref.hip)" if fmt in ("q4_0", "q5_0")
                   else "lamm::ref_mfma2_kernel<swizzled> (csrc/lamm_ref.hip)" if fmt == "q4_1"
                   else "lamm::ref_mfma_kernel (csrc/lamm_ref.hip)",
                   "bound": "valu (the reference's fp32 lane chains)", "per_launch_us": round(kern * 1e6, 2),
                   "floor_us": round(floor * 1e6, 2), "frac": round(floor / kern, 4),
                   "floor": f"M*N*K/4 fp32 FMAs (8 lane chains per output and block) at {F32_VALU_PEAK_TFLOPS} TFLOP/s",
                   "i8_frac": round(2.0 * M * N * K / kern / 1e12 / I8_DENSE_PEAK_TOPS, 4)}
    del A, B, C
    torch.cuda.empty_cache()
    return out


def config1_f32(ctx, steps):
    """BASELINE config 1: F32 M=N=K=512 (la-benchmark-matmult's plumbing shape) on the GPU's F32
    path (the dense prefill GEMM), hipGraph-replayed, inputs resident."""
    torch, la = ctx.torch, ctx.la
    n = 512
    gen = torch.Generator(device="cuda")
    gen.manual_seed(512)
    A = torch.randn(n * n, device="cuda", generator=gen)
    B = torch.randn(n * n, device="cuda", generator=gen)
    C = torch.zeros(n * n, device="cuda")
    Am, Bm, Cm = la.Matrix(A.data_ptr(), la.F32, n, n, n), la.Matrix(B.data_ptr(), la.F32, n, n, n), \
        la.Matrix(C.data_ptr(), la.F32, n, n, n)
    _, kern, _ = time_steps(ctx, lambda i: la.matmul(Am, Bm, Cm, torch.cuda.current_stream().cuda_stream),
                            max(steps, 200), 3)
    ref = (B.view(n, n) @ A.view(n, n).T).reshape(-1)
    err = float((C - ref).abs().max() / ref.abs().max())
    del A, B, C
    return {"workload": "F32 M=N=K=512 (BASELINE config 1, la-benchmark-matmult -d f32 shape), one call per step",
            "kernel": "lamm::gemm_dense_kernel (csrc/lamm_gemm_dense.hip)", "per_launch_us": round(kern * 1e6, 3),
            "GFLOPS": round(2.0 * n ** 3 / kern / 1e9, 1), "max_rel_err_vs_torch_fp32": err}


def llama_step_sharded(ctx, fmt):
    """Config 5's weight matmuls with every weight's rows sharded over the job's ranks: one
    llama-matmul-bench process per GPU (--rank / --world / --comm-id; RCCL all-gather of every
    projection's output, the whole step one hipGraph per process).  Returns rank 0's view with the
    step time maxed over ranks."""
    exe = os.path.join(ROOT, "la-llama.cpp_amd", "llama-matmul-bench")
    out = {"note": f"weight rows sharded over {ctx.world} GPU(s), one process per GPU, RCCL all-gather after every "
                   "projection (hipGraph per process); synthetic weights, weight matmuls only"}
    for name, argv in (("decode_n1_batch_proj", ["-n", "1", "-i", "50", "--batch-proj"]),
                       ("prefill_n512", ["-n", "512", "-i", "5", "-s", "--batch-proj"])):
        res = {}
        # a fresh RCCL unique id per communicator: an id's bootstrap root serves ONE init
        uid = [ctx.la.comm_unique_id().hex() if ctx.rank == 0 else None]
        if ctx.world > 1:
            ctx.dist.broadcast_object_list(uid, src=0)
        try:
            r = subprocess.run([exe, "-d", fmt, "--rank", str(ctx.rank), "--world", str(ctx.world), "--comm-id", uid[0],
                                "--device", str(ctx.device)] + argv, capture_output=True, text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            res = json.loads(line[-1]) if r.returncode == 0 and line else {"error": r.stderr[-300:]}
        except Exception as e:  # noqa: BLE001
            res = {"error": str(e)[:300]}
        ms = res.get("ms_per_step", float("inf"))
        (ms_max,) = ctx.max(ms)
        if "error" not in res:
            if ms_max != ms_max or ms_max == float("inf"):   # another rank failed
                res["error"] = "a rank failed: no step time from every rank"
            else:
                res["ms_per_step_max_over_ranks"] = round(ms_max, 4)
                res["tok_per_s"] = round(res["tokens_per_step"] / (ms_max * 1e-3), 2)
        out[name] = res
    return out


def cpu_baseline(fmt, M, N, K, budget_s, unit_bytes):
    """The real reference (lamm opt=3, AVX2; Q8_0 uses opt=0 stock ggml because lamm's AVX2 Q8_0
    is numerically wrong) timed like la-benchmark-matmult."""
    threads, cores_src = host_cores()
    variant = "lamm0" if fmt == "q8_0" else "lamm3"
    exe = os.path.join(ROOT, "oracle", "_ref", f"ref_driver_{variant}")
    if os.path.exists(exe):
        out = subprocess.run([exe, "bench", fmt, str(M), str(N), str(K), str(threads), "100000", str(budget_s)],
                             capture_output=True, text=True, timeout=budget_s * 4 + 120)
        if out.returncode == 0:
            r = json.loads(out.stdout.strip().splitlines()[-1])
            us = r["median_us"]
            return {"value": round(unit_bytes / (us * 1e-6) / 1e9, 3), "unit": "GB/s", "cores": threads,
                    "cores_source": cores_src,
                    "kind": "reference", "median_us": us, "gflops": r["gflops"],
                    "sample": f"{r['iters']} x {fmt} mul_mat M={M} N={N} K={K} via ggml_graph_compute "
                              f"(ref_driver_{variant}: la-llama.cpp lamm opt {3 if variant == 'lamm3' else 0} "
                              f"AVX2 build; INIT quantization of src1 included), median, ~{budget_s}s budget"}
        log("reference baseline failed:", out.stderr[-500:])
    # fallback: our scalar C port of the reference arithmetic, one thread
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib as ol
    o = ol.Oracle()
    t = ol.BY_NAME[fmt]
    rng = np.random.default_rng(0)
    A = o.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    B = o.quantize(o.vec_dot_type(t), rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX)
    ts, t_end = [], time.perf_counter() + budget_s
    while time.perf_counter() < t_end and len(ts) < 50:
        t0 = time.perf_counter()
        o.mul_mat(t, M, N, K, A, B)
        ts.append(time.perf_counter() - t0)
    med = sorted(ts)[len(ts) // 2]
    return {"value": round(unit_bytes / med / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "median_us": med * 1e6, "sample": f"{len(ts)} x scalar oracle mul_mat M={M} N={N} K={K}"}


def parity_sample(samples):
    """cpu_baseline leg: the GPU's outputs for sampled rows (last timed step) vs the oracle,
    |c - ref| / max(|ref|, sum |a b|)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib as ol
    o = ol.Oracle()
    out = {}
    for name, s in samples.items():
        if not s:
            continue
        t = ol.BY_NAME[s["fmt"]]
        vt = o.vec_dot_type(t)
        n, K, rows = s["N"], s["K"], s["rows"]
        A = np.ascontiguousarray(s["A"]).reshape(-1)
        ref = o.mul_mat(t, len(rows), n, K, A, s["B"])
        Ad = o.dequantize(t, A, len(rows), K).astype(np.float64)
        Bd = o.dequantize(vt, s["B"], n, K).astype(np.float64)
        denom = np.maximum(np.abs(Bd) @ np.abs(Ad).T, np.abs(ref)) + 1e-30
        got = np.asarray(s["C"], np.float64).reshape(n, len(rows))
        err = float((np.abs(got - ref) / denom).max())
        out[name] = {"rows": rows, "columns": n, "max_rel_err": err, "ok": err < 1e-3}
    return out


def llama_e2e(devices, n_prompt=512, n_gen=128, threads=16, exe=None, extra_env=None, timeout=600, keep_tokens=False,
              extra_args=()):
    """BASELINE config 5 through llama.cpp-b2430's own llama_decode (see module doc)."""
    exe = exe or os.path.join(ROOT, "integration", "_build", "llama_e2e_hip")
    model = os.path.join(os.environ.get("TMPDIR", "/tmp"), "lamm_synth_llama7b_q4_0.gguf")
    if not os.path.exists(exe):
        return {"error": f"{exe} missing (build with __graft_entry__.build())"}
    env = dict(os.environ, **(extra_env or {}))
    if devices:
        env["LAMM_HIP_DEVICES"] = ",".join(map(str, devices))
    try:
        r = subprocess.run([exe, "-m", model, "-t", str(threads), "-p", str(n_prompt), "-n", str(n_gen), *extra_args],
                           capture_output=True, text=True, timeout=timeout, env=env)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not line:
            return {"error": r.stderr[-400:]}
        d = json.loads(line[-1])
        if not keep_tokens:
            d.pop("tokens", None)
            d.pop("argmax", None)
        return d
    except Exception as e:  # noqa: BLE001 -- reported, never fatal for the main bench line
        return {"error": str(e)[:300]}


def llama_step(fmt):
    """The model's weight matmuls through the device API, hipGraph-replayed (llama-matmul-bench)."""
    exe = os.path.join(ROOT, "la-llama.cpp_amd", "llama-matmul-bench")
    res = {"note": "weight matmuls (and with ctx512 the attention matmuls; no softmax / norms / RoPE), "
                   "synthetic weights, hipGraph replay: the ceiling without the ggml boundary's host round trips"}
    # decode_n1: llama.cpp's 7 projection tensors per layer, one launch each; decode_n1_batch_proj:
    # q|k|v and gate|up stored as one tensor each (4 launches per layer, a GPU-native layout)
    for name, argv in (("decode_n1", ["-n", "1", "-i", "50"]),
                       ("decode_n1_batch_proj", ["-n", "1", "-i", "50", "--batch-proj"]),
                       ("prefill_n512", ["-n", "512", "-i", "5", "-s"]),
                       # every mul_mat of a decode step incl. KQ / KQV over a device-resident F16 KV
                       # cache of 512 cells per layer (the fully-GPU decode step)
                       ("decode_n1_batch_proj_ctx512", ["-n", "1", "-i", "50", "--batch-proj", "--ctx", "512"])):
        try:
            r = subprocess.run([exe, "-d", fmt] + argv, capture_output=True, text=True, timeout=180)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            res[name] = json.loads(line[-1]) if r.returncode == 0 and line else {"error": r.stderr[-300:]}
        except Exception as e:  # noqa: BLE001
            res[name] = {"error": str(e)[:300]}
    return res


def la_benchmark(dtype="q4_0", gpu_threads=4, iters=10):
    """The reference's OWN benchmark, src/la-benchmark-matmult.cpp compiled unchanged (integration/Makefile
    la-benchmark-matmult_hip: its ggml hook -> liblamm_hip.so), at its default shape (K=11008, M=4096,
    N=128, la-benchmark-matmult.cpp:180-182), beside the same source built as the reference builds it
    (oracle/_ref/la-benchmark-matmult_lamm3: lamm opt-3 AVX2) on this host's cores.  `Average` is the
    reference's own figure (test/test_matmult_performance.py:42); the GPU's first iteration includes the
    weight's upload into the device cache."""
    import re
    pat = re.compile(r"\nAverage\s*(\d+\.\d+)\n")
    row = re.compile(r"^\s*\d+;\s*\d+;.*;\s*(\d+);\s*(\d+\.\d+)$", re.M)
    out = {"workload": f"la-benchmark-matmult -d {dtype} -i {iters}: ggml_mul_mat of ({dtype} 4096 x 11008) x (F32 11008 "
                       "x 128), ggml INIT quantization of src1 included, the binary's own Average GFLOPS"}
    cores = host_cores()[0]
    for name, exe, th in (("gpu", os.path.join(ROOT, "integration", "_build", "la-benchmark-matmult_hip"), gpu_threads),
                          ("cpu_reference", os.path.join(ROOT, "oracle", "_ref", "la-benchmark-matmult_lamm3"), cores)):
        if not os.path.exists(exe):
            out[name] = {"error": f"{exe} missing"}
            continue
        try:
            r = subprocess.run([exe, "-d", dtype, "-t", str(th), "-i", str(iters)], capture_output=True, text=True,
                               timeout=300)
            m = pat.search(r.stdout)
            if r.returncode != 0 or not m:
                out[name] = {"error": (r.stdout + r.stderr)[-300:]}
                continue
            us = sorted(int(u) for u, _ in row.findall(r.stdout))
            out[name] = {"average_GFLOPS": float(m.group(1)), "threads": th,
                         "median_iteration_us": us[len(us) // 2] if us else None,
                         "binary": os.path.relpath(exe, ROOT)}
        except Exception as e:  # noqa: BLE001
            out[name] = {"error": str(e)[:300]}
    return out


def read_profile(kind, tag):
    """A committed per-launch measurement of config 2's kernel (profiles/<kind>_<tag>.json): the
    PMC traffic (tools/pmc_traffic_flat1.py) or the kernel tracer's paced durations
    (tools/kt_roofline.py), both written by tools/roofline_trace.sh."""
    p = os.path.join(ROOT, "profiles", f"{kind}_{tag}.json")
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except Exception:
            return None
    return None


def summary(out):
    """The headline kernels in a few keys (per-launch us and roofline fraction), printed as the LAST key
    of the JSON line so that a tail of the output still shows config 3 and the boundary's
    reference-order kernels."""
    s = {"config2_gemv": {"kernel": "gemv_flat1_kernel", "us": out["roofline"]["per_launch_us"],
                          "frac_hbm": out["roofline"]["frac"], "value_GBs": out["value"]}}
    st = out.get("gemv_stacked", {})
    if "per_launch_us" in st:   # the same GEMV, 33 weight slices in one launch: the streaming rate
        s["config2_gemv_stacked"] = {"kernel": "gemv_stream_dma_kernel", "us": st["per_launch_us"],
                                     "frac_hbm": st["frac"], "achieved_GBs": st["achieved_GBs"]}
    g3 = out.get("gemv_group3", {})
    if "per_launch_us" in g3:
        s["gemv_group3"] = {"kernel": "gemv_flat_group_kernel", "us": g3["per_launch_us"], "frac_hbm": g3["frac"],
                            "three_single_calls_us": g3["three_single_calls_us"]}
    gm = out.get("gemm", {}).get("slices1", {})
    if "roofline" in gm:
        s["config3_gemm"] = {"engine": gm["engine"], "us": gm["roofline"]["per_launch_us"],
                             "frac_i8": gm["roofline"]["frac"], "scope": "whole launch"}
    ro = out.get("ref_order", {})
    if "gemv" in ro:
        s["ref_order_gemv"] = {"kernel": "ref_gemv_kernel", "us": ro["gemv"]["per_launch_us"], "frac_hbm": ro["gemv"]["frac"]}
    if "gemv_group3" in ro:
        s["ref_order_gemv_group3"] = {"kernel": "ref_gemv_group_kernel", "us": ro["gemv_group3"]["per_launch_us"],
                                      "frac_hbm": ro["gemv_group3"]["frac"]}
    if "gemm" in ro:
        s["ref_order_gemm"] = {"kernel": ro["gemm"]["kernel"].split(" ")[0].split("::")[-1], "us": ro["gemm"]["per_launch_us"],
                               "frac_fma_floor": ro["gemm"]["frac"], "frac_i8": ro["gemm"]["i8_frac"]}
    c4 = out.get("config4", {})
    for f in ("q4_1", "q5_0", "q5_1", "q8_0", "q2_k"):
        e = c4.get(f, {})
        if "gemv_per_launch_us" in e:
            s[f] = {"gemv_us": e["gemv_per_launch_us"], "gemv_frac": e["gemv_frac"]}
            if "gemm_per_launch_us" in e:
                s[f].update({"gemm": e["gemm_engine"], "gemm_us": e["gemm_per_launch_us"], "gemm_frac": e["gemm_frac"]})
    lb = out.get("la_benchmark", {})
    if "average_GFLOPS" in lb.get("gpu", {}):
        s["la_benchmark_q4_0"] = {"gpu_GFLOPS": lb["gpu"]["average_GFLOPS"],
                                  "cpu_reference_GFLOPS": lb.get("cpu_reference", {}).get("average_GFLOPS")}
    e2e = out.get("llama7b_e2e", {})
    for k in ("t16", "t8", "t4_numa_isolate", "t16_reference_order"):
        r = e2e.get(k, {})
        if "pp_tok_s" in r:
            s[f"config5_{k}"] = {kk: r.get(kk) for kk in ("pp_tok_s", "tg_tok_s", "tg_from_empty_tok_s")}
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)   # 200 x ~4 us: the graph replay's start-up amortized
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--fmt", default="q4_0")
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--gemm-N", type=int, default=512)
    ap.add_argument("--no-gemm", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-llama", action="store_true", help="skip config 5 (llama e2e + weight-matmul step)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--sweep", action="store_true", help="also every weight format's stacked GEMV + GEMM")
    ap.add_argument("--no-config1", action="store_true", help="skip config 1 (F32 512^3)")
    ap.add_argument("--no-config4", action="store_true", help="skip config 4 (the per-format sweep)")
    args = ap.parse_args()

    import torch
    import lamm_amd as la

    if la.device_count() == 0:
        raise SystemExit("bench.py: no gfx950 device visible")
    ctx = Ctx(torch, la)
    world, rank = ctx.world, ctx.rank
    M, K, fmt = args.M, args.K, args.fmt
    unit = gemv_bytes(la, fmt, M, K)

    g = config2_gemv(ctx, fmt, M, K, args.steps, args.warmup)
    value = unit / g["per_step"] / 1e9
    achieved = g["slab_bytes"] / g["kern"] / 1e9
    traffic = read_profile("traffic", f"{fmt}_gemv_single")
    trace = read_profile("roofline", f"{fmt}_gemv_single")
    kname = "gemv_flat1_kernel" if la.gemm_engine(fmt, g["rows"], 1, K) == "gemv" and K == 4096 else None
    out = {
        "metric": "Q4_0xQ8_0 GEMM effective GFLOPS @ K=4096; achieved HBM GB/s (GEMV)",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(g["per_step"] * 1e3, 5), "gpu_ms_per_step": round(g["ev_step"] * 1e3, 5),
        "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "i8",
        "data": "synthetic (random block bytes with valid fp16 scales; B = GPU q8 quantizer of N(0,1))",
        "config": {"workload": f"{fmt.upper()}xQ8 GEMV M={M} N=1 K={K} (BASELINE config 2): ONE call per step, "
                               f"rotating over {g['R']} weight copies per rank (> 256 MiB MALL)"
                               + (f"; rows split over {world} GPUs ({g['rows']} on rank 0) + RCCL all-gather of C "
                                  f"every step" if world > 1 else ""),
                   "fmt": fmt, "M": M, "N": 1, "K": K, "rows_per_rank": g["rows"],
                   "parallelism": f"rows of A split over {world} GPU(s)" +
                                  ((" + all-gather through gloo (one-GPU rehearsal)" if ctx.rehearse else
                                    " + lamm_hip_allgather_rows (RCCL)") if world > 1 else ""),
                   "timing": "hipGraph of the K steps, replayed" if g["graphed"] else "eager launches"},
        # the same K steps as K calls from C on the library's own AQL queue (lamm_hip_direct_begin /
        # end: one packet per call, one completion signal for the region), same brackets
        "value_direct": round(unit / g["direct_step"] / 1e9, 2) if g["direct_step"] else None,
        "ms_per_step_direct": round(g["direct_step"] * 1e3, 5) if g["direct_step"] else None,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic.get("bytes_per_launch") if traffic and traffic.get(
                         "algorithmic_bytes_per_launch") == g["slab_bytes"] and traffic.get("kernel") == kname
                     else None,
                     "traffic_source": f"profiles/traffic_{fmt}_gemv_single.json (rocprofv3 --pmc FETCH_SIZE + "
                                       "WRITE_SIZE passes of tools/pmc_flat1.py, FETCH calibrated on a 312 MB launch "
                                       "of the same body, per launch)",
                     "kernel": "lamm::gemv_flat1_kernel (csrc/lamm_gemv_rpw.hip; gemv_rpw_kernel for other shapes)",
                     "per_launch_us": round(g["kern"] * 1e6, 3),
                     "per_launch_method": g["kern_method"],
                     "per_launch_us_back_to_back": round(g["kern_b2b"] * 1e6, 3) if g["kern_b2b"] else None,
                     # a read-only kernel on the same grid over the same weight bytes, timed the same way:
                     # what a single launch of this size can reach (tools/steps_loop.hip read_floor_kernel)
                     "single_launch_floor_us": round(g["floor"] * 1e6, 3) if g["floor"] else None,
                     "single_launch_floor_frac": round(g["slab_bytes"] / g["floor"] / 1e9 / HBM_PEAK_GBS, 4)
                     if g["floor"] else None,
                     # an EMPTY kernel on the same grid, timed the same way: the dispatch's own cost
                     "empty_launch_us": round(g["empty"] * 1e6, 3) if g["empty"] else None,
                     "algorithmic_bytes_per_launch": g["slab_bytes"]},
    }
    if trace and kname and trace.get("algorithmic_bytes_per_launch") == g["slab_bytes"]:
        # the kernel tracer's own durations of the same kernel, launched one at a time (the tracer
        # stretches back-to-back dispatches by its own per-dispatch cost)
        tm = trace["duration_us"]["median"]
        out["roofline"]["rocprof_paced"] = {
            "file": f"profiles/roofline_{fmt}_gemv_single.json", "median_us": tm,
            "frac_at_median": round(g["slab_bytes"] / (tm * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "events_over_trace": round(g["kern"] * 1e6 / tm, 4)}
    if g["gather_check"] is not None:
        out["config"]["gather_check"] = g["gather_check"]
    samples = {"gemv_config2": g["sample"]}
    extras = {}
    try:
        if world == 1:
            extras["gemv_stacked"] = stacked_gemv(ctx, fmt, M, K, max(5, args.steps // 2))
    except Exception as e:  # noqa: BLE001
        extras["gemv_stacked"] = {"error": str(e)[:300]}
    try:
        if world == 1:
            extras["gemv_group3"] = group3_fast(ctx, fmt, M, K, args.steps)
    except Exception as e:  # noqa: BLE001
        extras["gemv_group3"] = {"error": str(e)[:300]}
    if not args.no_gemm:
        gN = args.gemm_N
        gm = {}
        for gslices in ((4, 1) if world == 1 else (1,)):
            try:
                step, kern, rows, smp = config3_gemm(ctx, fmt, M, gN, K, gslices, max(3, args.steps // 4))
                ops = 2.0 * M * gN * K * gslices
                rops = 2.0 * rows * gN * K * gslices
                engine = la.gemm_engine(fmt, rows, gN, K, gslices, stationary=True)
                gm[f"slices{gslices}"] = {
                    "workload": f"{fmt.upper()}xQ8 GEMM M={M} N={gN} K={K} (BASELINE config 3), {gslices} slice(s) "
                                f"per launch, stationary weights" +
                                (f"; rows split over {world} GPUs + RCCL all-gather of C" if world > 1 and gslices == 1
                                 else ""),
                    "engine": engine, "value": round(ops / step / 1e9, 1), "unit": "GFLOPS",
                    "ms_per_step": round(step * 1e3, 4),
                    "roofline": {"bound": "mfma", "scope": "whole launch of this rank's slab (dq16: the one "
                                                           "kernel; exact engines: activation prep + main loop + "
                                                           "split-K reduce)",
                                 "kernel": GEMM_KERNELS.get(engine, engine),
                                 "achieved": round(rops / kern / 1e12, 2), "peak": I8_DENSE_PEAK_TOPS,
                                 "unit": "TFLOP/s", "frac": round(rops / kern / 1e12 / I8_DENSE_PEAK_TOPS, 4),
                                 "per_launch_us": round(kern * 1e6, 2)}}
                if smp:
                    samples["gemm_config3"] = smp
            except Exception as e:  # noqa: BLE001
                gm[f"slices{gslices}"] = {"error": str(e)[:300]}
        extras["gemm"] = gm
        if world == 1:
            try:
                extras["ref_order"] = ref_order_kernels(ctx, fmt, M, gN, K, max(3, args.steps // 4))
            except Exception as e:  # noqa: BLE001
                extras["ref_order"] = {"error": str(e)[:300]}
    if world == 1 and not args.no_config1:
        try:
            extras["config1"] = config1_f32(ctx, args.steps)
        except Exception as e:  # noqa: BLE001
            extras["config1"] = {"error": str(e)[:300]}
    if world == 1 and not args.no_config4:
        c4 = {"workload": "BASELINE config 4: per format, ONE M=4096 N=1 K=4096 GEMV per step (config 2's "
                          "measurement, weights rotated > MALL) and the M=4096 N=512 K=4096 GEMM (config 3's, "
                          "stationary weights, whole launch)"}
        for f in ("q4_1", "q5_0", "q5_1", "q8_0", "q2_k"):
            try:
                g4 = config2_gemv(ctx, f, M, K, args.steps, args.warmup)
                ent = {"gemv_per_launch_us": round(g4["kern"] * 1e6, 3),
                       "gemv_GBs": round(g4["slab_bytes"] / g4["kern"] / 1e9, 1),
                       "gemv_frac": round(g4["slab_bytes"] / g4["kern"] / 1e9 / HBM_PEAK_GBS, 4),
                       "gemv_bytes": g4["slab_bytes"]}
                if not args.no_gemm:
                    _, kern4, _, _ = config3_gemm(ctx, f, M, args.gemm_N, K, 1, max(3, args.steps // 4))
                    ops4 = 2.0 * M * args.gemm_N * K
                    ent.update({"gemm_engine": la.gemm_engine(f, M, args.gemm_N, K, 1, stationary=True),
                                "gemm_per_launch_us": round(kern4 * 1e6, 2),
                                "gemm_TFLOPs": round(ops4 / kern4 / 1e12, 2),
                                "gemm_frac": round(ops4 / kern4 / 1e12 / I8_DENSE_PEAK_TOPS, 4)})
                c4[f] = ent
            except Exception as e:  # noqa: BLE001
                c4[f] = {"error": str(e)[:200]}
        extras["config4"] = c4
    if args.sweep and world == 1:
        sw = {}
        for f in ["f32", "f16", "q4_0", "q4_1", "q5_0", "q5_1", "q8_0", "q2_k", "q4_k", "q5_k", "q6_k"]:
            try:
                st = stacked_gemv(ctx, f, M, K, max(5, args.steps // 2))
                sw[f] = {"gemv_stacked_GBs": st["achieved_GBs"]}
                if not args.no_gemm:
                    step, kern, _, _ = config3_gemm(ctx, f, M, args.gemm_N, K, 1, max(3, args.steps // 4))
                    sw[f].update({"gemm_GFLOPS": round(2.0 * M * args.gemm_N * K / kern / 1e9, 1),
                                  "gemm_us": round(kern * 1e6, 2),
                                  "gemm_engine": la.gemm_engine(f, M, args.gemm_N, K, 1, stationary=True)})
            except Exception as e:  # noqa: BLE001
                sw[f] = {"error": str(e)[:200]}
        extras["sweep"] = sw
    if rank == 0 and world == 1:
        extras["la_benchmark"] = la_benchmark(fmt)
    if not args.no_llama:
        extras["llama7b_matmul_step_sharded"] = llama_step_sharded(ctx, fmt)
        ctx.barrier()
        if rank == 0:
            devs = list(range(world)) if world > 1 and not ctx.rehearse else None
            e2e = {"note": "BASELINE config 5: llama.cpp-b2430's own llama_decode (integration/_build/llama_e2e_hip: "
                           "the reference's llama.cpp + ggml, LA_LLAMA hook -> liblamm_hip.so), synthetic "
                           "Llama-7B-shaped Q4_0 GGUF (Q6_K output, F16 KV cache), pp512 then tg128 greedy behind the "
                           "prompt (tg_tok_s), and llama-bench's own tg128 from an empty cache "
                           "(tg_from_empty_tok_s, examples/llama-bench/llama-bench.cpp:1234-1254); "
                           "weights device-resident after a warm-up pass; reference published (3A6000, 4 threads, "
                           "README.md:684,710): prompt 8.27 tok/s, text-gen 4.69 tok/s",
                   "devices": devs or [ctx.device],
                   "t16": llama_e2e(devs, threads=min(16, host_cores()[0])),
                   # the GPU build leaves ggml fewer CPU ops: 8 pool threads spin less against the
                   # boundary's thread (short-context decode 69 -> 97 tok/s, profiles/r03/boundary/)
                   "t8": llama_e2e(devs, threads=min(8, host_cores()[0])),
                   # the reference's own headline thread count (4), ggml's threads kept on one NUMA node
                   # (llama.cpp --numa isolate): with the matmuls on the GPU, ggml's per-node barriers
                   # cost more than extra threads save (profiles/r05/decode_threads/)
                   "t4_numa_isolate": llama_e2e(devs, threads=min(4, host_cores()[0]),
                                                extra_args=("--numa", "isolate")),
                   # the boundary runs the fast engines by default (round 6); in the reference's own
                   # float order (LAMM_HIP_ORDER=reference: bit-identical logits) for comparison
                   "t16_reference_order": llama_e2e(devs, threads=min(16, host_cores()[0]),
                                                    extra_env={"LAMM_HIP_ORDER": "reference"}),
                   "float_order": "fast engines (the default): t16 / t8 / t4; t16_reference_order: "
                                  "LAMM_HIP_ORDER=reference"}
            if world == 1:
                extras["llama7b_matmul_step"] = llama_step(fmt)
            extras["llama7b_e2e"] = e2e
        ctx.barrier()
    out.update(extras)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(fmt, M, 1, K, args.cpu_budget, unit)
        out["cpu_baseline"]["parity_sample"] = parity_sample(samples)
        if "gemm" in out:   # the same reference path at BASELINE config 3
            cb = cpu_baseline(fmt, M, args.gemm_N, K, args.cpu_budget, 0)
            us = cb["median_us"]
            out["gemm"]["cpu_baseline"] = {
                "value": round(2.0 * M * args.gemm_N * K / (us * 1e-6) / 1e9, 2), "unit": "GFLOPS",
                "cores": cb["cores"], "kind": cb["kind"], "median_us": round(us, 1), "sample": cb["sample"]}
        if "config1" in out and "error" not in out["config1"]:   # the reference's CPU path at config 1
            cb = cpu_baseline("f32", 512, 512, 512, min(args.cpu_budget, 5.0), 0)
            us = cb["median_us"]
            out["config1"]["cpu_baseline"] = {"value": round(2.0 * 512 ** 3 / (us * 1e-6) / 1e9, 2), "unit": "GFLOPS",
                                              "cores": cb["cores"], "kind": cb["kind"], "median_us": round(us, 1),
                                              "sample": cb["sample"]}
        if "llama7b_e2e" in out:   # the reference's own llama.cpp + lamm opt-3 on the host cores
            ref_exe = os.path.join(ROOT, "oracle", "_ref", "llama_e2e_lamm3")
            cpu = llama_e2e(None, n_prompt=512, n_gen=128, threads=out["cpu_baseline"]["cores"], exe=ref_exe)
            cpu["sample"] = "pp512 + tg128 (the GPU run's workload) of the same model and driver on la-llama.cpp lamm " \
                            "opt 3 AVX2"
            out["llama7b_e2e"]["cpu_baseline"] = cpu
            # parity of the full 32-layer model, teacher-forced (every build fed the reference's greedy
            # tokens, so each logits row comes from the same context): pp64 / tg16
            tmp = os.environ.get("TMPDIR", "/tmp")
            lc, lg = os.path.join(tmp, "lamm_e2e_ref.bin"), os.path.join(tmp, "lamm_e2e_gpu.bin")
            c = llama_e2e(None, n_prompt=64, n_gen=16, threads=out["cpu_baseline"]["cores"], exe=ref_exe,
                          keep_tokens=True, extra_args=("--logits", lc))
            par = {"run": "pp64 + tg16, same synthetic 32-layer model: llama_e2e_lamm3 (reference) greedy, then "
                          "llama_e2e_hip teacher-forced with the reference's tokens (--force)"}
            if c.get("tokens"):
                import numpy as np
                a = np.fromfile(lc, np.float32).reshape(-1, 32000)
                par.update({"tokens_reference": c["tokens"], "argmax_reference": c["argmax"], "rows": len(c["argmax"]),
                            "reference_own_spread": "scalar vs AVX2 lamm builds of the reference, same forced run: "
                                                    "max 0.0949 per row, argmax agree 15 of 17 "
                                                    "(profiles/r03/e2e_32_layers.txt)"})
                # the default build (fast engines) and LAMM_HIP_ORDER=reference (bit-identical expected)
                for key, env in (("default_fast_order", None), ("reference_order", {"LAMM_HIP_ORDER": "reference"})):
                    g = llama_e2e(None, n_prompt=64, n_gen=16, threads=min(16, host_cores()[0]), keep_tokens=True,
                                  extra_env=env, extra_args=("--logits", lg, "--force", ",".join(map(str, c["tokens"]))))
                    if g.get("argmax"):
                        b = np.fromfile(lg, np.float32).reshape(-1, 32000)
                        err = np.abs(b - a).max(axis=1) / np.abs(a).max(axis=1)
                        par[key] = {"argmax_gpu": g["argmax"],
                                    "argmax_agree": sum(x == y for x, y in zip(g["argmax"], c["argmax"])),
                                    "max_rel_dlogit_per_row": [round(float(e), 4) for e in err],
                                    "bit_identical_logits": bool(np.array_equal(a.view(np.uint32), b.view(np.uint32)))}
                    else:
                        par[key] = {"error": g.get("error")}
            else:
                par["error"] = c.get("error")
            out["llama7b_e2e"]["parity_32_layers"] = par
    ctx.close()
    if rank == 0:
        out["summary"] = summary(out)   # last key: what a tail of the line keeps
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

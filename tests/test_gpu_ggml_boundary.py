"""The drop-in boundary on the GPU: lamm_can_mul_mat / lamm_mul_mat driven exactly as
ggml_compute_forward_mul_mat drives the reference plug-in (tests/ggml_emu.py)."""
import ctypes

import numpy as np
import pytest

from conftest import rel_err
import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
import ggml_emu  # noqa: E402

ORACLE = ol.Oracle()


def make_node(t, M, N, K, ne2=(1, 1), ne3=(1, 1), seed=0, transpose_free=True):
    """src0 [K, M, ne02, ne03] of type t, src1 F32 [K, N, ne12, ne13]."""
    rng = np.random.default_rng(seed)
    n0 = ne2[0] * ne3[0]
    n1 = ne2[1] * ne3[1]
    a = rng.standard_normal((n0 * M, K), dtype=np.float32)
    b = rng.standard_normal((n1 * N, K), dtype=np.float32)
    A_q = ORACLE.quantize(t, a)
    src0 = ggml_emu.Tensor(t, [K, M, ne2[0], ne3[0]], data=A_q)
    src1 = ggml_emu.Tensor(ol.F32, [K, N, ne2[1], ne3[1]], data=b)
    return src0, src1, A_q, b


def expected(t, A_q, b, M, N, K, ne2, ne3):
    """ggml semantics incl. broadcast r2 = ne12/ne02, r3 = ne13/ne03."""
    vt = la.vec_dot_type(t)
    fl = ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF
    arow, brow = ORACLE.row_bytes(t, K), ORACLE.row_bytes(vt, K)
    B_q = ORACLE.quantize(vt, b, fl)
    r2, r3 = ne2[1] // ne2[0], ne3[1] // ne3[0]
    out = np.zeros((ne3[1], ne2[1], N, M), np.float32)
    for i13 in range(ne3[1]):
        for i12 in range(ne2[1]):
            a_slice = (i13 // r3) * ne2[0] + i12 // r2
            b_slice = i13 * ne2[1] + i12
            A = A_q[a_slice * M * arow:(a_slice + 1) * M * arow]
            B = B_q[b_slice * N * brow:(b_slice + 1) * N * brow]
            out[i13, i12] = ORACLE.mul_mat(t, M, N, K, A, B)
    return out


@pytest.mark.parametrize("t", ol.A_TYPES, ids=[ol.NAMES[t] for t in ol.A_TYPES])
def test_boundary_matches_oracle(t, monkeypatch):
    """Both INIT modes: src1 quantized on the GPU (default) and by ggml's CPU INIT
    (LAMM_HIP_GPU_QUANT=0).  The GPU quantizer is bit-exact with the AVX2 from_float the
    CPU path uses, so the two outputs must be identical bit for bit."""
    M, N, K = 67, 9, 512
    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("LAMM_HIP_GPU_QUANT", mode)
        src0, src1, A_q, b = make_node(t, M, N, K, seed=t)
        dst = ggml_emu.mul_mat_node(src0, src1)
        assert ggml_emu.compute(dst, nth=3) is True
        got = dst.buf.view(np.float32).reshape(N, M)
        want = expected(t, A_q, b, M, N, K, (1, 1), (1, 1))[0, 0]
        assert rel_err(got, want, np.abs(want) + 1.0).max() < 1e-3
        outs.append(got.copy())
    if t not in (ol.F32,):
        np.testing.assert_array_equal(outs[0], outs[1])
    assert la.get_opt_level() == 3


def test_boundary_batch_broadcast():
    """ne02=2 weights broadcast over ne12=4 activations (r2=2), ne13=2 over ne03=1."""
    t, M, N, K = ol.Q4_0, 32, 5, 256
    ne2, ne3 = (2, 4), (1, 2)
    src0, src1, A_q, b = make_node(t, M, N, K, ne2, ne3, seed=11)
    dst = ggml_emu.mul_mat_node(src0, src1)
    assert ggml_emu.compute(dst, nth=4)
    got = dst.buf.view(np.float32).reshape(ne3[1], ne2[1], N, M)
    want = expected(t, A_q, b, M, N, K, ne2, ne3)
    assert rel_err(got, want, np.abs(want) + 1.0).max() < 1e-3


def test_weight_cache_reuse_and_invalidation():
    t, M, N, K = ol.Q8_0, 64, 2, 1024
    la.cache_clear()
    src0, src1, A_q, b = make_node(t, M, N, K, seed=5)
    dst = ggml_emu.mul_mat_node(src0, src1)
    ggml_emu.compute(dst)
    first = dst.buf.view(np.float32).copy()
    used = la.cache_bytes()
    assert used > 0
    ggml_emu.compute(dst)                       # same weights: served from the cache
    assert la.cache_bytes() == used
    assert np.array_equal(first, dst.buf.view(np.float32))
    # overwrite the host weights in place (same pointer): fingerprint must catch it
    new_q = ORACLE.quantize(t, np.random.default_rng(6).standard_normal((M, K), dtype=np.float32))
    src0.buf[:] = new_q
    ggml_emu.compute(dst)
    want = expected(t, new_q, b, M, N, K, (1, 1), (1, 1))[0, 0]
    got = dst.buf.view(np.float32).reshape(N, M)
    assert rel_err(got, want, np.abs(want) + 1.0).max() < 1e-3
    la.cache_clear()
    assert la.cache_bytes() == 0


def test_non_compute_phases_and_unsupported(monkeypatch):
    t, M, N, K = ol.Q4_0, 16, 1, 256
    src0, src1, _, _ = make_node(t, M, N, K)
    dst = ggml_emu.mul_mat_node(src0, src1)
    p = la.GgmlComputeParams()
    p.ith, p.nth = 0, 1
    p.type = la.TASK_FINALIZE
    assert not la.can_mul_mat(p, dst.t)
    p.type = la.TASK_INIT        # claimed whenever the GPU quantizes src1
    # default: 1 .. 7 activation rows leave INIT to ggml as the reference does (decode: 4.25 KiB of
    # q8_0 cross PCIe instead of the 16 KiB F32 row), and from 8 rows the GPU quantizer (the same
    # bytes) takes it
    assert not la.can_mul_mat(p, dst.t)
    src02, src12, _, _ = make_node(t, M, 2, K)
    assert not la.can_mul_mat(p, ggml_emu.mul_mat_node(src02, src12).t)
    src0r, src1r, _, _ = make_node(t, M, 8, K)
    assert la.can_mul_mat(p, ggml_emu.mul_mat_node(src0r, src1r).t)
    monkeypatch.setenv("LAMM_HIP_FUSED", "1")    # opt-in: the one-column GEMV quantizes the F32 row
    monkeypatch.setenv("LAMM_HIP_ORDER", "reference")
    assert la.can_mul_mat(p, dst.t)              # (reference order: ref_gemv_kernel's staging)
    assert not la.can_mul_mat(p, ggml_emu.mul_mat_node(src02, src12).t)   # 2 rows: only the fast GEMVs
    monkeypatch.delenv("LAMM_HIP_ORDER")         # the default since round 6: the fast engines
    assert la.can_mul_mat(p, dst.t)
    assert la.can_mul_mat(p, ggml_emu.mul_mat_node(src02, src12).t)
    monkeypatch.delenv("LAMM_HIP_FUSED")
    assert not la.can_mul_mat(p, dst.t)          # N = 1 without fusion: ggml's CPU INIT
    monkeypatch.setenv("LAMM_HIP_GPU_QUANT", "1")
    assert la.can_mul_mat(p, dst.t)
    monkeypatch.setenv("LAMM_HIP_GPU_QUANT", "0")
    assert not la.can_mul_mat(p, dst.t)
    monkeypatch.delenv("LAMM_HIP_GPU_QUANT")
    s2k, s1k, _, _ = make_node(ol.Q2_K, M, 1, K)   # q8_K activations: no fused path, CPU INIT
    assert not la.can_mul_mat(p, ggml_emu.mul_mat_node(s2k, s1k).t)
    src0b, src1b, _, _ = make_node(t, M, 8, K)   # from 8 activation rows: GPU quantizer
    dstb = ggml_emu.mul_mat_node(src0b, src1b)
    assert la.can_mul_mat(p, dstb.t)
    p.type = la.TASK_COMPUTE
    assert la.can_mul_mat(p, dst.t)


def test_f16_policy(monkeypatch):
    """F16 src0 (the KV-cache attention matmuls) is on the GPU path by
    default and declined under LAMM_HIP_EXTRA_TYPES=0, the reference's exact 7-pair set
    (src/loongarch_matmul.cpp:37-52)."""
    M, N, K = 16, 2, 256
    src0, src1, _, _ = make_node(ol.F16, M, N, K)
    assert src0.t.nb[0] == 2
    dst = ggml_emu.mul_mat_node(src0, src1)
    p = la.GgmlComputeParams()
    p.ith, p.nth, p.type = 0, 1, la.TASK_COMPUTE
    assert la.can_mul_mat(p, dst.t)
    monkeypatch.setenv("LAMM_HIP_EXTRA_TYPES", "0")
    assert not la.can_mul_mat(p, dst.t)
    monkeypatch.delenv("LAMM_HIP_EXTRA_TYPES")
    # a view of a KV cache (view_src set) in decode (N < 8) is left to ggml's CPU loop unless
    # LAMM_HIP_VIEWS=1; prefill-sized calls take it
    cache = ggml_emu.Tensor(ol.F16, [K, M])
    src0.t.view_src = ctypes.pointer(cache.t)
    assert not la.can_mul_mat(p, dst.t)
    monkeypatch.setenv("LAMM_HIP_VIEWS", "1")
    assert la.can_mul_mat(p, dst.t)
    monkeypatch.setenv("LAMM_HIP_VIEWS", "0")
    src0b, src1b, _, _ = make_node(ol.F16, M, 16, K)
    src0b.t.view_src = ctypes.pointer(cache.t)
    dstb = ggml_emu.mul_mat_node(src0b, src1b)
    assert not la.can_mul_mat(p, dstb.t)
    monkeypatch.delenv("LAMM_HIP_VIEWS")
    # unset: prefill-sized views go to the GPU in either float order (the reference's order runs
    # them in ggml_vec_dot_f16's AVX2 order, ref_f16_kernel), decode-sized ones stay
    assert la.can_mul_mat(p, dstb.t)
    assert not la.can_mul_mat(p, dst.t)
    monkeypatch.setenv("LAMM_HIP_ORDER", "reference")
    assert la.can_mul_mat(p, dstb.t)
    assert not la.can_mul_mat(p, dst.t)


GGML_OP_VIEW = 31   # LC/ggml.h enum ggml_op (b2430)


@pytest.mark.parametrize("n_tokens,n_head", [(1, 4), (9, 8)], ids=["decode", "prefill_gqa"])
def test_kv_cache_views_fresh_every_token(n_tokens, n_head, monkeypatch):
    """b2430's attention matmuls on a live F16 KV cache (llm_build_kqv, llama.cpp:5322-5372):
    K view ne=[128, n_kv, n_head_kv], nb1 = n_embd_k_gqa*2, nb2 = 256; transposed V view
    ne=[n_kv, 128, n_head_kv], nb1 = 2*n_ctx, nb2 = 2*n_ctx*128; both keep the cache's data
    pointer while new token rows land inside a 32-padded window (kv_self.n, llama.cpp:8887).
    After every token KQ and KQV must match the oracle -- the boundary may not serve a
    device copy of an older cache."""
    monkeypatch.setenv("LAMM_HIP_VIEWS", "1")
    rng = np.random.default_rng(42)
    hd, n_head_kv, n_ctx = 128, 4, 96
    r2 = n_head // n_head_kv
    n_embd_gqa = hd * n_head_kv
    kcache = ggml_emu.Tensor(ol.F16, [n_ctx * n_embd_gqa])
    vcache = ggml_emu.Tensor(ol.F16, [n_ctx * n_embd_gqa])
    kc = kcache.buf.view(np.float16).reshape(n_ctx, n_embd_gqa)     # [token][head*128 + d]
    vc = vcache.buf.view(np.float16).reshape(n_embd_gqa, n_ctx)     # [head*128 + d][token]
    pos = 0
    for step in range(5):
        # append n_tokens new rows (the ggml_cpy into the cache views, llama.cpp:5254-5277)
        for _ in range(n_tokens):
            kc[pos] = rng.standard_normal(n_embd_gqa).astype(np.float16)
            vc[:, pos] = rng.standard_normal(n_embd_gqa).astype(np.float16)
            pos += 1
        n_kv = min(n_ctx, max(32, -(-pos // 32) * 32))
        # ---- KQ = mul_mat(k_view, q)
        k = ggml_emu.Tensor(ol.F16, [hd, n_kv, n_head_kv], data=kcache.buf, nb=[2, 2 * n_embd_gqa, 2 * hd, 2 * hd * n_head_kv])
        k.t.view_src = ctypes.pointer(kcache.t)
        k.t.op = GGML_OP_VIEW
        q = rng.standard_normal((n_head * n_tokens, hd), dtype=np.float32)
        qt = ggml_emu.Tensor(ol.F32, [hd, n_tokens, n_head], data=q)
        kq = ggml_emu.mul_mat_node(k, qt)
        assert ggml_emu.compute(kq, nth=2)
        got = kq.buf.view(np.float32).reshape(n_head, n_tokens, n_kv)
        qq = ORACLE.quantize(ol.F16, q).view(np.uint16).reshape(n_head, n_tokens, hd)
        for h in range(n_head):
            A = np.ascontiguousarray(kc[:n_kv, (h // r2) * hd:(h // r2 + 1) * hd]).view(np.uint8).reshape(-1)
            want = ORACLE.mul_mat(ol.F16, n_kv, n_tokens, hd, A, qq[h].view(np.uint8).reshape(-1))
            absdot = np.abs(q[h * n_tokens:(h + 1) * n_tokens]) @ np.abs(kc[:n_kv, (h // r2) * hd:(h // r2 + 1) * hd].astype(np.float32)).T
            assert rel_err(got[h], want, absdot).max() < 1e-3, (step, h)
        # ---- KQV = mul_mat(v_view, kq_softmax)
        v = ggml_emu.Tensor(ol.F16, [n_kv, hd, n_head_kv], data=vcache.buf, nb=[2, 2 * n_ctx, 2 * n_ctx * hd, 2 * n_ctx * hd * n_head_kv])
        v.t.view_src = ctypes.pointer(vcache.t)
        v.t.op = GGML_OP_VIEW
        p = rng.random((n_head * n_tokens, n_kv), dtype=np.float32)
        pt = ggml_emu.Tensor(ol.F32, [n_kv, n_tokens, n_head], data=p)
        kqv = ggml_emu.mul_mat_node(v, pt)
        assert ggml_emu.compute(kqv, nth=2)
        got = kqv.buf.view(np.float32).reshape(n_head, n_tokens, hd)
        pq = ORACLE.quantize(ol.F16, p).view(np.uint16).reshape(n_head, n_tokens, n_kv)
        for h in range(n_head):
            Vh = np.ascontiguousarray(vc[(h // r2) * hd:(h // r2 + 1) * hd, :n_kv])
            want = ORACLE.mul_mat(ol.F16, hd, n_tokens, n_kv, Vh.view(np.uint8).reshape(-1),
                                  pq[h].view(np.uint8).reshape(-1))
            absdot = np.abs(p[h * n_tokens:(h + 1) * n_tokens]) @ np.abs(Vh.astype(np.float32)).T
            assert rel_err(got[h], want, absdot).max() < 1e-3, (step, h)


def test_views_bypass_weight_cache(monkeypatch):
    """A view src0 is uploaded per call and never held in the weight cache."""
    monkeypatch.setenv("LAMM_HIP_VIEWS", "1")
    la.cache_clear()
    M, N, K = 64, 2, 256
    cache = ggml_emu.Tensor(ol.F16, [K * M])
    cache.buf.view(np.float16)[:] = np.random.default_rng(3).standard_normal(K * M).astype(np.float16)
    v = ggml_emu.Tensor(ol.F16, [K, M], data=cache.buf)
    v.t.view_src = ctypes.pointer(cache.t)
    b = np.random.default_rng(4).standard_normal((N, K), dtype=np.float32)
    dst = ggml_emu.mul_mat_node(v, ggml_emu.Tensor(ol.F32, [K, N], data=b))
    assert ggml_emu.compute(dst)
    assert la.cache_bytes() == 0
    cache.buf.view(np.float16)[5 * K + 7] = np.float16(100.0)    # one element of one row
    assert ggml_emu.compute(dst)
    want = ORACLE.mul_mat(ol.F16, M, N, K, cache.buf, ORACLE.quantize(ol.F16, b))
    got = dst.buf.view(np.float32).reshape(N, M)
    np.testing.assert_allclose(got[:, 5], want[:, 5], rtol=1e-5)


@pytest.mark.parametrize("quant", ["cpu_init", "gpu"])
@pytest.mark.parametrize("zc_split", ["0", "1"])
@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
@pytest.mark.parametrize("t,M,N,K", [(ol.Q4_0, 4096, 1, 4096), (ol.Q4_0, 1000, 20, 512), (ol.Q8_0, 77, 3, 256),
                                     (ol.Q2_K, 300, 9, 512)])
def test_boundary_rows_split_over_devices(devices, t, M, N, K, quant, zc_split, monkeypatch):
    """LAMM_HIP_DEVICES: the weight's rows split over the listed devices, each writing its rows
    of C into dst (host consumes C) by device copies, or with zc_split = "1" decode-sized
    calls zero-copy on every device (one pinned activation buffer read by all, each device's rows
    of one pinned C).  Rehearsed with one device listed several times (separate streams and
    caches, the same slab bookkeeping as real devices); the result must be bit-identical to the
    same slabs computed one by one, and match the oracle within the parity tolerance.  quant:
    ggml's CPU INIT (q8 rows) or the boundary's default (F32 rows quantized on the GPU).
    zc_split: device copies (default) or zero copy on every device (LAMM_HIP_ZERO_COPY_SPLIT=1)."""
    monkeypatch.setenv("LAMM_HIP_ZERO_COPY_SPLIT", zc_split)
    if quant == "cpu_init":
        monkeypatch.setenv("LAMM_HIP_GPU_QUANT", "0")
    else:
        monkeypatch.delenv("LAMM_HIP_GPU_QUANT", raising=False)
    src0, src1, A_q, b = make_node(t, M, N, K, seed=M + N)
    want = expected(t, A_q, b, M, N, K, (1, 1), (1, 1))[0, 0]
    try:
        monkeypatch.setenv("LAMM_HIP_DEVICES", devices)
        la.boundary_reset()
        dst = ggml_emu.mul_mat_node(src0, src1)
        assert ggml_emu.compute(dst, nth=2)
        got = dst.buf.view(np.float32).reshape(N, M).copy()
        assert la.cache_bytes() > 0
        ggml_emu.compute(dst, nth=2)                       # second call: served from the caches
        np.testing.assert_array_equal(dst.buf.view(np.float32).reshape(N, M), got)
    finally:
        monkeypatch.delenv("LAMM_HIP_DEVICES")
        la.boundary_reset()
    assert rel_err(got, want, np.abs(want) + 1.0).max() < 1e-3
    # every slab equals the same rows computed alone (one device)
    G = len(devices.split(","))
    arow = ORACLE.row_bytes(t, K)
    for g in range(G):
        r0, rows = la.shard_rows(M, G, g, 16)
        if rows == 0:
            continue
        s0 = ggml_emu.Tensor(t, [K, rows], data=A_q[r0 * arow:(r0 + rows) * arow].copy())
        d1 = ggml_emu.mul_mat_node(s0, ggml_emu.Tensor(ol.F32, [K, N], data=b))
        assert ggml_emu.compute(d1, nth=2)
        np.testing.assert_array_equal(d1.buf.view(np.float32).reshape(N, rows), got[:, r0:r0 + rows])


DECODE_MODES = {"cpu_init": {}, "fused": {"LAMM_HIP_FUSED": "1"}, "device_copies": {"LAMM_HIP_ZERO_COPY": "0"},
                "fused_watch": {"LAMM_HIP_FUSED": "1", "LAMM_HIP_C_WATCH": "1"},
                "kernel_signal": {"LAMM_HIP_KERNEL_SIGNAL": "1"}, "watch_coherent": {"LAMM_HIP_C_WATCH": "1"},
                "watch_noncoherent": {"LAMM_HIP_C_WATCH": "2"}, "no_spin": {"LAMM_HIP_SPIN": "0"},
                "direct": {"LAMM_HIP_DIRECT": "1"}, "fused_direct": {"LAMM_HIP_FUSED": "1", "LAMM_HIP_DIRECT": "1"},
                "pinned_in": {"LAMM_HIP_VRAM_X": "0"}, "fused_pinned_in": {"LAMM_HIP_FUSED": "1", "LAMM_HIP_VRAM_X": "0"}}
DECODE_KEYS = ("LAMM_HIP_FUSED", "LAMM_HIP_ZERO_COPY", "LAMM_HIP_KERNEL_SIGNAL", "LAMM_HIP_SPIN", "LAMM_HIP_C_WATCH",
               "LAMM_HIP_DIRECT", "LAMM_HIP_VRAM_X")


@pytest.mark.parametrize("n", [1, 3], ids=["n1", "n3"])   # n3: the multi-column decode kernels
@pytest.mark.parametrize("t", [ol.Q4_0, ol.Q4_1, ol.Q8_0, ol.Q6_K], ids=["q4_0", "q4_1", "q8_0", "q6_k"])
def test_decode_calls_fresh_every_call(t, n, monkeypatch):
    """Decode-sized calls through the boundary, as llama.cpp makes them: the SAME src1 / dst
    buffers with new contents every call (ggml's compute buffer is reused per token).  Modes:
    activations written by the host into device memory through the BAR (default where the host can
    reach it) or read in place from pinned host memory (LAMM_HIP_VRAM_X=0), C written back into pinned
    host memory (default), or both copied by HIP (LAMM_HIP_ZERO_COPY=0); the activations quantized by
    ggml's CPU INIT (default) or by the GEMV (LAMM_HIP_FUSED=1); the GEMV launched through HIP
    (default) or dispatched on the library's own AQL queue with its completion signal
    (LAMM_HIP_DIRECT=1, lamm_aql.cpp); completion by the signal launch (default), seen in C's own words
    (LAMM_HIP_C_WATCH=1 coherent C / 2 non-coherent C), by the GEMV's own last workgroup
    (LAMM_HIP_KERNEL_SIGNAL=1) or by hipStreamSynchronize (LAMM_HIP_SPIN=0).  The boundary re-reads
    its switches at lamm_hip_boundary_reset (they used to be frozen at the first call).
    Every call must match the oracle, and every mode must give the same bits (three columns: the
    direct queue takes none of those kernels, so the region falls back to HIP and its completion)."""
    M, N, K = 4096, n, 4096
    rng = np.random.default_rng(t)
    if t in ol.KQ_TYPES:
        A_q = ol.random_kq_blocks(t, M, K, rng)
    else:
        A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    xs = [rng.standard_normal((N, K), dtype=np.float32) for _ in range(6)]
    vt = la.vec_dot_type(t)
    Ad = ORACLE.dequantize(t, A_q, M, K).astype(np.float64)
    results = {}
    try:
        for mode, env in DECODE_MODES.items():
            for k in DECODE_KEYS:
                monkeypatch.delenv(k, raising=False)
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            la.boundary_reset()
            src0 = ggml_emu.Tensor(t, [K, M], data=A_q)
            src1 = ggml_emu.Tensor(ol.F32, [K, N])
            dst = ggml_emu.mul_mat_node(src0, src1)
            outs = []
            for it, x in enumerate(xs):
                src1.buf.view(np.float32)[:] = x.reshape(-1)
                assert ggml_emu.compute(dst, nth=2)
                got = dst.buf.view(np.float32).reshape(N, M).copy()
                B = ORACLE.quantize(vt, x, ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF)
                want = ORACLE.mul_mat(t, M, N, K, A_q, B)
                absdot = np.abs(ORACLE.dequantize(vt, B, N, K).astype(np.float64)) @ np.abs(Ad).T
                assert rel_err(got, want, absdot).max() < 1e-3, (mode, it)
                outs.append(got)
            results[mode] = np.stack(outs)
    finally:
        for k in DECODE_KEYS:
            monkeypatch.delenv(k, raising=False)
        la.boundary_reset()
    first = results["cpu_init"].view(np.uint32)
    for mode, r in results.items():
        np.testing.assert_array_equal(r.view(np.uint32), first, err_msg=mode)


@pytest.mark.parametrize("threaded", [True, False], ids=["pool_threads", "sequential"])
@pytest.mark.parametrize("case", ["gpu_quant_strided", "cpu_init", "slices_padded_dst"])
def test_pool_jobs(case, threaded, monkeypatch):
    """Prefill-sized calls put ggml's pool threads to work (LAMM_HIP_POOL; lamm_hip.cpp pool_run /
    pool_help): bit 1 quantizes the F32 src1 rows to q8_0 on the host (lamm_hip_quantize_host),
    bit 2 scatters C out of pinned memory.  Driven from nth concurrent worker threads as ggml's
    pool drives the hook -- or one worker after the other, when thread 0 finds no helper and runs
    every chunk itself -- every mode (5: bit 1 plus bit 4, the reference-order call as two
    pipelined column chunks on two streams) is bit-identical to thread 0 alone with HIP's pageable copies
    and the device quantizer (LAMM_HIP_POOL=0) and within the oracle's tolerance; strided src1
    rows and padded dst rows exercise the row offsets."""
    t, K = ol.Q4_0, 512
    M, N, ne2, ne3, k_pad, row_pad = 2048, 160, (1, 1), (1, 1), 0, 0
    if case == "gpu_quant_strided":
        k_pad = 40
    elif case == "slices_padded_dst":
        M, N, ne2, ne3, row_pad = 1536, 72, (1, 2), (1, 2), 24
    monkeypatch.setenv("LAMM_HIP_GPU_QUANT", "0" if case == "cpu_init" else "-1")
    rng = np.random.default_rng(41)
    n1 = ne2[1] * ne3[1]
    a = rng.standard_normal((M, K), dtype=np.float32)
    A_q = ORACLE.quantize(t, a)
    b = rng.standard_normal((n1 * N, K), dtype=np.float32)
    bp = np.zeros((n1 * N, K + k_pad), np.float32)
    bp[:, :K] = b
    nb1 = 4 * (K + k_pad)
    src0 = ggml_emu.Tensor(t, [K, M, ne2[0], ne3[0]], data=A_q)
    src1 = ggml_emu.Tensor(ol.F32, [K, N, ne2[1], ne3[1]], data=bp,
                           nb=[4, nb1, nb1 * N, nb1 * N * ne2[1]])
    want = expected(t, A_q, b, M, N, K, ne2, ne3)
    outs = []
    la.cache_clear()
    for pool in ("5", "1", "2", "3", "5", "0"):
        monkeypatch.setenv("LAMM_HIP_POOL", pool)
        dst = ggml_emu.mul_mat_node(src0, src1, row_pad=row_pad)
        assert ggml_emu.compute(dst, nth=6, threaded=threaded)
        got = dst.buf.view(np.float32).reshape(ne3[1], ne2[1], N, M + row_pad)
        if row_pad:
            assert not got[..., M:].any()          # nothing written between the rows
            got = got[..., :M]
        assert rel_err(got, want, np.abs(want) + 1.0).max() < 1e-3
        outs.append(got.copy())
    for o in outs[:-1]:
        np.testing.assert_array_equal(o, outs[-1])


@pytest.mark.parametrize("t", [ol.Q5_1, ol.Q8_0], ids=["q5_1", "q8_0"])
def test_boundary_prefill_value_range(t):
    """A prefill-sized call through the boundary whose weights reach |w| = 300 and whose activation
    rows reach |x| = 1e5 (half the rows) -- beyond the f16 range of the dequantizing engine the fast
    order runs q8_0 / q5_1 prefill on; its range guard computes those tiles with exact block dots, so
    the output is finite and within the bar, as the reference's is."""
    M, N, K = 4096, 256, 512
    rng = np.random.default_rng(17)
    a = rng.standard_normal((M, K), dtype=np.float32)
    a *= 300 / np.abs(a).max()
    b = rng.standard_normal((N, K), dtype=np.float32)
    b[::2] *= 1e5 / np.abs(b).max()
    A_q = ORACLE.quantize(t, a)
    src0 = ggml_emu.Tensor(t, [K, M], data=A_q)
    src1 = ggml_emu.Tensor(ol.F32, [K, N], data=b)
    dst = ggml_emu.mul_mat_node(src0, src1)
    assert ggml_emu.compute(dst, nth=4)
    got = dst.buf.view(np.float32).reshape(N, M)
    want = expected(t, A_q, b, M, N, K, (1, 1), (1, 1))[0, 0]
    vt = la.vec_dot_type(t)
    B_q = ORACLE.quantize(vt, b, ol.QUANT_AVX)
    absdot = np.abs(ORACLE.dequantize(vt, B_q, N, K).astype(np.float64)) @ \
        np.abs(ORACLE.dequantize(t, A_q, M, K).astype(np.float64)).T
    fin = np.isfinite(want)   # (q8_1's fp16 s overflows in the reference itself beyond |x| ~ 2e3)
    assert fin.all() or t == ol.Q5_1
    assert fin.any() and np.isfinite(got[fin]).all()
    assert rel_err(got[fin], want[fin], absdot[fin]).max() < 1e-3


SIBLING_MODES = {"default": {}, "kernel_signal": {"LAMM_HIP_KERNEL_SIGNAL": "1"},
                 "watch_coherent": {"LAMM_HIP_C_WATCH": "1"}, "watch_noncoherent": {"LAMM_HIP_C_WATCH": "2"}}


@pytest.mark.parametrize("mode", list(SIBLING_MODES))
def test_sibling_calls(mode, monkeypatch):
    """Sibling decode calls (lamm_hip.cpp Siblings): three weights multiplied by the same src1
    tensor one after another, as llama.cpp's wq / wk / wv, over several tokens.  With the prediction
    on, the first call of each token runs the other two GEMVs ahead and their calls take the kept
    results; every output must be the bits of the prediction-off run.  Token 2 changes src1 between
    the first and second call (the kept result must be discarded), token 3 rewrites the third
    weight in place (its fingerprint changes: discarded, re-uploaded, recomputed).  Over the
    completion modes: with a C watch no group is formed (the watch sees only the
    leader's words) and none with the kernel-written completion signal either (lamm_hip.cpp sib_form), so
    the calls run one by one -- still the same bits."""
    for k, v in SIBLING_MODES[mode].items():
        monkeypatch.setenv(k, v)
    M, K, t = 4096, 4096, ol.Q4_0
    rng = np.random.default_rng(77)
    As = [ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32)) for _ in range(3)]
    A_new = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    xs = [rng.standard_normal(K).astype(np.float32) for _ in range(6)]
    x_alt = rng.standard_normal(K).astype(np.float32)

    def run(siblings):
        monkeypatch.setenv("LAMM_HIP_SIBLINGS", siblings)
        la.boundary_reset()
        srcs = [ggml_emu.Tensor(t, [K, M], data=a.copy()) for a in As]
        x = ggml_emu.Tensor(ol.F32, [K, 1])
        dsts = [ggml_emu.mul_mat_node(s0, x) for s0 in srcs]
        l0, t0 = la.sibling_stats()
        outs = []
        for tok, xv in enumerate(xs):
            if tok == 3:
                srcs[2].buf[:] = A_new
            for i, d in enumerate(dsts):
                x.buf.view(np.float32)[:] = x_alt if (tok == 2 and i == 1) else xv
                assert ggml_emu.compute(d, nth=2)
                outs.append(d.buf.view(np.float32).reshape(M).copy())
        l1, t1 = la.sibling_stats()
        return outs, l1 - l0, t1 - t0

    try:
        off, l_off, t_off = run("0")
        on, l_on, t_on = run("1")
    finally:
        monkeypatch.delenv("LAMM_HIP_SIBLINGS", raising=False)
        for k in SIBLING_MODES[mode]:
            monkeypatch.delenv(k, raising=False)
        la.boundary_reset()
    assert (l_off, t_off) == (0, 0)
    if mode != "default":
        assert (l_on, t_on) == (0, 0)
    else:
        assert l_on >= 8 and t_on >= 6, (l_on, t_on)   # tokens 1..5 lead with 2 siblings each; 2 discarded
        assert t_on < l_on
    for i, (a, b) in enumerate(zip(off, on)):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), f"call {i}"
    # and against the oracle: the second call of token 2 used x_alt, the third of tokens >= 3 A_new
    B = ORACLE.quantize(ol.Q8_0, x_alt.reshape(1, K), ol.QUANT_AVX)
    want = ORACLE.mul_mat(t, M, 1, K, As[1], B)[0]
    assert np.abs(on[2 * 3 + 1] - want).max() <= 1e-3 * (np.abs(want).max() + 1.0)
    B = ORACLE.quantize(ol.Q8_0, xs[4].reshape(1, K), ol.QUANT_AVX)
    want = ORACLE.mul_mat(t, M, 1, K, A_new, B)[0]
    assert np.abs(on[4 * 3 + 2] - want).max() <= 1e-3 * (np.abs(want).max() + 1.0)

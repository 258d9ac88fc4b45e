"""Decode chains (lamm_chain.hip): single-token GEMVs of a Llama layer sequence as ONE
persistent launch, each op's input either external or an earlier op's output.

Every op's y must be BIT-identical to lamm_hip_matmul(A, F32 x) on the same x (the chain uses
the same row-per-wave block dot and the same AVX2-flavour activation quantization), where x for
a dependent op is the chain's own output of its producer; one op per chain is also checked
against the oracle on the reference's quantized bytes (north-star tolerance).  Replays (the
launch sequence number the kernel advances on the device) and graph capture must never serve a
previous launch's outputs.
"""
import numpy as np
import pytest

from conftest import rel_err
import oracle_lib as ol
from test_gpu_parity import ORACLE, absdot, dev_bytes, pitch_blocks, pitched_A

pytestmark = pytest.mark.gpu
TOL = 1e-3

torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available() or la.device_count() == 0:
        pytest.fail("GPU tests need a gfx950 device (run with -m 'not gpu' on CPU)")
    yield


class Net:
    """`layers` Llama-shaped layers (q, k, v: H x H on x; o: H x H on q; gate, up: F x H on o;
    down: H x F on up; the next layer's q/k/v on down) with random weights of type t."""

    def __init__(self, t, H, F, layers, seed):
        rng = np.random.default_rng(seed)
        self.t, self.H, self.F = t, H, F
        self.ops = []      # (name, A device bytes, M, K, lda, x tensor, y tensor, A_q)
        self.keep = []
        self.x0 = torch.from_numpy(rng.standard_normal(H, dtype=np.float32)).cuda()
        x = self.x0
        for layer in range(layers):
            def op(name, M, K, xin):
                A_q = ORACLE.quantize(t, (rng.standard_normal((M, K), dtype=np.float32) * np.sqrt(3.0 / K)).astype(np.float32))
                kb = K // 32
                lda = pitch_blocks(t, kb)
                A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
                y = torch.full((M,), float("nan"), dtype=torch.float32, device="cuda")
                self.ops.append((f"{name}{layer}", A, M, K, lda, xin, y, A_q))
                return y
            q = op("q", H, H, x)
            op("k", H, H, x)
            op("v", H, H, x)
            o = op("o", H, H, q)
            op("gate", F, H, o)
            up = op("up", F, H, o)
            x = op("down", H, F, up)

    def chain(self):
        return la.Chain([(la.Matrix(A.data_ptr(), self.t, M, K // 32, lda), xin.data_ptr(), y.data_ptr())
                         for (_, A, M, K, lda, xin, y, _) in self.ops])

    def check_bitwise(self):
        """every op's y == lamm_hip_matmul(A, F32 x) on the x the chain saw"""
        s = torch.cuda.current_stream().cuda_stream
        for (name, A, M, K, lda, xin, y, _) in self.ops:
            want = torch.full((M,), float("nan"), dtype=torch.float32, device="cuda")
            la.matmul(la.Matrix(A.data_ptr(), self.t, M, K // 32, lda), la.Matrix(xin.data_ptr(), la.F32, K, 1, K),
                      la.Matrix(want.data_ptr(), la.F32, M, 1, M), s)
            torch.cuda.synchronize()
            a, b = y.cpu().numpy(), want.cpu().numpy()
            assert np.isfinite(a).all(), name
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), name

    def check_oracle(self, i):
        name, A, M, K, lda, xin, y, A_q = self.ops[i]
        vt = ORACLE.vec_dot_type(self.t)
        x = xin.cpu().numpy().reshape(1, K)
        B_q = ORACLE.quantize(vt, x, ol.QUANT_AVX)
        ref = ORACLE.mul_mat(self.t, M, 1, K, A_q, B_q)
        err = rel_err(y.cpu().numpy().reshape(1, M), ref, absdot(self.t, A_q, B_q, M, 1, K)).max()
        assert err < TOL, (name, err)


CHAIN_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0]


@pytest.mark.parametrize("t", CHAIN_TYPES, ids=[ol.NAMES[t] for t in CHAIN_TYPES])
def test_chain_small_layers(t):
    """3 layers of H = 256, F = 704 (7 ops, 4 phases per layer): bit-identical to separate
    launches, oracle parity, three launches in a row (device-side sequence numbers)."""
    net = Net(t, 256, 704, 3, seed=10 + t)
    ch = net.chain()
    assert ch.phases == 12
    for _ in range(3):
        for (_, _, _, _, _, _, y, _) in net.ops:
            y.fill_(float("nan"))
        ch.run(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ch.status()
        net.check_bitwise()
    net.check_oracle(len(net.ops) - 1)
    ch.close()


def test_chain_llama7b_two_layers():
    """Two Llama-7B layers (H 4096, F 11008, q4_0): the shapes llama-matmul-bench chains."""
    net = Net(ol.Q4_0, 4096, 11008, 2, seed=7)
    ch = net.chain()
    assert ch.phases == 8
    ch.run(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ch.status()
    net.check_bitwise()
    net.check_oracle(3)    # o of layer 0 (input: the chain's own q)
    net.check_oracle(13)   # down of layer 1 (K = 11008, input: the chain's own up)
    ch.close()


def test_chain_ragged_and_tiny_phases():
    """Rows fewer than the grid's waves (phases some waves have no row in), ragged M and K
    (K = 32, 96, 4160), a phase of three ops with different M."""
    t = ol.Q4_0
    rng = np.random.default_rng(5)
    x0 = torch.from_numpy(rng.standard_normal(96, dtype=np.float32)).cuda()
    made, ops = {"x": x0}, []
    # (name, M, K, input): K equals the producer's M
    spec = [("a", 64, 96, "x"), ("b", 3000, 96, "x"), ("c", 37, 96, "x"), ("d", 4160, 64, "a"), ("e", 5, 4160, "d"),
            ("f", 32, 4160, "d"), ("g", 1, 32, "f")]
    for name, M, K, src in spec:
        A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
        kb = K // 32
        lda = pitch_blocks(t, kb)
        A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
        y = torch.full((M,), float("nan"), dtype=torch.float32, device="cuda")
        made[name] = y
        ops.append((name, A, M, K, lda, made[src], y, A_q))
    ch = la.Chain([(la.Matrix(A.data_ptr(), t, M, K // 32, lda), xin.data_ptr(), y.data_ptr())
                   for (_, A, M, K, lda, xin, y, _) in ops])
    assert ch.phases == 4   # {a, b, c} on x, {d} on a, {e, f} on d, {g} on f
    ch.run(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ch.status()
    net = Net.__new__(Net)
    net.t, net.ops = t, ops
    net.check_bitwise()
    net.check_oracle(len(ops) - 1)
    ch.close()


def test_chain_graph_replay_sees_new_inputs():
    """Captured once, replayed with a different external input each time: every replay's outputs
    follow its own input (a stale granule from the previous replay would be taken as ready)."""
    net = Net(ol.Q4_0, 512, 1024, 2, seed=3)
    ch = net.chain()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ch.run(s.cuda_stream)   # warm-up outside capture
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ch.run(s.cuda_stream)
    last = None
    for k in range(3):
        net.x0.copy_(torch.randn(512, device="cuda"))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        ch.status()
        net.check_bitwise()
        out = net.ops[-1][6].cpu().numpy().copy()
        if last is not None:
            assert not np.array_equal(out, last)
        last = out
    ch.close()

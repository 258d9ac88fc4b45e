"""Seeded randomized parity sweep over every weight format and every dispatch path: random
M / N / K (ragged against every kernel's tiles), padded A / B / C pitches, ggml batch dims
with broadcast (r2), and the engine switches (fp6 / i8 / split-K counts / super-block
variants / dense on-off / grouped GEMV).  Every case is checked against the oracle with the
north-star tolerance and for untouched C padding.  Deterministic: the case list is a pure
function of the seed below."""
import numpy as np
import pytest

from conftest import rel_err
import oracle_lib as ol

pytestmark = pytest.mark.gpu
TOL = 1e-3
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402

ORACLE = ol.Oracle()
ALL_TYPES = [ol.F32, ol.F16, ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0, ol.Q2_K, ol.Q4_K, ol.Q5_K, ol.Q6_K]
SUPER = (ol.Q2_K, ol.Q4_K, ol.Q5_K, ol.Q6_K)


def _env_choices(t, N):
    """Engine switches that apply to (t, N); one is drawn per case."""
    if N <= 8:
        return [{}]
    if t in (ol.Q4_0, ol.Q4_1, ol.Q5_0):
        return [{}, {"LAMM_GEMM_PATH": "i8"}, {"LAMM_GEMM_PATH": "fp6", "LAMM_FP6_SPLIT": "1"},
                {"LAMM_GEMM_PATH": "fp6", "LAMM_FP6_SPLIT": "3"}, {"LAMM_GEMM_PATH": "fp6", "LAMM_FP6_SUB": "1"},
                {"LAMM_GEMM_PATH": "fp6", "LAMM_FP6_SUB": "2"}]
    if t in SUPER:
        return [{}, {"LAMM_KQ_VARIANT": "1"}, {"LAMM_KQ_GEMM": "0"}]
    if t in (ol.F32, ol.F16):
        return [{}, {"LAMM_DENSE_SPLIT": "2"}, {"LAMM_DENSE_GEMM": "0"}]
    return [{}]


def _cases(n=240, seed=20261016):
    rng = np.random.default_rng(seed)
    out = []
    for c in range(n):
        t = ALL_TYPES[c % len(ALL_TYPES)]
        qk = la.blck_size(t)
        unit = 256 if t in SUPER else (32 if qk == 32 else 1)
        M = int(rng.integers(1, 300))
        N = int(rng.choice([1, 2, 3, 5, 8, 9, 17, 40, 130]))
        K = unit * int(rng.integers(1, 24 if unit == 256 else 160)) + (int(rng.integers(0, 8)) if unit == 1 else 0)
        ne02, r2 = int(rng.choice([1, 2])), int(rng.choice([1, 2]))
        envs = _env_choices(t, N)
        env = envs[int(rng.integers(0, len(envs)))]
        out.append((c, t, M, N, K, ne02, r2, env, int(rng.integers(0, 3)), int(rng.integers(0, 3))))
    return out


def _operands(t, M, N, K, seed):
    rng = np.random.default_rng(seed)
    vt = la.vec_dot_type(t)
    if t in ol.KQ_TYPES or t == ol.Q2_K and seed % 2:
        A_q = ol.random_kq_blocks(t, M, K, rng)
    else:
        A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    fl = ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF
    B_q = ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32), fl)
    return A_q, B_q


@pytest.mark.parametrize("case", _cases(), ids=lambda c: f"{c[0]}-{ol.NAMES[c[1]]}-{c[2]}x{c[3]}x{c[4]}"
                         f"-b{c[5]}x{c[6]}-{'-'.join(f'{k[5:]}={v}' for k, v in c[7].items()) or 'auto'}")
def test_fuzz_vs_oracle(case, monkeypatch):
    c, t, M, N, K, ne02, r2, env, pad_a, pad_c = case
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    vt = la.vec_dot_type(t)
    kb = K // la.blck_size(t)
    abpb, bbpb = la.type_size(t), la.type_size(vt)
    lda = kb + pad_a
    while (lda * abpb) % 16:
        lda += 1
    ldb = kb + (1 if (pad_a and vt not in (ol.Q8_K,)) else 0)   # B pitch padding (blocks)
    if vt == ol.Q8_K or vt == ol.F32:
        ldb = kb                                                   # keep 4-byte aligned rows
    ldc = M + pad_c
    ne12 = ne02 * r2
    As = [_operands(t, M, N, K, 1000 * c + s)[0] for s in range(ne02)]
    Bs = [_operands(t, M, N, K, 1000 * c + 100 + s)[1] for s in range(ne12)]
    a_slice = M * lda * abpb
    A = np.zeros(ne02 * a_slice + 64, np.uint8)
    for s, a in enumerate(As):
        A[s * a_slice:(s + 1) * a_slice].reshape(M, lda * abpb)[:, :kb * abpb] = a.reshape(M, kb * abpb)
    b_slice = N * ldb * bbpb
    B = np.zeros(ne12 * b_slice + 64, np.uint8)
    for s, b in enumerate(Bs):
        B[s * b_slice:(s + 1) * b_slice].reshape(N, ldb * bbpb)[:, :kb * bbpb] = b.reshape(N, kb * bbpb)
    c_slice = N * ldc
    dA = torch.from_numpy(A).cuda()
    dB = torch.from_numpy(B).cuda()
    dC = torch.full((ne12 * c_slice + 16,), float("nan"), dtype=torch.float32, device="cuda")
    bt = la.Batch(ne02, 1, ne12, 1, a_slice, ne02 * a_slice, b_slice, ne12 * b_slice, 4 * c_slice,
                  4 * c_slice * ne12)
    la.mul_mat_torch(t, dA, dB, dC, M, N, K, lda=lda, ldb=ldb, ldc=ldc, batch=bt)
    torch.cuda.synchronize()
    out = dC.cpu().numpy()
    for z in range(ne12):
        a = As[z // r2]
        got = out[z * c_slice:(z + 1) * c_slice].reshape(N, ldc)
        ref = ORACLE.mul_mat(t, M, N, K, a, Bs[z])
        Ad = ORACLE.dequantize(t, a, M, K).astype(np.float64)
        Bd = ORACLE.dequantize(vt, Bs[z], N, K).astype(np.float64)
        den = np.abs(Bd) @ np.abs(Ad).T
        assert rel_err(got[:, :M], ref.reshape(N, M), den).max() < TOL, (z, env)
        if ldc > M:
            assert np.isnan(got[:, M:]).all(), "wrote outside the logical C"

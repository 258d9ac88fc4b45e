"""ctypes view of oracle/liblamm_oracle.so -- TEST INFRASTRUCTURE (the parity checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liblamm_oracle.so")

F32, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1, Q2_K, Q8_K = 0, 2, 3, 6, 7, 8, 9, 10, 15
Q4_K, Q5_K, Q6_K = 12, 13, 14
F16 = 1
QUANT_REF, QUANT_AVX = 0, 1
NAMES = {F32: "f32", Q4_0: "q4_0", Q4_1: "q4_1", Q5_0: "q5_0", Q5_1: "q5_1",
         Q8_0: "q8_0", Q8_1: "q8_1", Q2_K: "q2_k", Q8_K: "q8_k",
         Q4_K: "q4_k", Q5_K: "q5_k", Q6_K: "q6_k", F16: "f16"}
BY_NAME = {v: k for k, v in NAMES.items()}
A_TYPES = [F32, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q2_K, F16]   # quantizers restated (F16: §8f)
KQ_TYPES = [Q4_K, Q5_K, Q6_K]                        # vec_dot only, no quantizer
# byte offsets of the fp16 scale fields of a block (random-byte test inputs keep them finite)
FP16_FIELDS = {Q4_K: [0, 2], Q5_K: [0, 2], Q6_K: [208], Q2_K: [80, 82]}


def random_kq_blocks(t, rows, k, rng):
    """Random bytes for `rows` x `k` elements of k-quant type t, with finite positive fp16
    scales (vec_dot is defined for every byte pattern; this is how the GPU tests feed the
    formats the oracle has no quantizer for)."""
    bpb = {Q4_K: 144, Q5_K: 176, Q6_K: 210, Q2_K: 84}[t]
    nb = rows * (k // 256)
    blk = rng.integers(0, 256, size=(nb, bpb), dtype=np.uint8)
    for off in FP16_FIELDS[t]:
        d = (rng.random(nb) * 0.02 + 1e-3).astype(np.float16)
        blk[:, off:off + 2] = d.view(np.uint8).reshape(nb, 2)
    return blk.reshape(-1)


def _ensure_built():
    src = os.path.join(ORACLE_DIR, "lamm_oracle.c")
    if (not os.path.exists(ORACLE_SO)) or (
            os.path.exists(src) and os.path.getmtime(src) > os.path.getmtime(ORACLE_SO)):
        subprocess.run(["make", "-C", ORACLE_DIR, "oracle"], check=True,
                       stdout=subprocess.DEVNULL)


class Oracle:
    def __init__(self):
        _ensure_built()
        L = ctypes.CDLL(ORACLE_SO)
        L.lo_block_elems.restype = ctypes.c_int
        L.lo_block_bytes.restype = ctypes.c_size_t
        L.lo_vec_dot_type.restype = ctypes.c_int
        L.lo_row_bytes.restype = ctypes.c_size_t
        L.lo_row_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
        L.lo_quantize_row.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.lo_dequantize_row.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.lo_vec_dot.restype = ctypes.c_float
        L.lo_vec_dot.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.lo_mul_mat.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                 ctypes.c_void_p, ctypes.c_size_t]
        L.lo_mul_mat_avx.argtypes = L.lo_mul_mat.argtypes
        L.lo_fp32_to_fp16.restype = ctypes.c_uint16
        L.lo_fp32_to_fp16.argtypes = [ctypes.c_float]
        L.lo_fp16_to_fp32.restype = ctypes.c_float
        L.lo_fp16_to_fp32.argtypes = [ctypes.c_uint16]
        self.L = L

    def block_elems(self, t):
        return self.L.lo_block_elems(t)

    def block_bytes(self, t):
        return self.L.lo_block_bytes(t)

    def vec_dot_type(self, t):
        return self.L.lo_vec_dot_type(t)

    def row_bytes(self, t, k):
        return self.L.lo_row_bytes(t, k)

    def quantize(self, t, x, flavour=QUANT_REF):
        x = np.ascontiguousarray(x, dtype=np.float32)
        rows, k = x.shape
        rb = self.row_bytes(t, k)
        out = np.zeros(rows * rb, dtype=np.uint8)
        for r in range(rows):
            self.L.lo_quantize_row(t, flavour, x[r].ctypes.data, out[r * rb:].ctypes.data, k)
        return out

    def dequantize(self, t, q, rows, k):
        q = np.ascontiguousarray(q, dtype=np.uint8)
        rb = self.row_bytes(t, k)
        out = np.zeros((rows, k), dtype=np.float32)
        for r in range(rows):
            self.L.lo_dequantize_row(t, q[r * rb:].ctypes.data, out[r].ctypes.data, k)
        return out

    def mul_mat(self, t, M, N, K, A, B):
        """C[N][M] with C[j][i] = vec_dot(A row i, B column j); A, B packed rows."""
        A = np.ascontiguousarray(A, dtype=np.uint8)
        B = np.ascontiguousarray(B, dtype=np.uint8)
        vt = self.vec_dot_type(t)
        C = np.zeros((N, M), dtype=np.float32)
        self.L.lo_mul_mat(t, M, N, K, A.ctypes.data, self.row_bytes(t, K), B.ctypes.data,
                          self.row_bytes(vt, K), C.ctypes.data, M)
        return C

    def mul_mat_avx(self, t, M, N, K, A, B):
        """C[N][M] in the reference's x86 float order (lo_vec_dot_avx: the lamm opt-3 AVX2
        kernels' eight FMA lanes and their reduction tree; ggml's AVX2 q6_K)."""
        A = np.ascontiguousarray(A, dtype=np.uint8)
        B = np.ascontiguousarray(B, dtype=np.uint8)
        vt = self.vec_dot_type(t)
        C = np.zeros((N, M), dtype=np.float32)
        self.L.lo_mul_mat_avx(t, M, N, K, A.ctypes.data, self.row_bytes(t, K), B.ctypes.data,
                              self.row_bytes(vt, K), C.ctypes.data, M)
        return C

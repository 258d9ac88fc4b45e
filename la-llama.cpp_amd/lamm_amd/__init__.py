"""lamm_amd -- Python view of liblamm_hip.so (the MI355X lamm backend).

Thin ctypes binding over the C ABI in include/lamm_hip.h.  It mirrors the reference's
operator surface for this path:

* ``ggml_compute_params`` / ``ggml_tensor`` ctypes structs at the llama.cpp-b2430 binary
  layout, so tests can drive ``lamm_can_mul_mat`` / ``lamm_mul_mat`` exactly as
  ``ggml_compute_forward_mul_mat`` does (LC/ggml.c:10858-10863);
* ``Matrix`` == ``struct Matrix`` (src/lamm_common.h:87-93) and ``matmul`` ==
  ``LAMMImpl<T>::matmul(A, B, C)`` (src/lamm_impl.hpp:20) on device memory.

There is no fallback: if the HIP library is missing this import fails loudly, and
``matmul`` raises if the library reports an error.  PyTorch is only used by callers
for device memory and streams.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LAMM_HIP_LIB: load another build of the library (A/B of compile-time kernel variants)
LIB_PATH = os.environ.get("LAMM_HIP_LIB") or os.path.join(os.path.dirname(_HERE), "liblamm_hip.so")

F32, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1, Q2_K, Q8_K = 0, 2, 3, 6, 7, 8, 9, 10, 15
Q4_K, Q5_K, Q6_K = 12, 13, 14   # SURVEY §8f "next" formats (beyond the reference's lamm set)
F16 = 1                         # F16 x F16 (attention / KV cache)
NAMES = {F32: "f32", Q4_0: "q4_0", Q4_1: "q4_1", Q5_0: "q5_0", Q5_1: "q5_1",
         Q8_0: "q8_0", Q8_1: "q8_1", Q2_K: "q2_k", Q8_K: "q8_k",
         Q4_K: "q4_k", Q5_K: "q5_k", Q6_K: "q6_k", F16: "f16"}
BY_NAME = {v: k for k, v in NAMES.items()}
WEIGHT_TYPES = [F32, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q2_K, Q4_K, Q5_K, Q6_K, F16]

LAMM_OK, LAMM_ERR_TYPE, LAMM_ERR_SHAPE, LAMM_ERR_ALIGN, LAMM_ERR_HIP, LAMM_ERR_NODEV = range(6)

TASK_INIT, TASK_COMPUTE, TASK_FINALIZE = 0, 1, 2
OP_MUL_MAT = 23


class LammError(RuntimeError):
    pass


if not os.path.exists(LIB_PATH):
    raise ImportError(f"lamm_amd: {LIB_PATH} is missing -- build it with "
                      f"`make -C la-llama.cpp_amd` (or __graft_entry__.build()); there is no fallback")

# Load order matters: PyTorch-ROCm ships its own libamdhip64.so.  If liblamm_hip.so pulled
# in /opt/rocm's HIP runtime first, torch would bind to that one and find no device; with
# torch imported first, both share torch's runtime.  (The C ABI itself needs no torch.)
try:
    import torch as _torch  # noqa: F401
except ImportError:
    _torch = None

lib = ctypes.CDLL(LIB_PATH)


class Matrix(ctypes.Structure):
    """struct lamm_matrix == struct Matrix (src/lamm_common.h:87-93)."""
    _fields_ = [("data", ctypes.c_void_p), ("type", ctypes.c_int), ("row", ctypes.c_int),
                ("col", ctypes.c_int), ("ld", ctypes.c_int64)]


class Batch(ctypes.Structure):
    """struct lamm_batch: ggml-style batch dims (src/loongarch_matmul.cpp:130-142)."""
    _fields_ = [("ne02", ctypes.c_int64), ("ne03", ctypes.c_int64), ("ne12", ctypes.c_int64),
                ("ne13", ctypes.c_int64), ("nba2", ctypes.c_size_t), ("nba3", ctypes.c_size_t),
                ("nbb2", ctypes.c_size_t), ("nbb3", ctypes.c_size_t), ("nbc2", ctypes.c_size_t),
                ("nbc3", ctypes.c_size_t)]


class GgmlComputeParams(ctypes.Structure):
    """struct ggml_compute_params, LC/ggml.h:668-677 (b2430)."""
    _fields_ = [("type", ctypes.c_int32), ("ith", ctypes.c_int32), ("nth", ctypes.c_int32),
                ("wsize", ctypes.c_size_t), ("wdata", ctypes.c_void_p)]


class GgmlTensor(ctypes.Structure):
    """struct ggml_tensor, LC/ggml.h:552-590 (b2430): 368 bytes."""


GgmlTensor._fields_ = [
    ("type", ctypes.c_int32), ("backend", ctypes.c_int32), ("buffer", ctypes.c_void_p),
    ("ne", ctypes.c_int64 * 4), ("nb", ctypes.c_size_t * 4), ("op", ctypes.c_int32),
    ("op_params", ctypes.c_int32 * 16), ("flags", ctypes.c_int32),
    ("grad", ctypes.POINTER(GgmlTensor)), ("src", ctypes.POINTER(GgmlTensor) * 10),
    ("perf_runs", ctypes.c_int32), ("perf_cycles", ctypes.c_int64), ("perf_time_us", ctypes.c_int64),
    ("view_src", ctypes.POINTER(GgmlTensor)), ("view_offs", ctypes.c_size_t), ("data", ctypes.c_void_p),
    ("name", ctypes.c_char * 64), ("extra", ctypes.c_void_p), ("padding", ctypes.c_char * 8)]

lib.lamm_can_mul_mat.restype = ctypes.c_bool
lib.lamm_can_mul_mat.argtypes = [ctypes.POINTER(GgmlComputeParams), ctypes.POINTER(GgmlTensor)]
lib.lamm_mul_mat.restype = None
lib.lamm_mul_mat.argtypes = [ctypes.POINTER(GgmlComputeParams), ctypes.POINTER(GgmlTensor)]
lib.lamm_get_opt_level.restype = ctypes.c_int
lib.lamm_hip_matmul.restype = ctypes.c_int
lib.lamm_hip_matmul.argtypes = [ctypes.POINTER(Matrix)] * 3 + [ctypes.c_void_p]
lib.lamm_hip_matmul_ex.restype = ctypes.c_int
lib.lamm_hip_matmul_ex.argtypes = [ctypes.POINTER(Matrix)] * 3 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
lib.lamm_hip_matmul_group.restype = ctypes.c_int
lib.lamm_hip_matmul_group.argtypes = [ctypes.POINTER(Matrix), ctypes.c_int, ctypes.POINTER(Matrix),
                                      ctypes.POINTER(Matrix), ctypes.c_int, ctypes.c_void_p]
GROUP_MAX = 4         # LAMM_GROUP_MAX
ORDER_REFERENCE = 1   # LAMM_ORDER_REFERENCE: the reference's x86 float order, bit for bit (lamm_ref.hip)
lib.lamm_hip_matmul_batched.restype = ctypes.c_int
lib.lamm_hip_matmul_batched.argtypes = [ctypes.POINTER(Matrix)] * 3 + [ctypes.POINTER(Batch), ctypes.c_void_p]
lib.lamm_hip_quantize.restype = ctypes.c_int
lib.lamm_hip_quantize.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                  ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.lamm_hip_weights_create.restype = ctypes.c_int
lib.lamm_hip_weights_create.argtypes = [ctypes.POINTER(Matrix), ctypes.c_int64, ctypes.c_int64, ctypes.c_size_t,
                                        ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
lib.lamm_hip_matmul_weights.restype = ctypes.c_int
lib.lamm_hip_matmul_weights.argtypes = [ctypes.c_void_p, ctypes.POINTER(Matrix), ctypes.POINTER(Matrix),
                                        ctypes.POINTER(Batch), ctypes.c_void_p]
lib.lamm_hip_weights_bytes.restype = ctypes.c_size_t
lib.lamm_hip_weights_bytes.argtypes = [ctypes.c_void_p]
lib.lamm_hip_weights_destroy.restype = None
lib.lamm_hip_weights_destroy.argtypes = [ctypes.c_void_p]
lib.lamm_hip_last_error.restype = ctypes.c_char_p
lib.lamm_hip_device_count.restype = ctypes.c_int
lib.lamm_blck_size.restype = ctypes.c_int
lib.lamm_type_size.restype = ctypes.c_size_t
lib.lamm_vec_dot_type.restype = ctypes.c_int
lib.lamm_hip_build_id.restype = ctypes.c_char_p
lib.lamm_hip_engine.restype = ctypes.c_char_p
lib.lamm_hip_engine.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int]
lib.lamm_hip_shard_rows.restype = None
lib.lamm_hip_shard_rows.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
lib.lamm_hip_comm_unique_id.argtypes = [ctypes.c_void_p]
lib.lamm_hip_comm_init_rank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_int]
lib.lamm_hip_comm_init_all.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
lib.lamm_hip_comm_size.argtypes = [ctypes.c_void_p]
lib.lamm_hip_comm_local_ranks.argtypes = [ctypes.c_void_p]
lib.lamm_hip_comm_rank.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.lamm_hip_comm_destroy.argtypes = [ctypes.c_void_p]
lib.lamm_hip_comm_destroy.restype = None
lib.lamm_hip_comm_last_error.restype = ctypes.c_char_p
lib.lamm_hip_allgather_rows.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_void_p), ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
lib.lamm_hip_direct_begin.restype = ctypes.c_int
lib.lamm_hip_direct_begin.argtypes = [ctypes.c_int]
lib.lamm_hip_direct_end.restype = ctypes.c_int
lib.lamm_hip_sibling_stats.restype = None
lib.lamm_hip_sibling_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
lib.lamm_hip_cache_clear.restype = None
lib.lamm_hip_cache_bytes.restype = ctypes.c_size_t
lib.lamm_hip_boundary_reset.restype = None
lib.lamm_hip_reload_env.restype = None

# The library reads its LAMM_* switches once (lamm_hip_reload_env re-reads them).  Tests and A/B
# tools flip them through os.environ between calls, so every entry point below re-syncs the
# library when the LAMM_* part of the environment changed since the last call.
_env_seen = None


def _sync_env():
    global _env_seen
    cur = tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("LAMM_")))
    if cur != _env_seen:
        if _env_seen is not None:
            lib.lamm_hip_reload_env()
        _env_seen = cur


def reload_env():
    """Re-read every LAMM_* switch now (lamm_hip_reload_env)."""
    global _env_seen
    _env_seen = tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("LAMM_")))
    lib.lamm_hip_reload_env()


def blck_size(t):
    return lib.lamm_blck_size(t)


def type_size(t):
    return lib.lamm_type_size(t)


def vec_dot_type(t):
    return lib.lamm_vec_dot_type(t)


def row_bytes(t, k):
    return (k // blck_size(t)) * type_size(t)


def last_error():
    return lib.lamm_hip_last_error().decode()


def device_count():
    return lib.lamm_hip_device_count()


def build_id():
    """Hash of the sources the loaded liblamm_hip.so was built from (Makefile BUILD_ID)."""
    return lib.lamm_hip_build_id().decode()


def source_build_id():
    """The same hash recomputed from this tree: sha256 over the Makefile's ID_FILES (SRCS +
    csrc/*.h + ../include/lamm_hip.h, sorted by path as make's $(sort) sorts them)."""
    import glob
    import hashlib
    pkg = os.path.dirname(_HERE)
    mk = open(os.path.join(pkg, "Makefile")).read()
    srcs = next(ln for ln in mk.splitlines() if ln.startswith("SRCS")).split(":=", 1)[1].split()
    hdrs = [os.path.relpath(p, pkg) for p in glob.glob(os.path.join(pkg, "csrc", "*.h"))] + ["../include/lamm_hip.h"]
    h = hashlib.sha256()
    for rel in sorted(set(srcs + hdrs)):
        with open(os.path.join(pkg, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _check(rc, what):
    if rc != LAMM_OK:
        raise LammError(f"{what} failed ({rc}): {last_error()}")


def matmul(A, B, C, stream=0):
    """LAMMImpl<T>::matmul on device memory; A, B, C are ``Matrix`` (device pointers)."""
    _sync_env()
    _check(lib.lamm_hip_matmul(ctypes.byref(A), ctypes.byref(B), ctypes.byref(C), ctypes.c_void_p(stream)),
           "lamm_hip_matmul")


def matmul_ex(A, B, C, batch=None, flags=0, stream=0):
    """lamm_hip_matmul_ex: flags = ORDER_REFERENCE computes in the reference's x86 float order."""
    _sync_env()
    _check(lib.lamm_hip_matmul_ex(ctypes.byref(A), ctypes.byref(B), ctypes.byref(C),
                                  ctypes.byref(batch) if batch is not None else None, flags, ctypes.c_void_p(stream)),
           "lamm_hip_matmul_ex")


def matmul_group(As, B, Cs, flags=0, stream=0):
    """lamm_hip_matmul_group: C[i] = A[i] * B for up to GROUP_MAX weights sharing the activation B
    (one launch for a one-column reference-order call; the bits of one matmul_ex per weight)."""
    _sync_env()
    n = len(As)
    if len(Cs) != n:
        raise ValueError("one C per A")
    arrA = (Matrix * max(n, 1))(*As)
    arrC = (Matrix * max(n, 1))(*Cs)
    _check(lib.lamm_hip_matmul_group(arrA, n, ctypes.byref(B), arrC, flags, ctypes.c_void_p(stream)),
           "lamm_hip_matmul_group")


def sibling_stats():
    """(launched, taken): sibling decode calls computed ahead / results taken (lamm_hip_sibling_stats)"""
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    lib.lamm_hip_sibling_stats(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


class direct:
    """Direct-dispatch region (lamm_hip_direct_begin / end): the one-kernel decode GEMVs launched
    inside go onto the library's own AQL queue; on exit every one of them has completed, and
    ``launches`` holds how many were dispatched that way."""

    def __init__(self, device=0):
        self.device = device
        self.launches = None

    def __enter__(self):
        _sync_env()
        _check(lib.lamm_hip_direct_begin(self.device), "lamm_hip_direct_begin")
        return self

    def __exit__(self, *exc):
        n = lib.lamm_hip_direct_end()
        if n < 0:
            raise LammError(f"lamm_hip_direct_end failed ({n}): {last_error()}")
        self.launches = n
        return False


def matmul_batched(A, B, C, batch, stream=0):
    _sync_env()
    _check(lib.lamm_hip_matmul_batched(ctypes.byref(A), ctypes.byref(B), ctypes.byref(C), ctypes.byref(batch),
                                       ctypes.c_void_p(stream)), "lamm_hip_matmul_batched")


def mul_mat_torch(wtype, a, b, c, M, N, K, lda=None, ldb=None, ldc=None, stream=None, batch=None, flags=0):
    """C[j*ldc+i] = A_i . B_j for torch device tensors (uint8 blocks for A/B, f32 C).

    lda/ldb in blocks (default: packed rows), ldc in floats (default M).
    Runs on ``stream`` (default: torch's current stream).  flags: ORDER_REFERENCE for the
    reference's float order (lamm_hip_matmul_ex)."""
    import torch
    vt = vec_dot_type(wtype)
    kb = K // blck_size(wtype)
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    A = Matrix(a.data_ptr(), wtype, M, kb, lda if lda is not None else kb)
    B = Matrix(b.data_ptr(), vt, kb, N, ldb if ldb is not None else kb)
    C = Matrix(c.data_ptr(), F32, M, N, ldc if ldc is not None else M)
    if flags:
        matmul_ex(A, B, C, batch, flags, stream)
    elif batch is None:
        matmul(A, B, C, stream)
    else:
        matmul_batched(A, B, C, batch, stream)


class Weights:
    """Weight-stationary handle (lamm_hip_weights_create): A stays where it is and must not
    change; q4_0 / q4_1 / q5_0 / q5_1 additionally keep their packed prefill-GEMM form on device.
    ``a`` is a torch device tensor of A blocks; lda in blocks; slice strides in bytes."""

    def __init__(self, wtype, a, M, K, lda=None, ne02=1, ne03=1, nba2=0, nba3=0, stream=None):
        import torch
        kb = K // blck_size(wtype)
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        self.wtype, self.M, self.K, self.kb = wtype, M, K, kb
        self.ne02, self.ne03, self.nba2, self.nba3 = ne02, ne03, nba2, nba3
        self._a = a   # keep the blocks alive
        self.A = Matrix(a.data_ptr(), wtype, M, kb, lda if lda is not None else kb)
        _sync_env()
        h = ctypes.c_void_p()
        _check(lib.lamm_hip_weights_create(ctypes.byref(self.A), ne02, ne03, nba2, nba3, ctypes.c_void_p(stream),
                                           ctypes.byref(h)), "lamm_hip_weights_create")
        self.h = h

    @property
    def packed_bytes(self):
        return lib.lamm_hip_weights_bytes(self.h)

    def matmul_torch(self, b, c, N, ldb=None, ldc=None, batch=None, stream=None):
        import torch
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        vt = vec_dot_type(self.wtype)
        B = Matrix(b.data_ptr(), vt, self.kb, N, ldb if ldb is not None else self.kb)
        C = Matrix(c.data_ptr(), F32, self.M, N, ldc if ldc is not None else self.M)
        _sync_env()
        _check(lib.lamm_hip_matmul_weights(self.h, ctypes.byref(B), ctypes.byref(C),
                                           ctypes.byref(batch) if batch is not None else None,
                                           ctypes.c_void_p(stream)), "lamm_hip_matmul_weights")

    def close(self):
        if self.h:
            lib.lamm_hip_weights_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def quantize_torch(vtype, x, y, flavour=1, stream=None):
    """GPU activation quantizer: x [N][K] f32 (torch, device) -> y blocks (uint8)."""
    import torch
    N, K = x.shape
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    ldy = K // blck_size(vtype)
    _sync_env()
    _check(lib.lamm_hip_quantize(vtype, flavour, ctypes.c_void_p(x.data_ptr()), x.stride(0),
                                 ctypes.c_void_p(y.data_ptr()), ldy, K, N, ctypes.c_void_p(stream)),
           "lamm_hip_quantize")


def gemm_engine(fmt, M, N, K, slices=1, stationary=False, b_f32=False):
    """Which engine lamm_hip_matmul* (or, stationary, lamm_hip_matmul_weights) runs the call on,
    as the library decides it under the current LAMM_* switches (lamm_hip_engine): "gemv",
    "gemv-groups", "dense", "superblock", "fp6" or "i8"."""
    t = BY_NAME[fmt] if isinstance(fmt, str) else fmt
    _sync_env()
    return lib.lamm_hip_engine(t, M, N, K, slices, int(bool(stationary)), int(bool(b_f32))).decode()


COMM_ID_BYTES = 128


def shard_rows(M, world, rank, align=1):
    """(r0, rows) of `rank`'s contiguous slab of M rows (lamm_hip_shard_rows)."""
    r0, rows = ctypes.c_int64(), ctypes.c_int64()
    lib.lamm_hip_shard_rows(M, world, rank, align, ctypes.byref(r0), ctypes.byref(rows))
    return r0.value, rows.value


def comm_unique_id():
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _check_comm(lib.lamm_hip_comm_unique_id(buf), "lamm_hip_comm_unique_id")
    return buf.raw


def _check_comm(rc, what):
    if rc != LAMM_OK:
        raise LammError(f"{what} failed ({rc}): {lib.lamm_hip_comm_last_error().decode()}")


class Comm:
    """lamm_comm: row-sharded multi-GPU communicator.  Comm.rank(world, rank, id,
    device) joins a one-process-per-GPU communicator; Comm.all(devices) drives several devices
    from this process (duplicate devices = loopback exchange, for one-GPU rehearsals)."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def rank(cls, world, rank, uid, device):
        h = ctypes.c_void_p()
        _check_comm(lib.lamm_hip_comm_init_rank(ctypes.byref(h), world, rank, uid, device), "lamm_hip_comm_init_rank")
        return cls(h)

    @classmethod
    def all(cls, devices):
        h = ctypes.c_void_p()
        arr = (ctypes.c_int * len(devices))(*devices)
        _check_comm(lib.lamm_hip_comm_init_all(ctypes.byref(h), len(devices), arr), "lamm_hip_comm_init_all")
        return cls(h)

    @property
    def size(self):
        return lib.lamm_hip_comm_size(self.h)

    @property
    def local_ranks(self):
        return lib.lamm_hip_comm_local_ranks(self.h)

    def global_rank(self, local=0):
        return lib.lamm_hip_comm_rank(self.h, local)

    def allgather_rows(self, slabs, ld_slabs, Cs, ldc, M, N, align, streams):
        """Per local rank i: slabs[i] (device pointer, column stride ld_slabs[i] floats) -> Cs[i]
        (whole C, C[j*ldc + row]); enqueued on streams[i]."""
        n = len(slabs)
        P = ctypes.c_void_p * n
        _check_comm(lib.lamm_hip_allgather_rows(self.h, P(*slabs), (ctypes.c_int64 * n)(*ld_slabs), P(*Cs), ldc, M, N,
                                                align, P(*streams)), "lamm_hip_allgather_rows")

    def close(self):
        if self.h:
            lib.lamm_hip_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def can_mul_mat(params, dst):
    _sync_env()
    return bool(lib.lamm_can_mul_mat(ctypes.byref(params), ctypes.byref(dst)))


def mul_mat(params, dst):
    _sync_env()
    lib.lamm_mul_mat(ctypes.byref(params), ctypes.byref(dst))


def get_opt_level():
    _sync_env()
    return lib.lamm_get_opt_level()


def cache_clear():
    lib.lamm_hip_cache_clear()


def cache_bytes():
    return lib.lamm_hip_cache_bytes()


def boundary_reset():
    """Drop the ggml boundary's devices (caches, streams) and re-read every LAMM_* switch; the next
    call re-reads LAMM_HIP_DEVICES."""
    global _env_seen
    _env_seen = tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("LAMM_")))
    lib.lamm_hip_boundary_reset()

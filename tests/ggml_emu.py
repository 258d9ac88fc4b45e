"""Drive the drop-in boundary the way ggml does -- TEST INFRASTRUCTURE.

Builds b2430-layout ``ggml_tensor`` structs over numpy host buffers and replays the
control flow of ``ggml_compute_forward_mul_mat`` (LC/ggml.c:10736-10891) for one
mul_mat node:

  INIT    : the hook is asked first (LC/ggml.c:10858-10863 precedes the INIT branch).
            The reference's hook says no (params->type != COMPUTE) and thread 0 then
            quantizes src1 into wdata with traits[vec_dot_type].from_float
            (LC/ggml.c:10865-10887) -- here the oracle's AVX2-flavour quantizer, i.e.
            what an x86 AVX2 build of ggml runs.  liblamm_hip claims INIT when it
            quantizes src1 on the GPU (LAMM_HIP_GPU_QUANT, default on): every worker
            calls the hook, which returns at once, and wdata stays untouched;
  COMPUTE : every worker ith in [0, nth) calls the hook (LC/ggml.c:10858-10863) -- one after
            the other by default, or (threaded=True) from nth concurrent threads, as ggml's
            pool does (LC/ggml.c:18404-18421): what the boundary's pool-parallel staging of
            prefill calls (LAMM_HIP_POOL_COPY) needs to be exercised.
"""
import ctypes
import threading

import numpy as np

import lamm_amd as la
import oracle_lib as ol


class Tensor:
    """numpy-backed ggml_tensor (keeps the host buffer alive)."""

    def __init__(self, type_, ne, data=None, nb=None):
        ne = list(ne) + [1] * (4 - len(ne))
        self.t = la.GgmlTensor()
        self.t.type = type_
        bs, ts = la.blck_size(type_), la.type_size(type_)
        if nb is None:
            nb = [ts, ts * (ne[0] // bs)]
            nb.append(nb[1] * ne[1])
            nb.append(nb[2] * ne[2])
        nbytes = nb[3] * ne[3]
        if data is None:
            self.buf = np.zeros(nbytes, dtype=np.uint8)
        else:
            self.buf = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
            assert self.buf.size >= nbytes, (self.buf.size, nbytes)
        for i in range(4):
            self.t.ne[i] = ne[i]
            self.t.nb[i] = nb[i]
        self.t.data = self.buf.ctypes.data
        self.ne, self.nb = ne, nb


def mul_mat_node(src0, src1, row_pad=0):
    """dst = ggml_mul_mat(src0, src1): dst F32 [ne01, ne11, ne12, ne13] (row_pad: dst rows of
    ne01 + row_pad floats, i.e. a view into a wider buffer)."""
    ne = [src0.ne[1], src1.ne[1], src1.ne[2], src1.ne[3]]
    nb = None
    if row_pad:
        nb = [4, 4 * (ne[0] + row_pad)]
        nb += [nb[1] * ne[1], nb[1] * ne[1] * ne[2]]
    dst = Tensor(ol.F32, ne, nb=nb)
    dst.t.op = la.OP_MUL_MAT
    dst.t.src[0] = ctypes.pointer(src0.t)
    dst.t.src[1] = ctypes.pointer(src1.t)
    dst._keep = (src0, src1)
    return dst


def _run_workers(params, dst, nth, threaded):
    if not threaded:
        for ith in range(nth):
            params.ith = ith
            la.mul_mat(params, dst.t)
        return
    la.can_mul_mat(params, dst.t)   # the environment is synced here, not in the workers
    ps = []
    for ith in range(nth):
        p = la.GgmlComputeParams()
        p.type, p.ith, p.nth, p.wsize, p.wdata = params.type, ith, params.nth, params.wsize, params.wdata
        ps.append(p)
    ths = [threading.Thread(target=la.lib.lamm_mul_mat, args=(ctypes.byref(p), ctypes.byref(dst.t))) for p in ps]
    for th in ths:
        th.start()
    for th in ths:
        th.join()


def compute(dst, nth=4, oracle=None, flavour=ol.QUANT_AVX, threaded=False):
    """Replay INIT + COMPUTE.  Returns True if the lamm hook took the node."""
    oracle = oracle or ol.Oracle()
    src0, src1 = dst._keep
    vt = la.vec_dot_type(src0.t.type)
    K = src1.ne[0]
    row = la.row_bytes(vt, K)
    nrows = src1.ne[1] * src1.ne[2] * src1.ne[3]
    wdata = np.zeros(max(row * nrows, 1), dtype=np.uint8)

    params = la.GgmlComputeParams()
    params.ith, params.nth = 0, nth
    params.wsize, params.wdata = wdata.size, wdata.ctypes.data

    params.type = la.TASK_INIT
    if la.can_mul_mat(params, dst.t):   # GPU quantizes src1 in COMPUTE
        _run_workers(params, dst, nth, threaded)
        params.ith = 0
        wdata[:] = 0xA5                  # poison: COMPUTE must not read wdata
    elif src1.t.type != vt:  # thread 0 quantizes src1 -> wdata (contiguous F32 src1 assumed)
        x = src1.buf.view(np.float32).reshape(nrows, K)
        wdata[:] = oracle.quantize(vt, x, flavour)

    params.type = la.TASK_COMPUTE
    if not la.can_mul_mat(params, dst.t):
        return False
    _run_workers(params, dst, nth, threaded)
    return True

"""Direct dispatch (lamm_hip_direct_begin / end) against HIP launches, config 2's q4_0 4096 x 4096
GEMV over 33 rotated weight copies: per-step wall time of 20- and 200-step regions, and one call
per region (launch + completion, median of 300).  The LAMM_AQL_* switches are read once per
process, so run once per setting.  Prints one JSON line."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402

fmt, M, K, R = "q4_0", 4096, 4096, 33
t = la.BY_NAME[fmt]
kb = K // 32
gen = torch.Generator(device="cuda")
gen.manual_seed(3)
A, arow = bench.make_weights(torch, la, fmt, R, M, K, gen)
B = bench.make_activations(torch, la, fmt, 1, K, gen)
C = torch.zeros(M, dtype=torch.float32, device="cuda")
mats = [la.Matrix(A.data_ptr() + c * M * arow, t, M, kb, kb) for c in range(R)]
Bm = la.Matrix(B.data_ptr(), la.vec_dot_type(t), kb, 1, kb)
Cm = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
lib = bench.steps_lib(la)
lib.lamm_steps_matmul.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(la.Matrix), ctypes.POINTER(la.Matrix),
                                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
arr = (la.Matrix * R)(*mats)
dev = torch.cuda.current_device()
out = {k: os.environ.get(k) for k in ("LAMM_AQL_SIGNAL", "LAMM_AQL_SCOPE", "LAMM_AQL_PRIO")}
w = ctypes.c_double()
torch.cuda.synchronize()
lib.lamm_steps_direct(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), 0, 5, dev, 0,
                      ctypes.byref(w))
for steps in (20, 200):
    v = []
    for rep in range(5):
        n = lib.lamm_steps_direct(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), rep, steps,
                                  dev, 0, ctypes.byref(w))
        assert n == steps, n
        v.append(w.value / steps)
    out[f"direct_{steps}_us"] = round(min(v), 3)
one = []
for i in range(300):
    lib.lamm_steps_direct(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), i, 1, dev, 0,
                          ctypes.byref(w))
    one.append(w.value)
out["direct_one_call_us"] = round(statistics.median(one), 2)
for gap in (20e-6, 100e-6):   # host idle between calls, as in llama.cpp's decode (~19 us of CPU ops)
    one = []
    for i in range(300):
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < gap:
            pass
        lib.lamm_steps_direct(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), i, 1, dev, 0,
                              ctypes.byref(w))
        one.append(w.value)
    out[f"direct_one_call_gap{int(gap * 1e6)}_us"] = round(statistics.median(one), 2)
st = torch.cuda.Stream()
one = []
for i in range(300):
    t0 = time.perf_counter()
    lib.lamm_steps_matmul(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), i, 1,
                          ctypes.c_void_p(st.cuda_stream))
    st.synchronize()
    one.append((time.perf_counter() - t0) * 1e6)
out["hip_one_call_sync_us"] = round(statistics.median(one), 2)
for gap in (20e-6, 100e-6):
    one = []
    for i in range(300):
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < gap:
            pass
        t0 = time.perf_counter()
        lib.lamm_steps_matmul(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), i, 1,
                              ctypes.c_void_p(st.cuda_stream))
        st.synchronize()
        one.append((time.perf_counter() - t0) * 1e6)
    out[f"hip_one_call_sync_gap{int(gap * 1e6)}_us"] = round(statistics.median(one), 2)
for steps in (20, 200):
    v = []
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lib.lamm_steps_matmul(ctypes.cast(arr, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), rep, steps,
                              ctypes.c_void_p(st.cuda_stream))
        st.synchronize()
        v.append((time.perf_counter() - t0) * 1e6 / steps)
    out[f"hip_eager_{steps}_us"] = round(min(v), 3)
print(json.dumps(out), flush=True)

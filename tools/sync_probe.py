import ctypes, os, sys, time, json
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
import torch, lamm_amd as la, bench
fmt, M, K = "q4_0", 4096, 4096
t = la.BY_NAME[fmt]; vt = la.vec_dot_type(t); kb = K // 32; arow = la.row_bytes(t, K); slab = M * arow; R = 33
g = torch.Generator(device="cuda"); g.manual_seed(1)
A, _ = bench.make_weights(torch, la, fmt, R, M, K, g)
B = bench.make_activations(torch, la, fmt, 1, K, g)
C = torch.zeros(M, dtype=torch.float32, device="cuda")
mats = [la.Matrix(A.data_ptr() + c * slab, t, M, kb, kb) for c in range(R)]
Bm = la.Matrix(B.data_ptr(), vt, kb, 1, kb); Cm = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
st = torch.cuda.Stream()
out = {}
for steps in (20, 200):
    with torch.cuda.stream(st):
        for i in range(5): la.matmul(mats[i % R], Bm, Cm, st.cuda_stream)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        for s in range(steps): la.matmul(mats[s % R], Bm, Cm, torch.cuda.current_stream().cuda_stream)
    gr.replay(); torch.cuda.synchronize()
    def m_sync():
        with torch.cuda.stream(st):
            torch.cuda.synchronize(); t0 = time.perf_counter(); gr.replay(); torch.cuda.synchronize(); return time.perf_counter() - t0
    def m_spin():
        with torch.cuda.stream(st):
            ev = torch.cuda.Event()
            torch.cuda.synchronize(); t0 = time.perf_counter(); gr.replay(); ev.record(st)
            while not ev.query(): pass
            torch.cuda.synchronize(); return time.perf_counter() - t0
    def m_empty():
        with torch.cuda.stream(st):
            torch.cuda.synchronize(); t0 = time.perf_counter(); torch.cuda.synchronize(); return time.perf_counter() - t0
    for name, fn in (("sync", m_sync), ("spin", m_spin), ("empty_sync", m_empty), ("sync2", m_sync), ("spin2", m_spin)):
        v = sorted(fn() for _ in range(15))
        out[f"{name}{steps}"] = round(v[len(v) // 2] * 1e6 / (steps if "empty" not in name else 1), 3)
    del gr
print(json.dumps(out))

"""Debug helper: which B element does A element p pair with? (f32, one-hot rows)."""
import sys, numpy as np, torch
sys.path.insert(0, "la-llama.cpp_amd")
import lamm_amd as la
K = int(sys.argv[1]) if len(sys.argv) > 1 else 256
M = 16
A = np.zeros((M, K), np.float32)
pos = [0, 1, 3, 4, 17, 63, 64, 65, 100, 200, K - 1][:M]
for r, p in enumerate(pos):
    A[r, p % K] = 1.0
B = (np.arange(K, dtype=np.float32) + 1)[None, :]
a = torch.from_numpy(A.view(np.uint8).reshape(-1).copy()).cuda()
b = torch.from_numpy(B.view(np.uint8).reshape(-1).copy()).cuda()
c = torch.zeros(M + 16, dtype=torch.float32, device="cuda")
la.mul_mat_torch(la.F32, a, b, c, M, 1, K)
torch.cuda.synchronize()
print("K", K, "want", [p % K + 1 for p in pos], "got", c.cpu().numpy()[:len(pos)].tolist())

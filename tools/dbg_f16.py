"""Debug probe: one-hot f16 rows through the dense GEMV (which B element pairs with which A)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "la-llama.cpp_amd"))
import lamm_amd as la

for K in (1, 2, 8, 16):
    M = K
    A = np.eye(M, K, dtype=np.float16); P = (-K) % 8 + 8
    Bv = (2.0 ** np.arange(K)).astype(np.float16)[None, :]
    dA = torch.from_numpy(np.pad(A, ((0, 0), (0, P))).reshape(-1).view(np.uint8).copy()).cuda()
    dB = torch.from_numpy(Bv.reshape(-1).view(np.uint8).copy()).cuda()
    dC = torch.zeros(M, dtype=torch.float32, device="cuda")
    la.mul_mat_torch(la.F16, dA, dB, dC, M, 1, K, lda=K + P)
    torch.cuda.synchronize()
    print("K", K, "got", dC.cpu().numpy(), "want", Bv[0].astype(np.float32))

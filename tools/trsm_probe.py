"""Large-N fp64 inverse formulations on this ROCm build (training-loss backward needs K^-1).

    python tools/trsm_probe.py <method> <N>
"""
import sys
import time

import torch

method, N = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(0)
A = torch.randn(N, 64, dtype=torch.float64, generator=g).to(dev)
K = A @ A.T / 64 + torch.eye(N, dtype=torch.float64, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
L, info = torch.linalg.cholesky_ex(K)
if method == "trsm":
    Kinv = torch.cholesky_inverse(L) if False else None
    Li = torch.linalg.solve_triangular(L, torch.eye(N, dtype=torch.float64, device=dev), upper=False)
    Kinv = Li.T @ Li
elif method == "inv_L":
    Li, _ = torch.linalg.inv_ex(L)
    Kinv = Li.T @ Li
elif method == "inv_K":
    Kinv, _ = torch.linalg.inv_ex(K)
elif method == "cholinv":
    Kinv = torch.cholesky_inverse(L)
torch.cuda.synchronize()
err = float(torch.linalg.matrix_norm(Kinv @ K - torch.eye(N, dtype=torch.float64, device=dev)))
print(method, N, "ok", f"{time.perf_counter() - t0:.2f} s", f"|K^-1 K - I| = {err:.2e}", flush=True)

"""Dev comparison: vendor-library fp64 rates on this MI355X at the headline size,
for context next to the hand-written Cholesky:
  torch.matmul (rocBLAS / hipBLASLt DGEMM), torch.linalg.cholesky (rocSOLVER POTRF).
Synthetic SPD input (diagonally dominated random), N from argv (default 16384)."""
import json
import sys
import time

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
dev = torch.device('cuda:0')
torch.manual_seed(0)
A = torch.randn(n, n, dtype=torch.float64, device=dev)
B = torch.randn(n, n, dtype=torch.float64, device=dev)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


t = timed(lambda: torch.matmul(A, B), 3)
print(json.dumps({'op': 'dgemm (torch.matmul)', 'n': n, 'ms': 1e3 * t,
                  'tflops': 2.0 * n ** 3 / t / 1e12}), flush=True)
del B
S = torch.matmul(A, A.T) / n
S.diagonal().add_(1.0)
del A
torch.cuda.empty_cache()
t = timed(lambda: torch.linalg.cholesky(S), 2)
print(json.dumps({'op': 'dpotrf (torch.linalg.cholesky)', 'n': n, 'ms': 1e3 * t,
                  'tflops': n ** 3 / 3.0 / t / 1e12}), flush=True)

# The trailing-update shape of the blocked Cholesky: C (n x n) -= A_p B_p^T with a
# k-panel of 512 / 1024 columns (outer panel of 4 / 8 tiles).
for kd in (512, 1024):
    P = torch.randn(n, kd, dtype=torch.float64, device=dev)
    C = torch.randn(n, n, dtype=torch.float64, device=dev)
    t = timed(lambda: C.addmm_(P, P.T, alpha=-1.0), 3)
    print(json.dumps({'op': 'dgemm update C -= P P^T (torch.addmm_)', 'n': n, 'k': kd,
                      'ms': 1e3 * t, 'tflops': 2.0 * n * n * kd / t / 1e12}), flush=True)
    del P, C
    torch.cuda.empty_cache()

"""Vendor-library ceiling for the fit's GEMM shapes on this box (rocBLAS / hipBLASLt through
torch.matmul): FP64 DGEMM and complex128 ZGEMM rates to put the library's own kernels in
context.  Usage: python tools/blas_ceiling.py"""
import time

import torch


def rate(a, b, flop, reps=10):
    torch.matmul(a, b)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return flop / dt / 1e12, dt * 1e3


def main():
    torch.manual_seed(0)
    dev = "cuda"
    for m, n, k in ((8192, 8192, 8192), (4096, 4096, 4096), (600, 46656, 600), (600, 600, 46656)):
        a = torch.randn(m, k, dtype=torch.float64, device=dev)
        b = torch.randn(k, n, dtype=torch.float64, device=dev)
        tf, ms = rate(a, b, 2.0 * m * n * k)
        print(f"dgemm {m}x{n}x{k}: {tf:.1f} TFLOP/s ({ms:.3f} ms)", flush=True)
    for m, n, k in ((600, 46656, 600), (600, 600, 46656), (4096, 4096, 4096)):
        a = torch.randn(m, k, dtype=torch.complex128, device=dev)
        b = torch.randn(k, n, dtype=torch.complex128, device=dev)
        tf, ms = rate(a, b, 8.0 * m * n * k)
        print(f"zgemm {m}x{n}x{k}: {tf:.1f} TFLOP/s algorithmic ({ms:.3f} ms)", flush=True)


if __name__ == "__main__":
    main()

"""Library GEMM rates on this box for the forward-GEMM lab's shapes (torch.matmul -> hipBLASLt/rocBLAS):
fp32 (fp32 MFMA, 157.3 TF/s peak) and bf16 (2516.8 TF/s dense peak), per shape: us per call and TF/s."""
import torch

shapes = [(9728, 640, 128), (23296, 640, 128), (65536, 640, 128), (23296, 1280, 256), (8192, 4096, 4096)]
for dt, peak in ((torch.float32, 157.3), (torch.bfloat16, 2516.8)):
    for M, K, N in shapes:
        a = torch.randn(M, K, device="cuda", dtype=dt)
        b = torch.randn(K, N, device="cuda", dtype=dt)
        for _ in range(3):
            a @ b
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            a @ b
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        tf = 2 * M * N * K / us / 1e6
        print(f"{str(dt):15s} M={M:6d} K={K:5d} N={N:5d} {us:9.2f} us {tf:8.1f} TF/s {tf / peak:.3f} of {peak}", flush=True)

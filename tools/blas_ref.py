"""Reference point: torch (hipBLASLt/rocBLAS) fp32 GEMM time on the C3 step shapes."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
B = 2048
shapes = [(B, 1024, 1024), (B, 1024, 480), (B, 512, 1024), (B, 256, 512), (1024, 1024, B),
          (4096, 4096, 4096), (8192, 8192, 8192)]
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(N, K, device="cuda")
    for _ in range(3):
        c = a @ b.t()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    s.record()
    for _ in range(n):
        c = a @ b.t()
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / n * 1e-3
    print(f"torch fp32 {M}x{N}x{K}: {t*1e6:8.1f} us  {2*M*N*K/t/1e12:6.1f} TF")

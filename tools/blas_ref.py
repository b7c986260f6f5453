"""Reference point: torch (hipBLASLt/rocBLAS) fp32 and bf16 GEMM time on the C3 step shapes
(the bf16 figure bounds what a split-bf16 fp32 GEMM could reach: six bf16 products)."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
B = 2048
shapes = [(B, 1024, 1024), (B, 1024, 480), (B, 512, 1024), (B, 256, 512), (1024, 1024, B),
          (512, 1024, B), (4096, 4096, 4096), (8192, 8192, 8192)]
for dt in (torch.float32, torch.bfloat16):
    for M, N, K in shapes:
        a = torch.randn(M, K, device="cuda").to(dt)
        b = torch.randn(N, K, device="cuda").to(dt)
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
        print(f"torch {str(dt)[6:]:8s} {M}x{N}x{K}: {t*1e6:8.1f} us  {2*M*N*K/t/1e12:7.1f} TF",
              flush=True)

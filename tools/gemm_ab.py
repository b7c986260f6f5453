"""A/B the GEMM of two builds of libdlrm_hip (default plans) on the C3 step shapes:
    python tools/gemm_ab.py <libA.so> <libB.so>
Each shape is timed as 20 launches captured in a hipGraph."""
import ctypes
import os
import sys

import torch

P, I32, I64, F32, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_size_t


def load(path):
    lib = ctypes.CDLL(path)
    lib.dlrm_gemm_f32.argtypes = [I32, I32, I64, I64, I64, F32, P, I64, P, I64, P, I64, I32, P,
                                  P, I64, P, SZ, P]
    lib.dlrm_gemm_f32.restype = I32
    lib.dlrm_gemm_f32_workspace_size.argtypes = [I32, I32, I64, I64, I64]
    lib.dlrm_gemm_f32_workspace_size.restype = SZ
    return lib


def timeit(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (n * reps) * 1e3


def pad4(n):
    return (n + 3) // 4 * 4


def main():
    libs = [load(p) for p in sys.argv[1:3]]
    dev = "cuda"
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    B = int(os.environ.get("AB_BATCH", "2048"))
    layers = [(13, 512), (512, 256), (256, 128), (479, 1024), (1024, 1024), (1024, 512),
              (512, 256)]
    tot = [0.0, 0.0]
    for li, (K, N) in enumerate(layers):
        Kp = pad4(K + 1)
        X = torch.randn(B, Kp, device=dev)
        W = torch.randn(N, Kp, device=dev)
        Y = torch.empty(B, pad4(N + 1), device=dev)
        G = torch.randn(B, N, device=dev)
        dX = torch.empty(B, Kp, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        cases = [("fwd", (0, 1, B, N, Kp, 1.0, X, Kp, W, Kp, Y, Y.stride(0), 6, None, None, 0))]
        if li != 0:
            cases.append(("dgrad", (0, 0, B, K, N, 1.0, G, N, W, Kp, dX, Kp, 3, None, X, Kp)))
        cases.append(("wgrad", (1, 0, N, Kp, B, 1e-9, G, N, X, Kp, W, Kp, 4, None, None, 0)))
        for name, a in cases:
            row = []
            for i, lib in enumerate(libs):
                args = [a[0], a[1], a[2], a[3], a[4], a[5], a[6].data_ptr(), a[7], a[8].data_ptr(),
                        a[9], a[10].data_ptr(), a[11], a[12], None,
                        a[14].data_ptr() if a[14] is not None else None, a[15], ws.data_ptr(),
                        ws.numel(), st]

                def fn(lib=lib, args=args):
                    args[-1] = torch.cuda.current_stream().cuda_stream  # the capture stream
                    rc = lib.dlrm_gemm_f32(*args)
                    assert rc == 0, rc
                t = timeit(fn)
                tot[i] += t
                row.append(t)
            fl = 2 * B * N * K
            print(f"L{li} {K:5d}->{N:5d} {name:6s} A {row[0]:7.1f} us  B {row[1]:7.1f} us  "
                  f"({fl / row[1] / 1e6:.1f} TF B)", flush=True)
    print(f"TOTAL A {tot[0]:.1f} us  B {tot[1]:.1f} us")


if __name__ == "__main__":
    main()

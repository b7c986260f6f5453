"""GEMM body lab (experiments, not product code): times the library's pipe_body at the
tiles / occupancies / LDS-stage depths of tools/gemm_lab.hip (tools/_lab/libgemm_lab.so,
built by `python tools/gemm_lab.py --build` on the CPU) on the C3 training-step GEMMs and
checks every result bitwise against the library's own launch of the same problem
(cfg = U * 100 + tile, U = 32-deep sub-tiles per LDS stage).

    python tools/gemm_lab.py [--cfgs 100,200,...] [--splits 1,2,4] [--shapes fwd,dgrad,wgrad]
"""
import argparse
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "_lab", "libgemm_lab.so")


TRACE_LIB = os.path.join(HERE, "_lab", "libgemm_trace.so")


def build(trace=False):
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
           f"-I{ROOT}/include", f"-I{ROOT}/dlrm-yx_amd/csrc", "-fno-slp-vectorize", "-shared",
           os.path.join(HERE, "gemm_lab.hip"), os.path.join(ROOT, "dlrm-yx_amd/csrc/abi.cpp"),
           "-o", TRACE_LIB if trace else LIB] + (["-DLAB_TRACE"] if trace else [])
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--build-trace", action="store_true")
    ap.add_argument("--cfgs", default="100,101,102,103,105,107,200,201,202,203,205,207,400,401")
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--wsplits", default="1,2,4,8")
    ap.add_argument("--shapes", default="fwd,dgrad,wgrad")
    ap.add_argument("--B", type=int, default=2048)
    args = ap.parse_args()
    if args.build or args.build_trace:
        build(trace=args.build_trace)
        return
    import torch
    sys.path.insert(0, os.path.join(ROOT, "dlrm-yx_amd"))
    from dlrm_hip import ops, _lib
    lab = ctypes.CDLL(LIB)
    lab.lab_gemm.restype = ctypes.c_int
    dev = "cuda"
    ws = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)

    def pad4(n):
        return (n + 3) // 4 * 4

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

    B = args.B
    layers = [(479, 1024), (1024, 1024), (1024, 512), (512, 256)]
    cfgs = [int(c) for c in args.cfgs.split(",")]
    tot = {}
    for kind in args.shapes.split(","):
        for li, (K, N) in enumerate(layers):
            Kp = pad4(K + 1)
            g = torch.Generator(device=dev).manual_seed(li)
            X = torch.randn(B, Kp, device=dev, generator=g)
            W = torch.randn(N, Kp, device=dev, generator=g)
            Y = torch.zeros(B, pad4(N + 1), device=dev)
            G = torch.randn(B, N, device=dev, generator=g)
            dX = torch.zeros(B, Kp, device=dev)
            nd = K if K % 4 == 0 else Kp
            if kind == "fwd":
                C = Y
                mk = lambda: ops.gemm_problem(X, W, trans_b=True, C=Y, epilogue=ops.EPI_RELU)[0]
                fl, shape = 2 * B * N * Kp, (B, N, Kp)
                splits = [int(s) for s in args.splits.split(",")]
            elif kind == "dgrad":
                C = dX
                mk = lambda: ops.gemm_problem(G, W[:, :nd], C=dX[:, :nd], epilogue=ops.EPI_DRELU,
                                              aux=X)[0]
                fl, shape = 2 * B * N * nd, (B, nd, N)
                splits = [int(s) for s in args.splits.split(",")]
            else:  # wgrad into a gradient bucket (multi-GPU form: plain store, ones_col bias)
                Wg = torch.zeros(N, Kp, device=dev)
                C = Wg
                if K % 4 == 0:
                    mk = lambda: ops.gemm_problem(G, X[:, :K], trans_a=True, C=Wg, ones_col=K)[0]
                else:
                    mk = lambda: ops.gemm_problem(G, X, trans_a=True, C=Wg)[0]
                fl, shape = 2 * B * N * Kp, (N, nd, B)
                splits = [int(s) for s in args.wsplits.split(",")]
            pr = mk()
            arr = (_lib.GemmProblem * 1)(pr)
            # reference: the library's launch (its own plan)
            C.zero_()
            ops.gemm_group([pr], ws)
            torch.cuda.synchronize()
            ref = C.clone()
            lib_us = timeit(lambda: ops.gemm_group([pr], ws))
            res = []
            for cfg in cfgs:
                for sp in splits:
                    def run():
                        rc = lab.lab_gemm(cfg, sp, 1, arr, ctypes.c_void_p(ws.data_ptr()),
                                          ctypes.c_size_t(ws.numel()),
                                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                        if rc:
                            raise RuntimeError(f"lab rc {rc}")
                    try:
                        C.zero_()
                        run()
                        torch.cuda.synchronize()
                        same = bool(torch.equal(C, ref))
                        close = float((C - ref).abs().max())
                        us = timeit(run)
                    except Exception as e:  # noqa: BLE001
                        print(f"  cfg {cfg} s{sp}: {e}", flush=True)
                        continue
                    res.append((us, cfg, sp, same, close))
            res.sort()
            best = res[0]
            key = f"{kind}{li}"
            tot[key] = (lib_us, best[0])
            print(f"{kind:5s} L{li} {shape}: lib {lib_us:6.1f} us ({fl / lib_us / 1e6:5.1f} TF) | "
                  f"best cfg {best[1]} s{best[2]} {best[0]:6.1f} us ({fl / best[0] / 1e6:5.1f} TF)"
                  f" same={best[3]}", flush=True)
            print("    " + " ".join(f"{c}s{s}:{u:.1f}{'' if sm else '!'}" for u, c, s, sm, _ in
                                    sorted(res, key=lambda r: (r[1], r[2]))), flush=True)
    print("TOTAL lib %.1f us, best-per-shape %.1f us" % (sum(v[0] for v in tot.values()),
                                                        sum(v[1] for v in tot.values())))


if __name__ == "__main__":
    main()

"""Launch-overhead lab (experiment, not product code): per-launch cost of an empty kernel,
of a one-float4-per-thread kernel, and of a grid-wide barrier inside one launch, all timed
from hipGraph replays (the step's own launch path).

    python tools/launch_lab.py --build      # on the CPU
    python tools/launch_lab.py              # on the GPU
"""
import argparse
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_lab", "liblaunch_lab.so")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                    "-shared", os.path.join(HERE, "launch_lab.hip"), "-o", LIB], check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    args = ap.parse_args()
    if args.build:
        build()
        return
    import torch
    lab = ctypes.CDLL(LIB)
    dev = "cuda"
    a = torch.randn(1 << 22, device=dev)
    b = torch.empty_like(a)
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.zeros(4096, device=dev)

    def per_launch(fn, n=50, reps=10):
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

    def st():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    for grid in (64, 256, 512, 1024):
        us = per_launch(lambda: lab.lab_empty(grid, st()))
        print(f"empty   grid {grid:5d}: {us:6.2f} us/launch", flush=True)
    for grid in (256, 1024, 4096):
        us = per_launch(lambda: lab.lab_touch(grid, ctypes.c_void_p(a.data_ptr()),
                                              ctypes.c_void_p(b.data_ptr()), st()))
        print(f"touch   grid {grid:5d}: {us:6.2f} us/launch ({grid * 256 * 32 / us / 1e3:.0f} GB/s)",
              flush=True)
    # grid barriers: the counter is monotonic across launches of one graph replay sequence,
    # so each launch gets its own base; replays re-run the same bases, so reset per replay.
    for grid in (256, 512):
        for nbar in (1, 21):
            state = {"base": 0}

            def run(grid=grid, nbar=nbar):
                lab.lab_barrier(grid, ctypes.c_void_p(ctr.data_ptr()), ctypes.c_uint(state["base"]),
                                nbar, ctypes.c_void_p(err.data_ptr()),
                                ctypes.c_void_p(out.data_ptr()), st())
                state["base"] += grid * nbar
            # a graph captures fixed bases: zero the counter inside the graph first
            n = 20

            def seq():
                ctr.zero_()
                state["base"] = 0
                for _ in range(n):
                    run()
            seq()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                seq()
            g.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                g.replay()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / (n * 10) * 1e3
            print(f"barrier grid {grid:5d} x {nbar:3d} barriers: {us:7.2f} us/launch "
                  f"(err {int(err.item())})", flush=True)


if __name__ == "__main__":
    main()

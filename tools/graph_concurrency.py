"""Does a captured HIP graph run two independent branches concurrently?
Two spin kernels on a forked stream inside one capture: replay time ~1x the
spin means the branches overlap, ~2x that they are serialized.
python tools/graph_concurrency.py"""
import time

import torch


def main():
    cyc = 2_000_000
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()

    def timeit(fn, n=20):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    one = timeit(lambda: torch.cuda._sleep(cyc))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        s1.wait_stream(cap)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        cap.wait_stream(s1)
    two = timeit(g.replay)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
    serial = timeit(g2.replay)

    def eager():
        s1.wait_stream(s0)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        s0.wait_stream(s1)
    ea = timeit(eager)
    print(f"one spin {one:.3f} ms; graph fork/join of two {two:.3f} ms; graph serial two "
          f"{serial:.3f} ms; eager two streams {ea:.3f} ms")


if __name__ == "__main__":
    main()

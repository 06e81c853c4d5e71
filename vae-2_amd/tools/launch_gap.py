"""Per-kernel cost of back-to-back dependent launches on one stream: N tiny kernels
(a 1-element in-place add) eager and captured as one HIP graph; prints us per launch.
The step issues ~3,700 launches, so this bounds what launch fusion can save."""
import time

import torch


def run(n=2000, reps=5):
    x = torch.zeros(1, device="cuda")

    def body():
        for _ in range(n):
            x.add_(1.0)
    body()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        body()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / (reps * n) * 1e6
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            body()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / (reps * n) * 1e6
    print(f"{n} dependent tiny kernels: eager {eager:.2f} us/launch, graph replay {graph:.2f} us/launch")


if __name__ == "__main__":
    run()

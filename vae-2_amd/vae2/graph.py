"""Whole-step HIP graph capture.

The eager step issues ~9,000 kernel launches through Python; at the benchmark
size the host needs about as long to issue them as the GPU needs to run them.
StepGraph captures one complete step — forward on the main and side streams,
autograd backward, gradient all-reduce hooks, Adam and the weight re-pack — into
a single HIP graph (torch.cuda.CUDAGraph over hipGraph) and replays it with one
launch.  Every buffer the step touches is either persistent (parameters, flat
gradients, optimizer state, packed weights, BN running statistics) or comes from
the graph's private memory pool, so replays are equivalent to eager steps:
tests/test_graph_gpu.py checks bit-identical parameters after several steps.

Inputs the step reads (clips, noise) must live in static device tensors that
the caller refills before replay (or draws inside the step with device RNG,
which CUDAGraph advances per replay).
"""
import torch

from . import streams


class StepGraph:
    def __init__(self, step_fn, warmup=2, capture_error_mode="global"):
        self.step_fn = step_fn
        dev = torch.cuda.current_device()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # allocator / autograd warm-up off the default stream
            for _ in range(warmup):
                step_fn()
            streams.join_all()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        streams._FORKED.clear()
        try:
            with torch.cuda.graph(self.graph, capture_error_mode=capture_error_mode):
                self.out = step_fn()
                streams.join_all()
        finally:
            streams._FORKED.clear()
        torch.cuda.synchronize()

    def replay(self):
        self.graph.replay()
        return self.out

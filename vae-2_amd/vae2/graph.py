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

Distributed steps (RCCL collectives inside the graph): the capture runs in
thread-local capture mode.  ProcessGroupNCCL's watchdog thread polls the events of
earlier (eager, warm-up) collectives with hipEventQuery; under the default global
mode HIP refuses that call from any thread while a capture is open
(hipErrorStreamCaptureUnsupported), the watchdog thread dies and aborts the process
(observed on MI355X with a world-size-1 RCCL group; round 4 saw the same capture
hang).  Thread-local mode restricts only the capturing thread.  Before capturing, the
warm-up collectives are drained: the GPU is synchronised and the watchdog (which polls
every 100 ms) is given time to retire them, so it holds no work whose events it still
queries while the capture is open (a watchdog query that met an event recorded in the
capturing stream aborted one run of the world-1 test: hipErrorCapturedEvent); callers
also disable ProcessGroupNCCL's event cache (`vae2.dist.prepare_nccl_env`), so no event
of an eager collective is re-recorded by a captured one.
"""
import time

import torch
import torch.distributed as dist

from . import streams


def _default_capture_mode():
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
        return "thread_local"  # the RCCL watchdog thread queries events during the capture
    return "global"


class StepGraph:
    def __init__(self, step_fn, warmup=2, capture_error_mode=None):
        self.step_fn = step_fn
        if capture_error_mode is None:
            capture_error_mode = _default_capture_mode()
        dev = torch.cuda.current_device()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # allocator / autograd warm-up off the default stream
            for _ in range(warmup):
                step_fn()
            streams.join_all()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if capture_error_mode == "thread_local":
            time.sleep(0.5)  # the NCCL watchdog retires the warm-up collectives first
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

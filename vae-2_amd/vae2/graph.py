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
hang).  Thread-local mode restricts only the capturing thread.

Before such a capture the eager collectives are drained by a CONDITION, not a clock
(`drain_collectives`): no early gradient bucket may be outstanding (vae2.dist._EARLY
empty: every eager step ran allreduce_grads, which waits on all of its Work handles),
the GPU is synchronised, and then the capture waits until ProcessGroupNCCL's watchdog has
RETIRED every eager collective -- read from its flight recorder (`retired` flips when the
watchdog removes the work from its list; vae2.dist.prepare_nccl_env turns the recorder
on).  A watchdog that still held a completed warm-up work while the capture was open
queried its event during the capture; one run of the world-1 test aborted with
hipErrorCapturedEvent that way (round 5, then hidden by a fixed 0.5 s sleep).  Once every
eager work is retired, the watchdog has no event to query until the capture ends:
collectives issued inside the capture are never handed to it.  A recorder that is off, or a
work not retired within the bound, raises instead of capturing into the race.  The event
cache is off as well (vae2.dist.prepare_nccl_env), so no event of an eager collective is
re-recorded by a captured one.
"""
import pickle
import time

import torch
import torch.distributed as dist

from . import streams

_CAPTURE_WINDOWS = []  # (t0_ns, t1_ns) of earlier captures: their collectives never retire


class DrainError(RuntimeError):
    pass


def _nccl_groups_exist():
    return dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"


def pending_collectives():
    """Flight-recorder entries of eager NCCL collectives the watchdog has not retired yet
    (entries created inside an earlier capture are skipped: captured work never reaches the
    watchdog).  Raises DrainError when the recorder is off."""
    import torch._C._distributed_c10d as c10d
    d = pickle.loads(c10d._dump_nccl_trace(True, False, False))
    ents = d.get("entries")
    if ents is None or (not ents and _collectives_issued()):
        raise DrainError("the NCCL flight recorder is off (TORCH_FR_BUFFER_SIZE=0): the "
                         "drain before a graph capture cannot see the watchdog's work; set "
                         "TORCH_FR_BUFFER_SIZE (vae2.dist.prepare_nccl_env) or run eager")
    out = []
    for e in ents:
        if e.get("retired", False):
            continue
        tc = e.get("time_created_ns") or 0
        if any(t0 <= tc <= t1 for t0, t1 in _CAPTURE_WINDOWS):
            continue
        out.append(e)
    return out


def _collectives_issued():
    try:
        be = dist.group.WORLD._get_backend(torch.device("cuda", torch.cuda.current_device()))
        return be._get_sequence_number_for_group() > 0
    except Exception:  # noqa: BLE001 (no NCCL backend object: nothing to drain)
        return False


def drain_collectives(timeout_s=30.0):
    """Block until no eager collective is outstanding anywhere: no early gradient bucket
    left un-waited (vae2.dist._EARLY), the device idle, and every eager NCCL collective
    retired by ProcessGroupNCCL's watchdog (flight recorder).  Returns the number of polls
    (0: nothing was pending).  Raises DrainError on an outstanding bucket, a disabled
    recorder or a work the watchdog has not retired within timeout_s."""
    if not _nccl_groups_exist():
        return 0
    from . import dist as vdist
    if any(vdist._EARLY.values()):
        raise DrainError("early gradient buckets are still outstanding (a backward without "
                         "allreduce_grads before the capture)")
    torch.cuda.synchronize()
    deadline = time.monotonic() + timeout_s
    polls = 0
    while True:
        pend = pending_collectives()
        if not pend:
            return polls
        if time.monotonic() > deadline:
            names = sorted({e.get("profiling_name", "?") for e in pend})
            raise DrainError(f"{len(pend)} eager collectives ({', '.join(names)}) not retired "
                             f"by the NCCL watchdog within {timeout_s:.0f} s")
        polls += 1
        time.sleep(0.002)


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
        self.drain_polls = drain_collectives()  # condition, not a clock (see above)
        self.graph = torch.cuda.CUDAGraph()
        streams._FORKED.clear()
        t0 = time.time_ns()
        try:
            with torch.cuda.graph(self.graph, capture_error_mode=capture_error_mode):
                self.out = step_fn()
                streams.join_all()
        finally:
            streams._FORKED.clear()
            _CAPTURE_WINDOWS.append((t0, time.time_ns()))
        torch.cuda.synchronize()

    def replay(self):
        self.graph.replay()
        return self.out

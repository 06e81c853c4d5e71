"""Concurrent execution of independent sub-networks on HIP streams.

The ELBO step has three independent branches per phase: the posterior net vs
the encoder trunk (stem .. stage 3 do not depend on z), and the future vs past
decoders.  Their low-resolution layers launch far fewer workgroups than the 256
CUs, so running them on separate streams fills the GPU.  PyTorch autograd replays
every backward op on the stream its forward op ran on, so the backward overlaps
the same way.  Tensors crossing streams are registered with record_stream so the
caching allocator never recycles them early.  Inside a HIP graph capture the
side streams fork from and join back into the capture stream (event waits), so
the captured graph keeps the same concurrency.
"""
import contextlib

import torch

_SIDE = {}
_FORKED = set()  # side streams forked into the capture in progress
ENABLED = True


def side_stream(device, idx):
    key = (str(device), idx)
    s = _SIDE.get(key)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _SIDE[key] = s
    return s


def role_of(stream):
    """The side-stream key of `stream`, or "main" (the default, a graph's capture stream or
    any other stream the caller runs on)."""
    for key, s in _SIDE.items():
        if s == stream:
            return key[1]
    return "main"


def _record(tensors, stream):
    for t in tensors:
        if isinstance(t, (list, tuple)):
            _record(t, stream)
        elif torch.is_tensor(t) and t.is_cuda:
            t.record_stream(stream)


@contextlib.contextmanager
def on_side(idx, inputs=()):
    """Run the block on side stream `idx` after the current stream's prior work."""
    if not ENABLED or not torch.cuda.is_available():
        yield None
        return
    main = torch.cuda.current_stream()
    s = side_stream(main.device, idx)
    s.wait_stream(main)
    if torch.cuda.is_current_stream_capturing():
        _FORKED.add(s)
    _record(inputs, s)
    with torch.cuda.stream(s):
        yield s


def join(stream, outputs=()):
    """Make the current stream wait for `stream` and adopt its outputs."""
    if stream is None:
        return
    main = torch.cuda.current_stream()
    main.wait_stream(stream)
    _record(outputs, main)


def fence_side(stream):
    """Make every other stream of the device wait for `stream`'s current work."""
    for (dev, _), s in _SIDE.items():
        if dev == str(stream.device) and s != stream:
            s.wait_stream(stream)
    if torch.cuda.is_current_stream_capturing():
        return  # the default stream is outside the graph; the capture stream joins at the end
    main = torch.cuda.default_stream(stream.device)
    if main != stream:
        main.wait_stream(stream)


def join_all():
    """Make the current stream wait for every side stream (e.g. before the optimizer
    step: parameter gradients are written by backward kernels on side streams)."""
    if not torch.cuda.is_available():
        return
    main = torch.cuda.current_stream()
    capturing = torch.cuda.is_current_stream_capturing()
    for (dev, _), s in _SIDE.items():
        if dev == str(main.device) and s != main and (not capturing or s in _FORKED):
            main.wait_stream(s)
    if capturing:
        return
    d = torch.cuda.default_stream(main.device)
    if d != main:
        main.wait_stream(d)

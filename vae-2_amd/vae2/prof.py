"""Live per-kernel timing with HIP events (for bench.py's roofline figure).

A KernelTimer brackets every vae2_conv2d_fwd launch that uses one kernel
instantiation (by name, as rocprof reports it) with torch.cuda.Events recorded on
the stream the kernel is launched on, and accumulates the launch's algorithmic
FLOPs (2 * output pixels * Cout * Cin * k^2).
"""
import ctypes

import torch

from . import _lib

_ACTIVE = None


def active():
    return _ACTIVE


def fwd_kernel_name(xa, yshape, k, stride, pad):
    """Kernel instantiation vae2_conv2d_fwd uses for input act `xa` (aligned) and
    output shape (n, oh, ow, cout)."""
    buf = ctypes.create_string_buffer(64)
    n, oh, ow, cout = yshape
    y = _lib.Act(n, oh, ow, cout, cout)
    _lib.check(_lib.load().vae2_conv2d_fwd_kernel_name(ctypes.byref(xa), ctypes.byref(y), k,
                                                       stride, pad, buf, 64))
    return buf.value.decode()


class KernelTimer:
    def __init__(self, kernel_name):
        self.kernel_name = kernel_name
        self.events = []
        self.flops = []
        self.bytes = []
        self.enabled = False
        self._names = {}

    def __enter__(self):
        global _ACTIVE
        _ACTIVE = self
        self.enabled = True
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = None
        self.enabled = False

    def matches(self, xa, yshape, spec):
        key = (xa.n, xa.h, xa.w, xa.c, xa.ps, yshape, spec.k, spec.stride, spec.pad)
        if key not in self._names:
            self._names[key] = fwd_kernel_name(xa, yshape, spec.k, spec.stride, spec.pad)
        return self._names[key] == self.kernel_name

    def record(self, flops, nbytes=0.0):
        """Start timing one launch on the current stream.  The launch is isolated
        from the side streams (they are waited for before it, and wait for it
        after) so the event span is the kernel's own execution, as rocprof sees it,
        not time spent queued behind a concurrent stream."""
        from . import streams
        streams.join_all()
        self.bytes.append(nbytes)
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record(torch.cuda.current_stream())
        self.events.append((s, e))
        self.flops.append(flops)
        return e

    @staticmethod
    def finish(ev):
        from . import streams
        cur = torch.cuda.current_stream()
        ev.record(cur)
        streams.fence_side(cur)

    def summary(self):
        torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e in self.events]
        n = len(ms)
        if n == 0:
            return None
        tot_ms = sum(ms)
        return {"launches": n, "avg_us": 1e3 * tot_ms / n,
                "flops_per_launch": sum(self.flops) / n,
                "bytes_per_launch": sum(self.bytes) / n,
                "tflops": sum(self.flops) / (tot_ms * 1e-3) / 1e12}

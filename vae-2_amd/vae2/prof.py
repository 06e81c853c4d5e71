"""Live per-kernel timing with HIP events (bench.py's roofline and per-family table).

StepProfiler brackets every C-ABI call of libvae2_hip with torch.cuda.Events on the
stream the call launches on, and attributes the span to the kernels the call
launched (the library's launch log, vae2_kernel_log: names as rocprofv3 reports
them).  Each timed call is isolated from the side streams (they are waited for
before it and wait for it after), so an event span is the kernels' own execution,
as rocprof measures it, not time queued behind a concurrent stream.  The ops
annotate the calls they make with algorithmic work (note()): FLOPs for the convs,
bytes moved once for the memory-bound kernels, and a layer-shape label.

Algorithmic FLOPs of a conv: 2 * output pixels * Cout * Cin * k^2 (forward, data
gradient and weight gradient alike; the data gradient of a stride-2 conv counts
the same MACs).  Algorithmic bytes: every input read once, every output written
once (weights included for convs).
"""
import ctypes
import re
from collections import defaultdict

import torch

from . import _lib

_ACTIVE = None

# (family, regex on a kernel name), first match wins (also used by tools/trace_steps.py)
FAMILIES = (
    ("conv_fwd", r"dconv3_(group_)?kernel<\d+, \d+, false|dconv3s_kernel<\d+, \d+, \d+, false|"
                 r"igemm_kernel<\d+, \d+, \w+, 0"),
    ("conv_dgrad", r"dconv3_(group_)?kernel<\d+, \d+, true|dconv3s_kernel<\d+, \d+, \d+, true|"
                   r"igemm_kernel<\d+, \d+, \w+, [12]"),
    ("conv_wgrad", r"wgrad"),
    ("conv_1x1", r"gemm1x1"),  # persistent 1x1 GEMM: forward and data gradient
    ("batchnorm", r"bn_|reduce_then|chan_partials|partials_reduce"),
    ("heads", r"upsum|head_|up_adj"),
    ("fuse_resample", r"upsample|fuse_sum|relu_bwd|copy_act|tile_kernel|spatial_|codemap"),
    ("optimizer", r"adam|pack_weight"),
    ("loss_elbo", r"l1_|reparam|weighted_sum|finish_sum|scale_kernel|nonfinite|nchw|nhwc|"
                  r"sqdiff"),
    ("torch_aten", r"at::native|^at::"),
    ("copies", r"rocclr_copy|rocclr_fill"),
)

FP32_MFMA_PEAK_TF = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 dense
BF16_MFMA_PEAK_TF = 2500.0  # MI355X_MICROARCH.md: bf16 dense (no sparsity)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E
MFMA_PEAK_TF = FP32_MFMA_PEAK_TF  # the conv MFMA operand dtype in use (set_mfma_dtype)


def set_mfma_dtype(dtype):
    """Price conv FLOPs against the peak of the MFMA operand dtype ("fp32" / "bf16")."""
    global MFMA_PEAK_TF
    MFMA_PEAK_TF = BF16_MFMA_PEAK_TF if dtype == "bf16" else FP32_MFMA_PEAK_TF


def family(kernel):
    for f, rx in FAMILIES:
        if re.search(rx, kernel):
            return f
    return "other"


_ABI_FAMILY = (("conv_dgrad", "bwd_data"), ("conv_wgrad", "bwd_weight"), ("conv_fwd", "conv2d"),
               ("heads", "head_|upsum"), ("batchnorm", "bn_"))


def _abi_family(name):
    """Family of a C-ABI call that launched no kernel (its work still counts)."""
    for f, key in _ABI_FAMILY:
        if re.search(key, name):
            return f
    return "other"


def active():
    return _ACTIVE


def note(flops=0.0, nbytes=0.0, shape=None):
    """Annotate the NEXT C-ABI call with its own algorithmic work (no-op unless profiling).
    Every note belongs to exactly one call: a note still pending when another is made is
    counted in StepProfiler.conflicts (bench.py reports it; the profiler test asserts 0) and
    replaced.  A launch queued for a later call carries its note there (take / put)."""
    if _ACTIVE is not None:
        if _ACTIVE.pending is not None:
            _ACTIVE.conflicts += 1
        _ACTIVE.pending = (float(flops), float(nbytes), shape)


def take():
    """Pop the pending note (a queued launch: ops.ConvGroup stores it with the job)."""
    if _ACTIVE is None:
        return None
    w, _ACTIVE.pending = _ACTIVE.pending, None
    return w


def put(work):
    """Re-arm a note taken earlier for the call about to issue its launch."""
    if _ACTIVE is not None and work is not None:
        if _ACTIVE.pending is not None:
            _ACTIVE.conflicts += 1
        _ACTIVE.pending = work


def conv_label(kind, cin, cout, k, stride, h, w):
    return f"{kind} {cin}->{cout} k{k} s{stride} @{h}x{w}"


def fwd_kernel_name(xa, yshape, k, stride, pad):
    """Kernel instantiation vae2_conv2d_fwd uses for input act `xa` (aligned) and
    output shape (n, oh, ow, cout)."""
    buf = ctypes.create_string_buffer(64)
    n, oh, ow, cout = yshape
    y = _lib.Act(n, oh, ow, cout, cout)
    _lib.check(_lib.load().vae2_conv2d_fwd_kernel_name(ctypes.byref(xa), ctypes.byref(y), k,
                                                       stride, pad, buf, 64))
    return buf.value.decode()


_SLEEP_RATE = {}


def _sleep_cycles(us):
    """torch.cuda._sleep argument that spins the stream for about `us` microseconds
    (calibrated once per device against HIP events)."""
    dev = torch.cuda.current_device()
    rate = _SLEEP_RATE.get(dev)
    if rate is None:
        n = 1 << 20
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(n)  # warm
        a.record()
        torch.cuda._sleep(n)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b)
        rate = n / max(ms * 1e3, 1e-3)  # cycles per microsecond
        _SLEEP_RATE[dev] = rate
    return max(int(us * rate), 1)


class StepProfiler:
    def __init__(self, lead_us=40.0):
        self.records = []  # (abi fn, kernels label, start ev, end ev, flops, bytes, shape)
        self.pending = None
        self.lead_cycles = _sleep_cycles(lead_us) if lead_us else 0
        self.conflicts = 0  # notes overwritten before their call (must stay 0)
        self._buf = ctypes.create_string_buffer(1 << 14)

    def __enter__(self):
        global _ACTIVE
        _ACTIVE = self
        _lib.load().vae2_kernel_log(1)
        _lib.CALL_HOOK = self._call
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = None
        _lib.CALL_HOOK = None
        _lib.load().vae2_kernel_log(0)

    def _call(self, name, fn, args):
        from . import streams
        lib = _lib.load()
        streams.join_all()
        cur = torch.cuda.current_stream()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        lib.vae2_kernel_log_read(None, 0)  # drop launches made outside annotated calls
        # keep the stream busy while the host queues the start event, the call's kernels
        # and the end event: the bracket then holds the kernels' execution, not the host's
        # launch latency (the eager profiled step is host-bound, so without it every short
        # kernel's span included the gap before its launch)
        if self.lead_cycles:
            torch.cuda._sleep(self.lead_cycles)
        s.record(cur)
        rc = fn(*args)
        e.record(cur)
        streams.fence_side(cur)
        n = lib.vae2_kernel_log_read(self._buf, len(self._buf))
        work = self.pending or (0.0, 0.0, None)
        self.pending = None
        # a call that launched nothing keeps its record (zero time): its work still counts
        self.records.append((name, self._buf.value.decode() if n > 0 else "", s, e) + work)
        return rc

    def summary(self, steps):
        """Per kernel (as rocprof names it), per family and per conv layer shape:
        time per step, launches per step, algorithmic FLOPs / bytes and the rates."""
        torch.cuda.synchronize()
        ker = defaultdict(lambda: [0.0, 0, 0.0, 0.0])
        fam = defaultdict(lambda: [0.0, 0, 0.0, 0.0])
        shp = defaultdict(lambda: [0.0, 0, 0.0, 0.0])
        total = 0.0
        for name, kernels, s, e, flops, nbytes, shape in self.records:
            ms = s.elapsed_time(e) if kernels else 0.0
            total += ms
            ks = kernels.split(";")
            fk = family(ks[0]) if kernels else _abi_family(name)
            for d, key in ((ker, kernels or name), (fam, fk)):
                d[key][0] += ms
                d[key][1] += 1
                d[key][2] += flops
                d[key][3] += nbytes
            if shape is not None:  # one row per (layer shape, launched kernel instance)
                d = shp[f"{shape} | {kernels or '(no launch)'}"]
                d[0] += ms
                d[1] += 1
                d[2] += flops
                d[3] += nbytes

        def rows(d):
            out = []
            for k, (ms, n, fl, by) in sorted(d.items(), key=lambda kv: -kv[1][0]):
                r = {"name": k, "ms_per_step": round(ms / steps, 4),
                     "launches_per_step": round(n / steps, 2),
                     "avg_us": round(1e3 * ms / max(n, 1), 2)}
                if fl:
                    r["gflop_per_step"] = round(fl / steps / 1e9, 3)
                    r["tflops"] = round(fl / (ms * 1e-3) / 1e12, 2)
                    r["frac_mfma_peak"] = round(fl / (ms * 1e-3) / 1e12 / MFMA_PEAK_TF, 4)
                if by:
                    r["gb_per_step"] = round(by / steps / 1e9, 3)
                    r["gbs"] = round(by / (ms * 1e-3) / 1e9, 1)
                    r["frac_hbm_peak"] = round(by / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                out.append(r)
            return out

        return {"kernel_ms_per_step": round(total / steps, 3), "families": rows(fam),
                "kernels": rows(ker), "conv_shapes": rows(shp), "note_conflicts": self.conflicts}

    def dominant(self, steps):
        """The single kernel (one instantiation) with the most time: its launches'
        average duration and algorithmic work per launch (the roofline object)."""
        torch.cuda.synchronize()
        agg = defaultdict(lambda: [0.0, 0, 0.0, 0.0])
        for name, kernels, s, e, flops, nbytes, shape in self.records:
            if ";" in kernels or not kernels:
                continue
            a = agg[kernels]
            a[0] += s.elapsed_time(e)
            a[1] += 1
            a[2] += flops
            a[3] += nbytes
        if not agg:
            return None
        k, (ms, n, fl, by) = max(agg.items(), key=lambda kv: kv[1][0])
        avg_s = ms * 1e-3 / n
        out = {"kernel": k, "launches": n, "avg_launch_us": round(avg_s * 1e6, 2),
               "ms_per_step": round(ms / steps, 3), "flops_per_launch": fl / n,
               "algorithmic_bytes_per_launch": by / n}
        if fl > 0:
            out.update(bound="mfma", achieved=round(fl / n / avg_s / 1e12, 3),
                       peak=MFMA_PEAK_TF, unit="TFLOP/s")
        else:
            out.update(bound="hbm", achieved=round(by / n / avg_s / 1e9, 1),
                       peak=HBM_PEAK_GBS, unit="GB/s")
        out["frac"] = round(out["achieved"] / out["peak"], 4)
        return out

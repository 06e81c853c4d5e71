"""Per-branch head path (vae2/heads.py) against the reference's formulation in fp64.

Reference (enc_hrnet.py:833-847, :323-370): x = cat([y0, up(y1), up(y2), up(y3)]),
out_k = Conv1x1(ReLU(BN_train(Conv1x1(x)))), cat over k.  The HIP path computes the
wide conv per branch at the branch resolution; it is the same linear map, so it is
held to fp64 of the reference formulation at fp32 accuracy: outputs and running
statistics 1e-5 relative; every input / parameter gradient within relative-L2
max(1e-4, 3 x the distance of the reference formulation run in fp32) of fp64 (the BN
backward cancels, so fp32 gradient accuracy falls with the pixel count for any
implementation; the conv biases in front of BN have an analytically zero gradient and
are held to an absolute bound against the gradient scale instead).
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from helpers import build, make_cfg, max_rel, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


def ref_heads(heads, ys):
    """fp64 reference formulation on NCHW tensors (the reference's own op sequence)."""
    H, W = ys[0].shape[2:]
    x = torch.cat([ys[0]] + [F.interpolate(y, size=(H, W), mode="bilinear", align_corners=False)
                             for y in ys[1:]], 1)
    outs = []
    for h in heads:
        r = F.conv2d(x, h[0].weight, h[0].bias)
        r = F.batch_norm(r, h[1].running_mean, h[1].running_var, h[1].weight, h[1].bias,
                         training=True, momentum=h[1].momentum, eps=h[1].eps)
        outs.append(F.conv2d(F.relu(r), h[3].weight, h[3].bias))
    return torch.cat(outs, 1)


def _heads_and_inputs(arch, hw, n, seed=0):
    ed, _ = build(make_cfg(arch, hw=hw))
    heads = [getattr(ed, f"last_layer_{k}") for k in (1, 2, 3)]
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for h in heads:  # O(1) activations (the reference init std 0.001 makes BN see ~0)
            for m in (h[0], h[3]):
                m.weight.normal_(0, (1.0 / m.in_channels) ** 0.5, generator=g)
                m.bias.normal_(0, 0.1, generator=g)
            h[1].weight.uniform_(0.5, 1.5, generator=g)
            h[1].bias.normal_(0, 0.1, generator=g)
    split = ed.last_stage_channels
    sizes = [hw]
    for _ in split[1:]:
        h_, w_ = sizes[-1]
        sizes.append(((h_ + 1) // 2, (w_ + 1) // 2))  # stride-2 3x3 convs
    ys = [torch.randn(n, c, s[0], s[1], generator=g) for c, s in zip(split, sizes)]
    return heads, ys


@pytest.mark.parametrize("arch,hw,n", [("w18", (32, 64), 2), ("tiny", (30, 22), 3),
                                       ("w18", (34, 50), 2), ("w18", (64, 128), 2)])
def test_heads_match_reference_formulation(arch, hw, n):
    from vae2 import heads as vheads
    heads, ys = _heads_and_inputs(arch, hw, n)
    assert vheads.supported(heads, [y.shape[1] for y in ys])
    ref_h = [copy.deepcopy(h).double() for h in heads]
    ys_ref = [y.double().requires_grad_() for y in ys]
    out_ref = ref_heads(ref_h, ys_ref)
    gout = torch.randn(out_ref.shape, generator=torch.Generator().manual_seed(7),
                       dtype=torch.float64)
    (out_ref * gout).sum().backward()
    f32_h = [copy.deepcopy(h).float() for h in heads]
    ys_f32 = [y.clone().requires_grad_() for y in ys]
    (ref_heads(f32_h, ys_f32) * gout.float()).sum().backward()

    def tol(a32, a64):
        return max(1e-4, 3 * rel(a32, a64))

    hip_h = [copy.deepcopy(h).to(DEV) for h in heads]
    ys_hip = [y.detach().permute(0, 2, 3, 1).contiguous().to(DEV).requires_grad_() for y in ys]
    out = vheads.run(hip_h, ys_hip)
    out.backward(gout.float().permute(0, 2, 3, 1).contiguous().to(DEV))
    torch.cuda.synchronize()

    got = out.detach().permute(0, 3, 1, 2).cpu()
    assert max_rel(got, out_ref) < 1e-5, max_rel(got, out_ref)
    for yh, yr, y32 in zip(ys_hip, ys_ref, ys_f32):
        e = rel(yh.grad.permute(0, 3, 1, 2), yr.grad)
        assert e < tol(y32.grad, yr.grad), (e, rel(y32.grad, yr.grad))
    for hh, hr, h32 in zip(hip_h, ref_h, f32_h):
        for (name, p), (_, pr), (_, p32) in zip(hh.named_parameters(), hr.named_parameters(),
                                                h32.named_parameters()):
            if name == "0.bias":  # analytically zero in front of BN: rounding-level only
                scale = float(hr[0].weight.grad.abs().max())
                assert float(p.grad.abs().max()) < 1e-4 * scale, (name, p.grad.abs().max())
                continue
            e = rel(p.grad, pr.grad)
            assert e < tol(p32.grad, pr.grad), (name, e, rel(p32.grad, pr.grad))
        for name in ("running_mean", "running_var"):
            a, b = getattr(hh[1], name), getattr(hr[1], name)
            assert max_rel(a, b) < 1e-5, (name, max_rel(a, b))
        assert int(hh[1].num_batches_tracked) == 1  # (F.batch_norm does not count)


def test_heads_packed_cols_follow_optimizer_updates():
    """The PackPlan's per-branch packed blocks track in-place weight updates."""
    from vae2 import heads as vheads
    from vae2.optim import FusedAdam
    heads, ys = _heads_and_inputs("tiny", (16, 16), 2)
    mod = torch.nn.ModuleList(heads).to(DEV)
    opt = FusedAdam([mod], lr=1e-2)
    ys_d = [y.permute(0, 2, 3, 1).contiguous().to(DEV) for y in ys]
    for _ in range(2):
        opt.zero_grad()
        out = vheads.run(list(mod), ys_d)
        out.square().sum().backward()
        opt.step()
    # after the updates, a fresh eager evaluation must equal the reference formulation
    ref_h = [copy.deepcopy(h).double().cpu() for h in mod]
    for h in ref_h:  # undo the running-stat updates of the HIP forward we compare against
        h[1].reset_running_stats()
    with torch.no_grad():
        hip_h = [copy.deepcopy(h) for h in mod]
        for h in hip_h:
            h[1].reset_running_stats()
        got = vheads.run(hip_h, ys_d).permute(0, 3, 1, 2).cpu()
        want = ref_heads(ref_h, [y.double() for y in ys])
    assert max_rel(got, want) < 1e-5, max_rel(got, want)


@pytest.mark.parametrize("hw,n", [((64, 128), 2), ((32, 64), 3)])
def test_upsample_adjoint_streaming_equals_lane_kernel(hw, n):
    """The row-streaming vertical pass of the power-of-two upsampling adjoint
    (up_adj2_vs_kernel) against the per-channel-lane one (vae2_heads_set_algo bit 0), both
    in the two-pass form (bit 2): same weights, same summation order."""
    from vae2 import _lib
    from vae2 import heads as vheads
    heads, ys = _heads_and_inputs("w18", hw, n)
    gout = None
    grads = []
    lib = _lib.load()
    try:
        for algo in (4, 5):
            lib.vae2_heads_set_algo(algo)
            hip_h = [copy.deepcopy(h).to(DEV) for h in heads]
            ys_hip = [y.permute(0, 2, 3, 1).contiguous().to(DEV).requires_grad_() for y in ys]
            out = vheads.run(hip_h, ys_hip)
            if gout is None:
                gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(3)).to(DEV)
            out.backward(gout)
            torch.cuda.synchronize()
            grads.append([y.grad.cpu() for y in ys_hip])
    finally:
        lib.vae2_heads_set_algo(0)
    for a, b in zip(*grads):
        assert max_rel(a, b) < 1e-6, max_rel(a, b)


@pytest.mark.parametrize("n,c,H,W,nsrc", [(2, 270, 64, 128, 3), (1, 70, 8, 64, 3),
                                          (1, 18, 96, 192, 3), (2, 36, 40, 128, 2),
                                          (1, 20, 34, 64, 1), (3, 64, 32, 64, 3)])
def test_upsample_adjoint_multi_against_fp64(n, c, H, W, nsrc):
    """vae2_upsample_bilinear_bwd_multi (the heads' dL/dz_j = up_j^T(dL/dy)) against
    torch's fp64 autograd of F.interpolate(bilinear, align_corners=False)
    (enc_hrnet.py:839-845): the one-pass band kernel at its default and at 8 / 64 dy rows
    per workgroup, and the two-pass form (vae2_heads_set_algo bit 2).  Shapes cover one
    band, several bands, a last band shorter than the others, 1-row coarsest targets (both
    vertical folds in one row) and pad channels (c % 64 != 0)."""
    import ctypes
    from vae2 import _lib, ops
    from vae2._lib import Act, call
    lib = _lib.load()
    g = torch.Generator().manual_seed(H * W + c)
    dy = torch.randn(n, c, H, W, generator=g, dtype=torch.float64)
    refs = []
    for s in range(nsrc):
        z = torch.zeros(n, c, H >> (s + 1), W >> (s + 1), dtype=torch.float64,
                        requires_grad=True)
        F.interpolate(z, size=(H, W), mode="bilinear", align_corners=False).backward(dy)
        refs.append(z.grad)
    gt = ops.new_act((n, H, W, c), torch.empty(0, device=DEV))
    gt.copy_(dy.float().permute(0, 2, 3, 1))
    gp, ga = ops.act_of(gt)
    try:
        for algo in (0, 8 << 8, 64 << 8, 4):
            lib.vae2_heads_set_algo(algo)
            dxs = [ops.new_act((n, H >> (s + 1), W >> (s + 1), c), gt) for s in range(nsrc)]
            for d in dxs:
                d.fill_(float("nan"))  # every target element must be written
            views = [ops.act_of(d) for d in dxs]
            acts = (Act * 3)(*[a for _, a in views])
            ptrs = (ctypes.c_void_p * 3)(*[p for p, _ in views])
            wsz = lib.vae2_upsample_bilinear_bwd_multi_ws_size(ctypes.byref(ga), nsrc, acts)
            ws = torch.empty(max(wsz, 1), device=DEV)
            call("vae2_upsample_bilinear_bwd_multi", gp, ctypes.byref(ga), nsrc, ptrs, acts,
                 ws.data_ptr(), wsz, None)
            torch.cuda.synchronize()
            for d, r in zip(dxs, refs):
                got = d.permute(0, 3, 1, 2).double().cpu()
                assert torch.isfinite(got).all(), algo
                assert max_rel(got, r) < 2e-6, (algo, max_rel(got, r))
    finally:
        lib.vae2_heads_set_algo(0)


@pytest.mark.parametrize("n,H,W,cin,nup", [(2, 64, 128, 18, 3), (1, 128, 256, 18, 3),
                                           (2, 32, 64, 7, 2), (1, 16, 64, 4, 1)])
def test_upsum_one_pass_against_fp64(n, H, W, cin, nup):
    """vae2_conv1x1_upsum_fwd's one-pass kernel (upsum2_kernel: W0 x0 on MFMA, source rows
    in registers) and the LDS-staged one (vae2_heads_set_algo bit 3) against fp64 of
    y = W0 x0 + b + sum_j up(z_j) (enc_hrnet.py:839-847 with the 1x1 conv commuted),
    and the shifted BN statistics rows of y - b summed over rows."""
    import ctypes
    from vae2 import _lib, ops
    from vae2._lib import Act, call
    lib = _lib.load()
    g = torch.Generator().manual_seed(n * H + cin)
    C = 270
    x0 = torch.randn(n, cin, H, W, generator=g, dtype=torch.float64)
    zs = [torch.randn(n, C, H >> (s + 1), W >> (s + 1), generator=g, dtype=torch.float64)
          for s in range(nup)]
    w = torch.randn(C, cin, generator=g, dtype=torch.float64) / cin ** 0.5
    b = torch.randn(C, generator=g, dtype=torch.float64)
    ref = torch.einsum("ck,nkhw->nchw", w, x0)
    for z in zs:
        ref = ref + F.interpolate(z, size=(H, W), mode="bilinear", align_corners=False)
    s1, s2 = ref.sum((0, 2, 3)), (ref * ref).sum((0, 2, 3))
    ref = ref + b[None, :, None, None]
    dev = torch.empty(0, device=DEV)
    xa = ops.new_act((n, H, W, cin), dev)
    xa.copy_(x0.float().permute(0, 2, 3, 1))
    xp, xd = ops.act_of(xa)
    za = []
    for z in zs:
        t = ops.new_act((n, z.shape[2], z.shape[3], C), dev)
        t.copy_(z.float().permute(0, 2, 3, 1))
        za.append(t)
    wd = w.float().to(DEV).contiguous()
    wp = torch.empty(lib.vae2_conv2d_packed_size(C, cin, 1, 0), device=DEV)
    call("vae2_conv2d_pack_weight_ld", ops.ptr(wd), C, cin, 1, 0, cin, ops.ptr(wp), None)
    bd = b.float().to(DEV)
    ya = Act(n, H, W, C, C)
    rows = lib.vae2_conv1x1_upsum_stats_rows(ctypes.byref(ya))
    ups = (ctypes.c_void_p * 3)(*[ops.act_of(t)[0] for t in za])
    upds = (Act * 3)(*[ops.act_of(t)[1] for t in za])
    ncb = -(-C // 64)
    try:
        for algo in (0, 8):
            lib.vae2_heads_set_algo(algo)
            y = torch.full((ncb * n * H * W * 64,), float("nan"), device=DEV)
            stats = torch.empty(2 * rows * C, device=DEV)
            call("vae2_conv1x1_upsum_fwd", xp, ctypes.byref(xd), ops.ptr(wp), ops.ptr(bd), nup,
                 ups, upds, ops.ptr(y), ctypes.byref(ya), ops.ptr(stats), None)
            torch.cuda.synchronize()
            got = y.view(ncb, n, H, W, 64).permute(1, 0, 4, 2, 3).reshape(n, ncb * 64, H, W)
            got = got[:, :C].double().cpu()
            assert max_rel(got, ref) < 1e-5, (algo, max_rel(got, ref))
            st = stats.view(2, rows, C).double().sum(1).cpu()
            assert max_rel(st[0], s1) < 1e-4, (algo, max_rel(st[0], s1))
            assert max_rel(st[1], s2) < 1e-5, (algo, max_rel(st[1], s2))
    finally:
        lib.vae2_heads_set_algo(0)

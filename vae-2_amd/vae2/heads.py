"""The three output heads of an HRNet stack, computed per branch.

Reference (enc_hrnet.py:833-847 encoder, :889-905 / :947-963 decoders):

    x = cat([y0, up(y1), up(y2), up(y3)], channels)          # C = 18+36+72+144 = 270
    out_k = last_layer_k(x)   k = 1..3                      # :323-370
          = Conv1x1(C->NC, bias)(ReLU(BN(Conv1x1(C->C, bias)(x))))
    return cat([out_1, out_2, out_3], channels)

A 1x1 conv commutes with the bilinear upsampling, so with W = [W0 | W1 | W2 | W3]
split by input branch

    Conv1x1(x) = W0 y0 + b + up(W1 y1) + up(W2 y2) + up(W3 y3)

and the branch products run at the branch's own resolution (1/4, 1/16, 1/64 of the
pixels): the wide conv costs sum_j C*c_j*P_j instead of C*C*P MACs (8x fewer for
w18), the 270-channel concatenation is never materialised, and in the backward the
upsampling adjoint is applied once to the conv's output gradient.  The result is the
same linear map up to fp32 summation order (tests/test_heads_gpu.py holds it to the
oracle).  Kernels:

  vae2_conv2d_fwd          z_j = W_j y_j              (j >= 1, branch resolution)
  vae2_conv1x1_upsum_fwd   y = W0 y0 + b + sum_j up(z_j), BN partial stats fused
  vae2_bn_reduce_finalize_shifted  BN batch statistics of y - b (SyncBN: reduce, all-reduce,
                           finalize)
  vae2_head_out_fwd        out = W2 ReLU(BN(y)) + b2 (the ReLU output is never stored)
  backward: vae2_head_out_bwd_reduce / _apply (-> dL/dy), vae2_upsample_bilinear_bwd_multi
  (dL/dz_j for all branches, dL/dy read once), vae2_conv2d_bwd_weight_ld (dW_j into
  column blocks of dW) and vae2_conv2d_bwd_data (dL/dy_j, summed over the three heads).
"""
import ctypes

import torch

from . import _lib, prof
from ._lib import Act, call
from .ops import (_WS_HOLD, _all_reduce_sums, _bn_group, _defer_off, _empty, _grad_sink, act_of,
                  as_act, new_act, packed_weight_cols, ptr, stream_ptr, wgrad_batch)

_PER_HEAD = 6  # conv weight, conv bias, BN weight, BN bias, out weight, out bias


def supported(heads, split):
    """True when the per-branch path applies: 1x1 convs, <= 4 branches, <= 4 outputs."""
    if not heads or any(h is None for h in heads) or not 1 <= len(split) <= 4:
        return False
    for h in heads:
        c0, bn, c3 = h[0], h[1], h[3]
        if c0.kernel_size != (1, 1) or c3.kernel_size != (1, 1) or c0.stride != (1, 1):
            return False
        if c3.stride != (1, 1) or c3.padding != (0, 0) or c0.padding != (0, 0):
            return False
        if c0.in_channels != sum(split) or c3.out_channels > 4 or bn.momentum is None:
            return False
        if c0.groups != 1 or c3.groups != 1:
            return False
    return True


def mark_split(heads, split):
    """Let the optimizer's PackPlan pack the wide head convs per branch block."""
    if supported(heads, split):
        for h in heads:
            h[0]._vae2_col_split = tuple(split)


class _Heads(torch.autograd.Function):
    @staticmethod
    def forward(ctx, heads, nb, *args):
        ys, params = args[:nb], args[nb:]
        lib = _lib.load()
        s = stream_ptr()
        split = tuple(int(y.shape[3]) for y in ys)
        x0 = ys[0]
        n, H, W, _ = x0.shape
        C = sum(split)
        nh = len(heads)
        ncls = heads[0][3].out_channels
        out = new_act((n, H, W, ncls * nh), x0)
        x0p, x0a = act_of(x0)
        yshape = Act(n, H, W, C, (C + 3) // 4 * 4)
        rows = lib.vae2_conv1x1_upsum_stats_rows(ctypes.byref(yshape))
        count = float(n * H * W)
        group = _bn_group()
        training = [h[1].training or not h[1].track_running_stats for h in heads]
        ys_saved, saves = [], []
        for k, head in enumerate(heads):
            w, b, gamma, beta, w2, b2 = params[_PER_HEAD * k:_PER_HEAD * (k + 1)]
            bn = head[1]
            # branch products at their own resolution
            zs = []
            for j in range(1, nb):
                yj = ys[j]
                z = new_act((yj.shape[0], yj.shape[1], yj.shape[2], C), yj)
                yjp, yja = act_of(yj)
                zp, za = act_of(z)
                if prof.active():
                    pj = yja.n * yja.h * yja.w
                    prof.note(2.0 * pj * C * yja.c, 4.0 * (pj * yja.c + pj * C + C * yja.c),
                              prof.conv_label("head fwd", yja.c, C, 1, 1, yja.h, yja.w))
                call("vae2_conv2d_fwd", yjp, ctypes.byref(yja),
                     ptr(packed_weight_cols(w, split, j, 0)), None, zp, ctypes.byref(za), 1, 1, 0,
                     0.0, None, s)
                zs.append((z, zp, za))
            ups = (ctypes.c_void_p * 3)(*[zp for _, zp, _ in zs])
            upds = (Act * 3)(*[za for _, _, za in zs])
            y = _empty((-(-C // 64) * n * H * W * 64,), x0)  # B64 layout (heads.hip)
            yp, ya = ptr(y), yshape
            stats = _empty((2 * rows * C,), x0) if training[k] else None
            P0 = n * H * W
            if prof.active():  # W0 x0 on MFMA + the upsampled branch products, y written once
                prof.note(2.0 * P0 * C * split[0],
                          4.0 * (P0 * split[0] + P0 * C + sum(z.numel() for z, _, _ in zs)),
                          prof.conv_label("head upsum", split[0], C, 1, 1, H, W))
            call("vae2_conv1x1_upsum_fwd", x0p, ctypes.byref(x0a),
                 ptr(packed_weight_cols(w, split, 0, 0)), ptr(b), nb - 1, ups, upds, yp,
                 ctypes.byref(ya), ptr(stats), s)
            save = _empty((4 * C,), x0)
            if training[k]:
                sums = _empty((2 * C,), x0, torch.float64)
                track = bn.track_running_stats and bn.running_mean is not None
                stat_ptrs = (ptr(bn.running_mean) if track else None,
                             ptr(bn.running_var) if track else None,
                             ptr(bn.num_batches_tracked) if track else None)
                if group is None:
                    if count <= 1:
                        raise ValueError("Expected more than 1 value per channel when training, "
                                         f"got input size {(n, C, H, W)}")
                    call("vae2_bn_reduce_finalize_shifted", ptr(stats), rows, C, ptr(sums),
                         count, ptr(b), ptr(gamma), ptr(beta), *stat_ptrs, float(bn.momentum),
                         float(bn.eps), ptr(save), s)
                    gcount = count
                else:
                    call("vae2_bn_partials_reduce", ptr(stats), rows, C, ptr(sums), 0, s)
                    sums, gcount = _all_reduce_sums(sums, count, group)
                    if gcount <= 1:
                        raise ValueError("Expected more than 1 value per channel when training")
                    call("vae2_bn_finalize_shifted", ptr(sums), gcount, ptr(b), ptr(gamma),
                         ptr(beta), *stat_ptrs, float(bn.momentum), float(bn.eps), C, ptr(save),
                         s)
            else:
                gcount = count
                call("vae2_bn_eval_coeffs", ptr(gamma), ptr(beta), ptr(bn.running_mean),
                     ptr(bn.running_var), float(bn.eps), C, ptr(save), s)
            o = out[..., ncls * k:ncls * (k + 1)]
            op, oa = act_of(o)
            if prof.active():
                prof.note(2.0 * P0 * C * ncls, 4.0 * (P0 * C + P0 * ncls),
                          prof.conv_label("head out", C, ncls, 1, 1, H, W))
            call("vae2_head_out_fwd", yp, ctypes.byref(ya), ptr(save), ptr(w2), ptr(b2), ncls, op,
                 ctypes.byref(oa), s)
            ys_saved.append(y)
            saves.append(save)
        ctx.heads = heads
        ctx.nb = nb
        ctx.split = split
        ctx.count = gcount
        ctx.group = group
        ctx.training = training
        ctx.params = params
        ctx.save_for_backward(*ys, *ys_saved, *saves)
        return out

    @staticmethod
    def backward(ctx, dout):
        if not all(ctx.training):
            raise RuntimeError("backward through an eval-mode BatchNorm is not supported")
        lib = _lib.load()
        s = stream_ptr()
        nb, heads, split = ctx.nb, ctx.heads, ctx.split
        nh = len(heads)
        saved = ctx.saved_tensors
        ys, yv, saves = saved[:nb], saved[nb:nb + nh], saved[nb + nh:]
        ncls = heads[0][3].out_channels
        C = sum(split)
        dout = as_act(dout)
        dxs = [None] * nb
        pgrads = []
        need = ctx.needs_input_grad[2 + nb:]
        for k in range(nh):
            w, b, gamma, beta, w2, b2 = ctx.params[_PER_HEAD * k:_PER_HEAD * (k + 1)]
            nw, nbias, ng, nbt, nw2, nb2 = need[_PER_HEAD * k:_PER_HEAD * (k + 1)]
            y, save = yv[k], saves[k]
            yp, ya = ptr(y), Act(*ys[0].shape[:3], C, C)
            dk = dout[..., ncls * k:ncls * (k + 1)]
            dkp, dka = act_of(dk)
            wsz = lib.vae2_head_out_bwd_ws_size(ctypes.byref(ya), ncls)
            ws = _empty((wsz,), y)
            lsums = _empty((2 * C,), y, torch.float64)
            gsink, gret = _grad_sink(gamma, ng)
            btsink, btret = _grad_sink(beta, nbt)
            w2sink, w2ret = _grad_sink(w2, nw2)
            b2sink, b2ret = _grad_sink(b2, nb2)
            P0 = ys[0].shape[0] * ys[0].shape[1] * ys[0].shape[2]
            Hh, Ww = ys[0].shape[1], ys[0].shape[2]
            if prof.active():  # the 270 -> 3 conv's weight gradient + BN backward sums
                prof.note(2.0 * P0 * C * ncls, 4.0 * (P0 * C + P0 * ncls),
                          prof.conv_label("head out wgrad", C, ncls, 1, 1, Hh, Ww))
            call("vae2_head_out_bwd_reduce", yp, ctypes.byref(ya), ptr(save), ptr(w2), ncls, dkp,
                 ctypes.byref(dka), ptr(lsums), ptr(gsink), ptr(btsink), ptr(w2sink),
                 ptr(b2sink), ptr(ws), wsz, s)
            gsums, _ = _all_reduce_sums(lsums, ctx.count, ctx.group)
            dy = new_act((*ys[0].shape[:3], C), y)
            dyp, dya = act_of(dy)
            bsink, bret = _grad_sink(b, nbias)
            if prof.active():  # the 270 -> 3 conv's data gradient + BN backward, dL/dy written
                prof.note(2.0 * P0 * C * ncls, 4.0 * (2 * P0 * C + P0 * ncls),
                          prof.conv_label("head out dgrad", C, ncls, 1, 1, Hh, Ww))
            call("vae2_head_out_bwd_apply", yp, ctypes.byref(ya), ptr(save), ptr(gamma), ptr(w2),
                 ncls, dkp, ctypes.byref(dka), ptr(gsums), ctx.count, dyp, ctypes.byref(dya),
                 ptr(bsink), ptr(ws), wsz, s)
            wsink, wret = _grad_sink(w, nw)
            # dL/dz_j = up_j^T(dL/dy) for every lower branch, dL/dy read once
            gs = [(dy, dyp, dya)]
            for xj in ys[1:]:
                g = new_act((xj.shape[0], xj.shape[1], xj.shape[2], C), xj)
                gs.append((g, *act_of(g)))
            if nb > 1:
                gptrs = (ctypes.c_void_p * 3)(*[gp for _, gp, _ in gs[1:]])
                gacts = (Act * 3)(*[ga for _, _, ga in gs[1:]])
                usz = lib.vae2_upsample_bilinear_bwd_multi_ws_size(ctypes.byref(dya), nb - 1, gacts)
                uws = _empty((usz,), y)
                if prof.active():
                    prof.note(0.0, 4.0 * (dy.numel() + sum(g.numel() for g, _, _ in gs[1:])))
                call("vae2_upsample_bilinear_bwd_multi", dyp, ctypes.byref(dya), nb - 1, gptrs,
                     gacts, ptr(uws), usz, s)
            c0 = 0
            with wgrad_batch():  # the branch blocks' dW reductions in one launch
                for j in range(nb):
                    xj = ys[j]
                    g, gp, ga = gs[j]
                    xjp, xja = act_of(xj)
                    if wsink is not None:
                        wsz2 = lib.vae2_conv2d_bwd_weight_ws_size(ctypes.byref(xja),
                                                                  ctypes.byref(ga), 1)
                        ws2 = _empty((max(wsz2, 1),), xj)
                        if prof.active():
                            pj = xja.n * xja.h * xja.w
                            prof.note(2.0 * pj * xja.c * C, 4.0 * (pj * xja.c + pj * C + C * xja.c),
                                      prof.conv_label("head wgrad", xja.c, C, 1, 1, xja.h, xja.w))
                        with _defer_off(wret is not None):  # autograd takes wret on return
                            call("vae2_conv2d_bwd_weight_ld", xjp, ctypes.byref(xja), gp,
                                 ctypes.byref(ga), ctypes.c_void_p(wsink.data_ptr() + 4 * c0),
                                 C, None, 1, 1, 0, 1, ptr(ws2), wsz2, s)
                        if wret is None:
                            _WS_HOLD.append((torch.cuda.current_stream().cuda_stream, ws2))
                    if ctx.needs_input_grad[2 + j]:
                        first = dxs[j] is None
                        if first:
                            dxs[j] = new_act(tuple(xj.shape), xj)
                        dxp, dxa = act_of(dxs[j])
                        if prof.active():
                            pj = dxa.n * dxa.h * dxa.w
                            prof.note(2.0 * pj * dxa.c * C, 4.0 * (pj * dxa.c + pj * C + C * dxa.c),
                                      prof.conv_label("head dgrad", dxa.c, C, 1, 1, dxa.h, dxa.w))
                        call("vae2_conv2d_bwd_data", gp, ctypes.byref(ga),
                             ptr(packed_weight_cols(w, split, j, 1)), dxp, ctypes.byref(dxa), 1,
                             1, 0, 0.0 if first else 1.0, s)
                    c0 += split[j]
            pgrads += [wret, bret, gret, btret, w2ret, b2ret]
        return (None, None, *dxs, *pgrads)


def run(heads, ys):
    """cat([last_layer_k(cat([y0, up(y1), ...])) for k]) on NHWC branch maps."""
    params = []
    for h in heads:
        params += [h[0].weight, h[0].bias, h[1].weight, h[1].bias, h[3].weight, h[3].bias]
    return _Heads.apply(tuple(heads), len(ys), *ys, *params)

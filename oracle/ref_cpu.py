"""ORACLE — test infrastructure only, never on the product path.

CPU fp32 restatement of the reference's VAE² ELBO step with plain PyTorch CPU
operators on NCHW tensors.  Only tests/, __graft_entry__.smoke() and bench.py's
`cpu_baseline` leg may import this module, and only as the checker / baseline;
the product path (vae2.*) must never call it.

It walks the parameter tree of the vae2.hrnet modules (whose shape, names and
seeded initialisation are verified identical to the reference's) and evaluates
the reference's forward semantics:

  conv3x3 / BasicBlock / Bottleneck      enc_hrnet.py:27-103
  HighResolutionModule.forward (fuse)    enc_hrnet.py:226-250
  transitions / stages                   enc_hrnet.py:796-831
  code maps + transition3_e              enc_hrnet.py:454-462, :818-830, :880-888, :938-946
  heads (upsample + cat + 3 heads)       enc_hrnet.py:833-847
  HighResolutionNetED.forward            enc_hrnet.py:965-981
  HighResolutionNetEDz.forward           enc_hrnet.py:1070-1122
  FullModel_encdec.forward (reparam,     utils.py:67-155
    L1 / KL, loss assembly)              criterion.py:61-87
  HighResolutionNetDsc (HighResolution-  enc_hrnet.py:464-510, :1125-1154
    Net.forward + 1-channel head)
  LSGAN terms / FullModel_D              criterion.py:90-103, utils.py:114-119, :256-276
  Adam step                              tools/train.py:251-261 (torch.optim.Adam)

Parity is pinned by tests/golden/ fixtures generated from the reference itself
(tests/golden/make_golden.py); see tests/test_oracle_golden.py.
"""
import torch
import torch.nn.functional as F


SYNC_GROUP = None  # set to a torch.distributed group for SyncBatchNorm semantics


def _bn(x, bn):
    if bn.training and bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
    if SYNC_GROUP is not None and bn.training:
        return _sync_bn(x, bn)
    return F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                        bn.training or not bn.track_running_stats, bn.momentum, bn.eps)


class _SyncStats(torch.autograd.Function):
    """all_reduce(sum) of per-rank statistics with an all_reduce(sum) backward
    (nn.SyncBatchNorm's gradient exchange, train.py:216-218)."""

    @staticmethod
    def forward(ctx, t):
        import torch.distributed as dist
        out = t.clone()
        dist.all_reduce(out, group=SYNC_GROUP)
        return out

    @staticmethod
    def backward(ctx, g):
        import torch.distributed as dist
        g = g.clone()
        dist.all_reduce(g, group=SYNC_GROUP)
        return g


def _sync_bn(x, bn):
    """Training BatchNorm with statistics over all ranks (nn.SyncBatchNorm)."""
    n_local = torch.tensor([float(x.numel() // x.shape[1])], dtype=x.dtype)
    s = torch.cat([x.sum(dim=(0, 2, 3)), (x * x).sum(dim=(0, 2, 3)), n_local])
    s = _SyncStats.apply(s)
    c = x.shape[1]
    cnt = s[2 * c].detach()
    mean = s[:c] / cnt
    var = s[c:2 * c] / cnt - mean * mean
    with torch.no_grad():
        m = bn.momentum
        bn.running_mean.mul_(1 - m).add_(m * mean.detach())
        bn.running_var.mul_(1 - m).add_(m * var.detach() * cnt / (cnt - 1))
    shape = (1, c, 1, 1)
    xh = (x - mean.view(shape)) / torch.sqrt(var.view(shape) + bn.eps)
    return xh * bn.weight.view(shape) + bn.bias.view(shape)


def _conv(x, c):
    return F.conv2d(x, c.weight, c.bias, c.stride, c.padding)


def _seq(seq, x):
    """Sequential of Conv2d / BatchNorm2d / ReLU containers."""
    for m in seq:
        name = type(m).__name__
        if name == "Conv2d":
            x = _conv(x, m)
        elif name == "BatchNorm2d":
            x = _bn(x, m)
        elif name == "ReLU":
            x = F.relu(x)
        elif name == "AdaptiveAvgPool2d":
            x = F.adaptive_avg_pool2d(x, 1)
        else:
            raise TypeError(name)
    return x


def _block(b, x):
    name = type(b).__name__
    res = x if b.downsample is None else _seq(b.downsample, x)
    if name == "BasicBlock":
        out = F.relu(_bn(_conv(x, b.conv1), b.bn1))
        out = _bn(_conv(out, b.conv2), b.bn2)
    elif name == "Bottleneck":
        out = F.relu(_bn(_conv(x, b.conv1), b.bn1))
        out = F.relu(_bn(_conv(out, b.conv2), b.bn2))
        out = _bn(_conv(out, b.conv3), b.bn3)
    else:
        raise TypeError(name)
    return F.relu(out + res)


def _blocks(seq, x):
    for b in seq:
        x = _block(b, x)
    return x


def _up(x, hw):
    return F.interpolate(x, size=list(hw), mode="bilinear", align_corners=False)


def _hr_module(m, xs):
    xs = [_blocks(m.branches[i], xs[i]) for i in range(m.num_branches)]
    if m.num_branches == 1:
        return xs
    out = []
    for i, row in enumerate(m.fuse_layers):
        y = xs[0] if i == 0 else _seq_chain(row[0], xs[0])
        for j in range(1, m.num_branches):
            if j == i:
                y = y + xs[j]
            elif j > i:
                y = y + _up(_seq(row[j], xs[j]), xs[i].shape[-2:])
            else:
                y = y + _seq_chain(row[j], xs[j])
        out.append(F.relu(y))
    return out


def _seq_chain(chain, x):
    for unit in chain:
        x = _seq(unit, x)
    return x


def _transition(trans, ys, nb):
    xs = []
    for i in range(nb):
        t = trans[i]
        if t is None:
            xs.append(ys[i])
        elif i < len(ys):
            xs.append(_seq(t, ys[i]))
        else:
            xs.append(_seq_chain(t, ys[-1]))
    return xs


def _trunk(net, prefix, x):
    g = lambda n: getattr(net, prefix + n)  # noqa: E731
    x = F.relu(_bn(_conv(x, g("conv1")), g("bn1")))
    x = F.relu(_bn(_conv(x, g("conv2")), g("bn2")))
    x = _blocks(g("layer1"), x)
    ys = [x]
    for s in (2, 3):
        xs = _transition(g(f"transition{s - 1}"), ys, getattr(net, f"stage{s}_cfg")["NUM_BRANCHES"])
        for m in g(f"stage{s}"):
            xs = _hr_module(m, xs)
        ys = xs
    return _transition(g("transition3"), ys, net.stage4_cfg["NUM_BRANCHES"])


def _stage4(net, prefix, xs):
    for m in getattr(net, prefix + "stage4"):
        xs = _hr_module(m, xs)
    return xs


def _upcat(ys):
    hw = ys[0].shape[-2:]
    return torch.cat([ys[0]] + [_up(y, hw) for y in ys[1:]], 1)


def _codes(net, prefix, xs, codes):
    trans = getattr(net, prefix + "transition3_e")
    out = []
    for b, x in enumerate(xs):
        maps = []
        for c in codes:
            if isinstance(c, (list, tuple)):
                maps.append(c[b])
            else:
                maps.append(c.repeat(1, 1, x.shape[2], x.shape[3]))
        xe = torch.cat(maps + [x], 1)
        out.append(xe if trans[b] is None else _seq(trans[b], xe))
    return out


def _heads(net, prefix, ys):
    x = _upcat(ys)
    return torch.cat([_seq(getattr(net, f"{prefix}last_layer_{k}"), x) for k in (1, 2, 3)], 1)


def run_encoder(ed, x, z, code):
    xs = _trunk(ed, "", x)
    if ed.enable_random_code:
        xs = _codes(ed, "", xs, [code, z] if not ed.is_baseline else [z])
    return _heads(ed, "", _stage4(ed, "", xs))


def run_decoder(ed, prefix, x, z):
    xs = _trunk(ed, prefix, x)
    if ed.enable_random_code:
        xs = _codes(ed, prefix, xs, [z])
    return _heads(ed, prefix, _stage4(ed, prefix, xs))


def run_ed(ed, x, z, code, is_baseline=False):
    x2t = run_encoder(ed, x, z, code)
    if is_baseline:
        with torch.no_grad():
            x3t = run_decoder(ed, "decf_", x2t, z)
            x1t = run_decoder(ed, "decp_", x2t, z)
    else:
        x3t = run_decoder(ed, "decf_", x2t, z)
        x1t = run_decoder(ed, "decp_", x2t, z)
    return x1t, x2t, x3t


def run_encz(ez, x):
    ys = _stage4(ez, "", _trunk(ez, "", x))
    if ez.hd_z:
        return [_seq(ez.last_layer[i], y) for i, y in enumerate(ys)]
    return _seq(ez.last_layer, _upcat(ys))


def run_dsc(d, x):
    """Discriminator: trunk + stage 4 + upsample/cat + last_layer -> (N, 1, H, W)."""
    ys = _stage4(d, "", _trunk(d, "", x))
    return _seq(d.last_layer, _upcat(ys))


def lsgan(sample, real):
    """MSELoss(sum) against ones (real) / zeros (fake), / batch (criterion.py:90-103)."""
    target = torch.ones_like(sample) if real else torch.zeros_like(sample)
    return torch.sum((sample - target) ** 2) / sample.shape[0]


def _frames(x, clip_length):
    """The frame slices the reference feeds D_frame: x.shape[1] // clip_length of
    them, 3 channels each (utils.py:116-118)."""
    return [x[:, 3 * f:3 * f + 3] for f in range(x.shape[1] // clip_length)]


def gan_terms(ds, df, x2p):
    """Generator LSGAN terms on x2t_hat (utils.py:114-119)."""
    seq = 0.5 * lsgan(run_dsc(ds, x2p), True)
    frame = torch.sum(torch.stack([0.5 * lsgan(run_dsc(df, f), True)
                                   for f in _frames(x2p, ds.clip_length)]))
    return seq, frame


def d_losses(ds, df, x2t, x2p, gan_lambda=1.0):
    """FullModel_D.forward (utils.py:256-276): [D_all (1,), D_seq, D_frame]."""
    x2t, x2p = x2t.detach(), x2p.detach()
    seq = 0.5 * lsgan(run_dsc(ds, x2t), True) + 0.5 * lsgan(run_dsc(ds, x2p), False)
    real = [0.5 * lsgan(run_dsc(df, f), True) for f in _frames(x2t, ds.clip_length)]
    fake = [0.5 * lsgan(run_dsc(df, f), False) for f in _frames(x2p, ds.clip_length)]
    frame = torch.sum(torch.stack(real)) + torch.sum(torch.stack(fake))
    return [torch.unsqueeze(gan_lambda * (seq + frame), 0), seq, frame]


def l1(p, t):
    return torch.sum(torch.abs(p - t)) / p.shape[0]


def kl(mu, logvar):
    if isinstance(mu, list):
        loss = 0.0
        for m, v in zip(mu, logvar):
            loss = loss + torch.sum(0.5 * (m ** 2 + torch.exp(v) - v - 1)) / m.shape[0]
        return loss
    return torch.sum(0.5 * (mu ** 2 + torch.exp(logvar) - logvar - 1)) / mu.shape[0]


def elbo(ez, ed, xt, x2t, x3t, eps, code, lambdas=(1.0, 0.1, 1.0), multiplier=1.0,
         is_baseline=False, baseline_mode="VAE_NATIVE", prior=False, ds=None, df=None,
         gan_lambda=0.0):
    """Reference ELBO step with explicit noise. Returns (terms dict, preds tuple, aux dict).
    With discriminators (ds, df) the LSGAN terms are formed as the reference does
    (always in non-baseline mode, in baseline only for VAE_GAN) and weighted by gan_lambda."""
    l1w, l2w, l3w = lambdas
    kl_w = l3w * multiplier if baseline_mode == "VAE_ANNEAL" else l3w
    aux = {}
    z = None
    mus = logvars = None
    if baseline_mode != "DETERMINISTIC":
        mv = run_encz(ez, torch.cat([xt, x2t, x3t] if is_baseline else [xt, x3t], 1))
        zc = ez.z_dim
        if isinstance(mv, list):
            mus = [m[:, :zc] for m in mv]
            logvars = [m[:, zc:] for m in mv]
            z = list(eps) if prior else [m + torch.exp(v * 0.5) * e
                                         for m, v, e in zip(mus, logvars, eps)]
        else:
            mus, logvars = mv[:, :zc], mv[:, zc:]
            z = eps if prior else mus + torch.exp(torch.mul(logvars, 0.5)) * eps
        aux["muvar"] = mv
        aux["z"] = z
    enc_in = torch.cat([xt, x2t], 1) if is_baseline else xt
    x1p, x2p, x3p = run_ed(ed, enc_in, z, code, is_baseline)
    if not is_baseline:
        t = {"xt_recon": l1(x1p, xt), "x2t_recon": l1(x2p, x2t), "x3t_recon": l1(x3p, x3t),
             "z_KL": kl(mus, logvars)}
        total = l1w * t["xt_recon"] + l2w * t["x2t_recon"] + l3w * t["x3t_recon"] + kl_w * t["z_KL"]
        if ds is not None:
            t["gan_seq"], t["gan_frame"] = gan_terms(ds, df, x2p)
            total = total + gan_lambda * (t["gan_seq"] + t["gan_frame"])
    else:
        t = {"x2t_recon": l1(x2p, x3t)}
        total = l2w * t["x2t_recon"]
        if baseline_mode != "DETERMINISTIC":
            t["z_KL"] = kl(mus, logvars)
            total = total + kl_w * t["z_KL"]
        if baseline_mode == "VAE_GAN" and ds is not None:
            t["gan_seq"], t["gan_frame"] = gan_terms(ds, df, x2p)
            total = total + gan_lambda * (t["gan_seq"] + t["gan_frame"])
    t["loss_all"] = total
    return t, (x1p, x2p, x3p), aux

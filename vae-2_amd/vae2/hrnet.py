"""HRNet-W18-small-v2 stacks of VAE² with a HIP execution path.

The nn.Module trees built here have the reference's exact shape: every
parameter / buffer has the same state_dict key and shape, and the Conv2d
containers are created (default-initialised) and then re-initialised
(N(0, 0.001^2)) in the same order, so `torch.manual_seed(s)` followed by the
factories yields bit-identical weights to the reference
(enc_hrnet.py:259-370 HighResolutionNet.__init__, :530-751 HighResolutionNetED,
:984-1041 HighResolutionNetEDz, :1125-1154 HighResolutionNetDsc,
:753-785/:1043-1068 init_weights, :1185-1210 factories).

nn.Conv2d / nn.BatchNorm2d are used only as parameter containers; forward
passes never call them.  Execution goes through vae2.ops (libvae2_hip kernels)
on NHWC activations:
  trunk      stem (:788-793) -> layer1 -> transitions / stages (:796-831)
  encoder    trunk + code maps (:818-830) + heads (:833-847)   -> x2t_hat
  decoders   trunk + z code map + heads (:849-963)             -> x3t_hat, xt_hat
  z-net      trunk + upsample/cat/avgpool/1x1 head (:1070-1122) -> mu|logvar
"""
import contextlib
import logging
import os

import torch
import torch.nn as nn

from . import heads as vheads
from . import dist as vdist
from . import ops, streams

BN_MOMENTUM = 0.01
vdist.guard_ddp()  # DDP around these networks would silently skip the gradient all-reduce
logger = logging.getLogger(__name__)


def _bn(c):
    return nn.BatchNorm2d(c, momentum=BN_MOMENTUM)


def _conv(cin, cout, k, stride=1, bias=False):
    return nn.Conv2d(cin, cout, kernel_size=k, stride=stride, padding=k // 2 if k == 3 else 0,
                     bias=bias)


# ------------------------------------------------------------------ blocks ----
class BasicBlock(nn.Module):
    """conv3x3-BN-ReLU-conv3x3-BN (+shortcut) -ReLU  (enc_hrnet.py:33-62)."""

    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv(inplanes, planes, 3, stride)
        self.bn1 = _bn(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv(planes, planes, 3)
        self.bn2 = _bn(planes)
        self.downsample = downsample
        self.stride = stride

    def run(self, x):
        # x feeds conv1 and the shortcut: its two gradient contributions are summed in
        # the producing kernels (ops.GradLink), not by an autograd add
        link = ops.GradLink(2)
        out = ops.conv_bn(x, self.conv1, self.bn1, relu=True, x_link=link)
        if self.downsample is None:
            return ops.conv_bn(out, self.conv2, self.bn2, relu=True, residual=x, res_link=link)
        sc = _run_convbn_seq(self.downsample, x, link)
        return ops.conv_bn(out, self.conv2, self.bn2, relu=True, residual=sc)


class Bottleneck(nn.Module):
    """1x1-3x3-1x1 bottleneck with x4 expansion (enc_hrnet.py:65-103)."""

    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv(inplanes, planes, 1)
        self.bn1 = _bn(planes)
        self.conv2 = _conv(planes, planes, 3, stride)
        self.bn2 = _bn(planes)
        self.conv3 = _conv(planes, planes * self.expansion, 1)
        self.bn3 = _bn(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def run(self, x):
        link = ops.GradLink(2)  # x feeds conv1 and the shortcut (see BasicBlock.run)
        # bn1's normalised output feeds only conv2 (3x3): normalised in conv2's staging
        # where the direct 3x3 kernels run (ops.LazyBN, as in run_blocks_lockstep); bn2's
        # feeds only conv3 (1x1): its backward partials come from conv3's data gradient
        pb = ops.PartBN() if ops.PART_BN else None
        out = _lazy_pair(x, self.conv1, self.bn1, self.conv2, self.bn2, x_link=link, part=pb)
        if self.downsample is None:
            return ops.conv_bn(out, self.conv3, self.bn3, relu=True, residual=x, res_link=link,
                               bn_part=pb)
        if len(self.downsample) == 2:  # conv + BN: its output is only bn3's residual (ops.ResBN)
            return ops.conv_bn_multi([out, x], [self.conv3, self.downsample[0]],
                                     [self.bn3, self.downsample[1]], [True, False],
                                     x_links=[None, link], res_bns=[1, None],
                                     bn_ins=[pb, None])[0]
        sc = _run_convbn_seq(self.downsample, x, link)
        return ops.conv_bn(out, self.conv3, self.bn3, relu=True, residual=sc, bn_part=pb)


BLOCKS = {"BASIC": BasicBlock, "BOTTLENECK": Bottleneck}


def _lazy_pair(x, conv_a, bn_a, conv_b, bn_b, x_link=None, part=None):
    """relu(bn_b(conv_b(relu(bn_a(conv_a(x)))))) where bn_a's output feeds only conv_b: with
    the direct 3x3 kernels for conv_b it is never stored (ops.LazyBN) -- the Bottleneck's
    bn1 -> conv2 (enc_hrnet.py:84-90) and the stem's bn1 -> conv2 (:788-793); otherwise its
    backward partials come from conv_b's data gradient (ops.PartBN).  part: bn_b's PartBN
    (its output's only consumer takes it as bn_part), or None."""
    n, h, w, _ = x.shape
    spec = ops.ConvSpec(conv_a)
    oh, ow = spec.out_hw(h, w)
    lz = ops.LazyBN() if ops.lazy_bn_ok((n, oh, ow, conv_a.out_channels), conv_b) else None
    if lz is None and ops.PART_BN:
        lz = ops.PartBN()
    lazy = [lz]
    out = ops.conv_bn_multi([x], [conv_a], [bn_a], True, x_links=[x_link], bn_outs=lazy)
    return ops.conv_bn_multi(out, [conv_b], [bn_b], True, bn_ins=lazy,
                             bn_outs=[part] if part is not None else None)[0]


def _run_convbn_seq(seq, x, x_link=None):
    """Sequential(Conv2d, BatchNorm2d[, ReLU])."""
    return ops.conv_bn(x, seq[0], seq[1], relu=len(seq) > 2, x_link=x_link)


def _run_convbn_seqs(seqs, xs, x_links=None, bn_outs=None, bn_ins=None):
    """Independent Sequential(Conv2d, BatchNorm2d[, ReLU]) units of one depth level,
    their BatchNorm steps in shared launches (ops.conv_bn_multi).  bn_outs: per unit a
    LazyBN whose output is handed over un-normalised (set to None where it is stored), or a
    PartBN (output stored, partials from the consumer); bn_ins: the producers' markers."""
    if not seqs:
        return []
    return ops.conv_bn_multi(xs, [q[0] for q in seqs], [q[1] for q in seqs],
                             [len(q) > 2 for q in seqs], x_links=x_links, bn_outs=bn_outs,
                             bn_ins=bn_ins)


def run_blocks_lockstep(blocks, xs):
    """One residual block per branch (same depth in a HighResolutionModule), in lockstep:
    conv1 of every branch, then conv2 + residual of every branch, BatchNorm batched."""
    if not all(isinstance(b, BasicBlock) and b.downsample is None for b in blocks):
        return [b.run(x) for b, x in zip(blocks, xs)]
    links = [ops.GradLink(2) for _ in blocks]  # x feeds conv1 and the shortcut
    # bn1's normalised output feeds only conv2: conv2 normalises it while staging its input
    # (ops.LazyBN) where the direct 3x3 kernels run, so it is never stored
    res_ok = all(ops._bn_quad_ok(x) for x in xs)
    # (elsewhere -- the 144-channel branch, whose conv2 is a gather-kernel conv -- bn1's
    # output is stored and conv2's data gradient writes its partials: ops.PartBN)
    lazy = [ops.LazyBN() if res_ok and ops.lazy_bn_ok(tuple(x.shape[:3]) + (b.conv1.out_channels,),
                                                      b.conv2) else
            (ops.PartBN() if ops.PART_BN else None)
            for b, x in zip(blocks, xs)]
    outs = ops.conv_bn_multi(xs, [b.conv1 for b in blocks], [b.bn1 for b in blocks], True,
                             x_links=links, bn_outs=lazy)
    return ops.conv_bn_multi(outs, [b.conv2 for b in blocks], [b.bn2 for b in blocks], True,
                             residuals=xs, res_links=links, bn_ins=lazy)


def _shortcut(cin, cout, stride):
    if stride == 1 and cin == cout:
        return None
    return nn.Sequential(nn.Conv2d(cin, cout, kernel_size=1, stride=stride, bias=False), _bn(cout))


def make_layer(block, inplanes, planes, nblocks, stride=1):
    """Sequential of `nblocks` blocks; the first adapts channels (enc_hrnet.py:408-423)."""
    ds = _shortcut(inplanes, planes * block.expansion, stride)
    seq = [block(inplanes, planes, stride, ds)]
    seq += [block(planes * block.expansion, planes) for _ in range(1, nblocks)]
    return nn.Sequential(*seq)


def run_seq(seq, x):
    for blk in seq:
        x = blk.run(x)
    return x


def _down_chain(cin, cout, steps):
    """`steps` stride-2 3x3 conv+BN(+ReLU) units; the last one maps cin->cout w/o ReLU
    when used in a fuse layer (relu_last=False) (enc_hrnet.py:199-218)."""
    units = []
    for k in range(steps):
        last = k == steps - 1
        co = cout if last else cin
        mods = [nn.Conv2d(cin, co, 3, 2, 1, bias=False), _bn(co)]
        if not last:
            mods.append(nn.ReLU(inplace=True))
        units.append(nn.Sequential(*mods))
    return nn.Sequential(*units)


class HighResolutionModule(nn.Module):
    """Parallel branches + multi-resolution fuse (enc_hrnet.py:106-250)."""

    def __init__(self, num_branches, block, num_blocks, num_inchannels, num_channels,
                 fuse_method, multi_scale_output=True):
        super().__init__()
        for name, seq in (("NUM_BLOCKS", num_blocks), ("NUM_CHANNELS", num_channels),
                          ("NUM_INCHANNELS", num_inchannels)):
            if len(seq) != num_branches:
                msg = f"NUM_BRANCHES({num_branches}) <> {name}({len(seq)})"
                logger.error(msg)
                raise ValueError(msg)
        self.num_inchannels = num_inchannels  # mutated in place, as the reference does
        self.fuse_method = fuse_method
        self.num_branches = num_branches
        self.multi_scale_output = multi_scale_output
        branches = []
        for b in range(num_branches):
            width = num_channels[b] * block.expansion
            ds = _shortcut(self.num_inchannels[b], width, 1)
            seq = [block(self.num_inchannels[b], num_channels[b], 1, ds)]
            self.num_inchannels[b] = width
            seq += [block(width, num_channels[b]) for _ in range(1, num_blocks[b])]
            branches.append(nn.Sequential(*seq))
        self.branches = nn.ModuleList(branches)
        self.fuse_layers = self._build_fuse()
        self.relu = nn.ReLU(inplace=True)

    def _build_fuse(self):
        nb = self.num_branches
        if nb == 1:
            return None
        ch = self.num_inchannels
        rows = []
        for i in range(nb if self.multi_scale_output else 1):
            row = []
            for j in range(nb):
                if j > i:
                    row.append(nn.Sequential(nn.Conv2d(ch[j], ch[i], 1, 1, 0, bias=False),
                                             _bn(ch[i])))
                elif j == i:
                    row.append(None)
                else:
                    row.append(_down_chain(ch[j], ch[i], i - j))
            rows.append(nn.ModuleList(row))
        return nn.ModuleList(rows)

    def get_num_inchannels(self):
        return self.num_inchannels

    def run(self, xs):
        nb = self.num_branches
        depths = {len(self.branches[b]) for b in range(nb)}
        if len(depths) == 1:  # branches in lockstep (enc_hrnet.py:226-231)
            for d in range(depths.pop()):
                xs = run_blocks_lockstep([self.branches[b][d] for b in range(nb)], xs)
        else:
            xs = [run_seq(self.branches[b], xs[b]) for b in range(nb)]
        if nb == 1:
            return xs
        # fuse (enc_hrnet.py:233-249): every j > i 1x1 conv + BN in one batch (upsampled
        # in the fuse kernel), the j < i stride-2 chains batched by chain position.
        # Branch output j feeds one unit per fuse row (its identity term in row j, an
        # up or down path in the others): their gradients meet in one buffer
        # (ops.GradLink) instead of autograd add kernels.
        rows = list(enumerate(self.fuse_layers))
        links = [ops.GradLink(len(rows)) if len(rows) > 1 else None for _ in range(nb)]
        # the units feeding a fuse sum (every up path, the last unit of every down chain)
        # hand over their pre-BN output: the fuse kernel normalises it (ops.fuse_sum_relu
        # lazies), so their BN apply pass never runs and the output is never stored
        terms, lazy = {}, {}
        ups = [(i, j) for i, _ in rows for j in range(nb) if j > i]
        lz_up = [ops.LazyBN() if ops.FUSE_LAZY else None for _ in ups]
        for (i, j), t, lz in zip(ups, _run_convbn_seqs([self.fuse_layers[i][j] for i, j in ups],
                                                       [xs[j] for _, j in ups],
                                                       [links[j] for _, j in ups], lz_up),
                                 lz_up):
            terms[(i, j)], lazy[(i, j)] = t, lz
        downs = [(i, j) for i, _ in rows for j in range(nb) if j < i]
        cur = {(i, j): xs[j] for i, j in downs}
        parts = {}  # the inner units' PartBN markers, by chain, for the next unit's call
        for k in range(max((i - j for i, j in downs), default=0)):
            live = [(i, j) for i, j in downs if k < i - j]
            # the last unit's output is normalised by the fuse sum (LazyBN); an inner unit's
            # (conv + BN + ReLU, stored) feeds only the next stride-2 conv (PartBN)
            lz_dn = [ops.LazyBN() if ops.FUSE_LAZY and k == i - j - 1 else
                     (ops.PartBN() if ops.PART_BN and k < i - j - 1 else None)
                     for i, j in live]
            ins = [parts.get(ij) for ij in live]
            outs = _run_convbn_seqs([self.fuse_layers[i][j][k] for i, j in live],
                                    [cur[ij] for ij in live],
                                    [links[j] if k == 0 else None for _, j in live], lz_dn,
                                    bn_ins=ins if any(b is not None for b in ins) else None)
            parts = {ij: lz for ij, lz in zip(live, lz_dn) if isinstance(lz, ops.PartBN)}
            cur.update(zip(live, outs))
            lazy.update((ij, lz) for ij, lz in zip(live, lz_dn)
                        if not isinstance(lz, ops.PartBN) and (lz is not None or
                                                               k == ij[0] - ij[1] - 1))
        terms.update(cur)
        out = []
        for i, _ in rows:
            out.append(ops.fuse_sum_relu([xs[j] if j == i else terms[(i, j)] for j in range(nb)],
                                         xs[i].shape[1:3],
                                         [links[i] if j == i else None for j in range(nb)],
                                         [None if j == i else lazy.get((i, j)) for j in range(nb)]))
        return out


def make_transition(pre, cur):
    """ModuleList mapping branch lists between stages (enc_hrnet.py:372-406)."""
    mods = []
    for i, c in enumerate(cur):
        if i < len(pre):
            if c != pre[i]:
                mods.append(nn.Sequential(nn.Conv2d(pre[i], c, 3, 1, 1, bias=False), _bn(c),
                                          nn.ReLU(inplace=True)))
            else:
                mods.append(None)
        else:
            units = []
            extra = i + 1 - len(pre)
            for j in range(extra):
                co = c if j == extra - 1 else pre[-1]
                units.append(nn.Sequential(nn.Conv2d(pre[-1], co, 3, 2, 1, bias=False), _bn(co),
                                           nn.ReLU(inplace=True)))
            mods.append(nn.Sequential(*units))
    return nn.ModuleList(mods)


def make_stage(cfg, num_inchannels, multi_scale_output=True):
    """Sequential of HighResolutionModules (enc_hrnet.py:425-452)."""
    block = BLOCKS[cfg["BLOCK"]]
    mods = []
    n = cfg["NUM_MODULES"]
    for i in range(n):
        mso = multi_scale_output or i != n - 1
        mods.append(HighResolutionModule(cfg["NUM_BRANCHES"], block, cfg["NUM_BLOCKS"],
                                         num_inchannels, cfg["NUM_CHANNELS"], cfg["FUSE_METHOD"],
                                         mso))
        num_inchannels = mods[-1].get_num_inchannels()
    return nn.Sequential(*mods), num_inchannels


def run_transition(trans, ys, nbranches):
    """Branch inputs of the next stage from the previous stage's outputs; the first
    conv+BN unit of every transition in one batch."""
    xs = [ys[i] if trans[i] is None else None for i in range(nbranches)]
    todo = [i for i in range(nbranches) if trans[i] is not None]
    firsts = [trans[i] if i < len(ys) else trans[i][0] for i in todo]
    ins = [ys[i] if i < len(ys) else ys[-1] for i in todo]
    # an input feeding two of these convs (the last branch: its own transition and the new
    # branch's) gets one GradLink: the second data gradient accumulates in-kernel
    links = [None] * len(ins)
    for j in range(len(ins)):
        users = [k for k in range(len(ins)) if ins[k] is ins[j]]
        if len(users) > 1 and links[j] is None:
            lk = ops.GradLink(len(users))
            for k in users:
                links[k] = lk
    outs = _run_convbn_seqs(firsts, ins, x_links=links if any(links) else None)
    for i, x in zip(todo, outs):
        if i >= len(ys):
            for unit in list(trans[i])[1:]:
                x = _run_convbn_seq(unit, x)
        xs[i] = x
    return xs


def run_stage(stage, xs):
    for m in stage:
        xs = m.run(xs)
    return xs


def _head(nin, nclass, final_k):
    return nn.Sequential(
        nn.Conv2d(nin, nin, kernel_size=1, stride=1, padding=0),
        _bn(nin),
        nn.ReLU(inplace=True),
        nn.Conv2d(nin, nclass, kernel_size=final_k, stride=1, padding=1 if final_k == 3 else 0))


def run_head(head, x):
    h = ops.conv_bn(x, head[0], head[1], relu=True)
    return ops.conv(h, head[3])


def _ch_list(cfg):
    block = BLOCKS[cfg["BLOCK"]]
    return [c * block.expansion for c in cfg["NUM_CHANNELS"]]


# -------------------------------------------------------------------- nets ----
class HighResolutionNet(nn.Module):
    """Shared trunk: stem, layer1, stages 2-4, transitions, optional code-map
    transition and three heads (enc_hrnet.py:259-370)."""

    _vae2_hip_module = True  # gradients go to main_grad (vae2.dist.guard_ddp)

    def __init__(self, config, **kwargs):
        extra = config.MODEL.EXTRA
        self.is_baseline = extra.IS_BASELINE
        super().__init__()
        self.enable_random_code = kwargs["enable_random_code"]
        self.clip_length = config.TRAIN.CLIP_LENGTH
        self.hd_z = extra.HD_Z
        self.z_dim = extra.Z_DIM
        self.conv1 = nn.Conv2d(3, 64, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn1 = _bn(64)
        self.conv2 = nn.Conv2d(64, 64, kernel_size=3, stride=2, padding=1, bias=False)
        self.bn2 = _bn(64)
        self.relu = nn.ReLU(inplace=True)
        self.last_stage_channels = self._build_trunk("", extra, code_extra=(
            self.z_dim * 2 if not self.is_baseline else self.z_dim)
            if self.enable_random_code else None)
        self.last_inp_channels = int(sum(self.last_stage_channels))
        for k in (1, 2, 3):
            setattr(self, f"last_layer_{k}", _head(self.last_inp_channels,
                                                   config.DATASET.NUM_CLASSES,
                                                   extra.FINAL_CONV_KERNEL))
        vheads.mark_split([getattr(self, f"last_layer_{k}") for k in (1, 2, 3)],
                          self.last_stage_channels)

    def _build_trunk(self, prefix, extra, code_extra):
        """layer1 .. stage4 under `prefix` (enc_hrnet.py:279-319 / :555-594)."""
        s1 = extra["STAGE1"]
        self.stage1_cfg = s1
        block = BLOCKS[s1["BLOCK"]]
        setattr(self, prefix + "layer1", make_layer(block, 64, s1["NUM_CHANNELS"][0],
                                                     s1["NUM_BLOCKS"][0]))
        pre = [block.expansion * s1["NUM_CHANNELS"][0]]
        for s in (2, 3, 4):
            cfg = extra[f"STAGE{s}"]
            setattr(self, f"stage{s}_cfg", cfg)
            cur = _ch_list(cfg)
            setattr(self, f"{prefix}transition{s - 1}", make_transition(pre, cur))
            if s == 4 and code_extra is not None:
                setattr(self, f"{prefix}transition3_e",
                        make_transition([c + code_extra for c in cur], cur))
            stage, pre = make_stage(cfg, cur, multi_scale_output=True)
            setattr(self, f"{prefix}stage{s}", stage)
        return pre

    # ---- execution ----
    def _stem(self, prefix, x):
        g = lambda n: getattr(self, prefix + n)  # noqa: E731
        x = _lazy_pair(x, g("conv1"), g("bn1"), g("conv2"), g("bn2"))
        return run_seq(g("layer1"), x)

    def _trunk_to_stage4_inputs(self, prefix, x):
        g = lambda n: getattr(self, prefix + n)  # noqa: E731
        x = self._stem(prefix, x)
        ys = [x]
        for s in (2, 3):
            nb = getattr(self, f"stage{s}_cfg")["NUM_BRANCHES"]
            xs = run_transition(g(f"transition{s - 1}"), ys, nb)
            ys = run_stage(g(f"stage{s}"), xs)
        nb = self.stage4_cfg["NUM_BRANCHES"]
        return run_transition(g("transition3"), ys, nb)

    def _apply_codes(self, prefix, xs, codes):
        """cat((code maps..., x_b)) -> transition3_e (enc_hrnet.py:818-830, :880-888)."""
        trans = getattr(self, prefix + "transition3_e")
        xes = []
        for b, x in enumerate(xs):
            parts, tiles = [], []
            for c in codes:
                if isinstance(c, (list, tuple)):  # HD_Z: per-branch code maps
                    parts.append(c[b])
                    tiles.append(False)
                else:  # per-clip vector (N,1,1,z) tiled over the branch
                    parts.append(c)
                    tiles.append(True)
            parts.append(x)
            tiles.append(False)
            xes.append(ops.cat(parts, x.shape[1:3], tiles))
        todo = [b for b in range(len(xs)) if trans[b] is not None]
        outs = dict(zip(todo, _run_convbn_seqs([trans[b] for b in todo], [xes[b] for b in todo])))
        return [outs.get(b, xes[b]) for b in range(len(xs))]

    def _heads(self, prefix, ys):
        heads = [getattr(self, f"{prefix}last_layer_{k}") for k in (1, 2, 3)]
        if vheads.supported(heads, [int(y.shape[3]) for y in ys]):
            return vheads.run(heads, ys)  # per-branch 1x1 convs (vae2/heads.py)
        x = ops.up_cat(ys)
        outs = [run_head(getattr(self, f"{prefix}last_layer_{k}"), x) for k in (1, 2, 3)]
        return ops.cat(outs, x.shape[1:3])

    def init_weights(self, pretrained=""):
        logger.info("=> init weights from normal distribution")
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.normal_(m.weight, std=0.001)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if pretrained and os.path.isfile(pretrained):
            self._load_pretrained(pretrained)

    def _load_pretrained(self, path):
        state = torch.load(path, map_location="cpu", weights_only=True)
        own = self.state_dict()
        upd = {}
        for k, v in state.items():
            k2 = k.replace("model.", "")
            if k2 in own and "last_layer" not in k:
                upd[k2] = v
        upd.update(self._expand_pretrained(upd))
        for k in upd:
            logger.info("=> loading %s pretrained model %s", k, path)
        own.update(upd)
        self.load_state_dict(own)

    def _expand_pretrained(self, upd):
        return {}


class HighResolutionNetED(HighResolutionNet):
    """Encoder (xt [+z, random code] -> x2t_hat) and future / past decoders
    (x2t_hat + z -> x3t_hat / xt_hat) (enc_hrnet.py:530-981)."""

    def __init__(self, config, **kwargs):
        extra = config.MODEL.EXTRA
        super().__init__(config, **kwargs,
                         enable_random_code=extra.BASELINE_MODE != "DETERMINISTIC")
        self.extra = extra
        L = self.clip_length
        self.conv1 = nn.Conv2d(3 * L * 2 if extra.IS_BASELINE else 3 * L, 64, kernel_size=3,
                               stride=1, padding=1, bias=False)
        self.conv2 = nn.Conv2d(64, 64, kernel_size=3, stride=1, padding=1, bias=False)
        for d in ("decf_", "decp_"):
            setattr(self, d + "conv1", nn.Conv2d(3 * L, 64, kernel_size=3, stride=1, padding=1,
                                                 bias=False))
            setattr(self, d + "bn1", _bn(64))
            setattr(self, d + "conv2", nn.Conv2d(64, 64, kernel_size=3, stride=1, padding=1,
                                                 bias=False))
            setattr(self, d + "bn2", _bn(64))
            setattr(self, d + "relu", nn.ReLU(inplace=True))
            pre = self._build_trunk(d, extra, self.z_dim if self.enable_random_code else None)
            nin = int(sum(pre))
            for k in (1, 2, 3):
                setattr(self, f"{d}last_layer_{k}", _head(nin, config.DATASET.NUM_CLASSES,
                                                          extra.FINAL_CONV_KERNEL))
            vheads.mark_split([getattr(self, f"{d}last_layer_{k}") for k in (1, 2, 3)], pre)

    def _expand_pretrained(self, upd):
        L = self.clip_length
        out = {}
        for k, v in upd.items():
            if k == "conv1.weight":
                out[k] = v.repeat([1, L * 2 if self.extra.IS_BASELINE else L, 1, 1])
                out["decf_" + k] = v.repeat([1, L, 1, 1])
                out["decp_" + k] = v.repeat([1, L, 1, 1])
            else:
                out["decf_" + k] = v
                out["decp_" + k] = v
        return out

    def encode_trunk(self, x):
        """Encoder stem .. stage 3 + transition3 (independent of z)."""
        return self._trunk_to_stage4_inputs("", x)

    def encode(self, x, z, code, trunk=None):
        """x: (N,H,W,3L) NHWC -> x2t_hat (N,H,W,3*NUM_CLASSES)."""
        xs = trunk if trunk is not None else self._trunk_to_stage4_inputs("", x)
        if self.enable_random_code:
            codes = [code, z] if not self.is_baseline else [z]
            xs = self._apply_codes("", xs, codes)
        ys = run_stage(self.stage4, xs)
        return self._heads("", ys)

    def decode(self, prefix, x, z):
        xs = self._trunk_to_stage4_inputs(prefix, x)
        if self.enable_random_code:
            xs = self._apply_codes(prefix, xs, [z])
        ys = run_stage(getattr(self, prefix + "stage4"), xs)
        return self._heads(prefix, ys)

    def run(self, x, z=None, code=None, is_baseline=False, trunk=None):
        """Encoder then both decoders; the past decoder runs on a side stream
        concurrently with the future decoder (they are independent)."""
        x2t = self.encode(x, z, code, trunk)
        flat = getattr(self, "_vae2_flat", None)
        if flat is not None and not is_baseline:  # the decoders' gradient buckets start early
            if not hasattr(self, "_dec_start"):
                self._dec_start = vdist.tail_range(flat)
            vdist.early_reduce_hook(x2t, flat, self._dec_start)
        with torch.no_grad() if is_baseline else contextlib.nullcontext():
            with streams.on_side(1, inputs=[x2t, z]) as sp:
                x1t = self.decode("decp_", x2t, z)
            x3t = self.decode("decf_", x2t, z)
            streams.join(sp, [x1t])
        return x1t, x2t, x3t

    def forward(self, x, z=None, is_baseline=False, code=None):
        """Reference-compatible call on NCHW tensors (enc_hrnet.py:965-981).

        z: (N, z, 1, 1) tensor or, with HD_Z, a list of (N, z, h_b, w_b) maps.
        code: the encoder's random code (N, z, 1, 1); drawn from the CPU
        generator like the reference when omitted.
        """
        xn = ops.to_nhwc(x)
        zn = _z_to_nhwc(z)
        if self.enable_random_code and code is None:
            code = torch.randn(x.shape[0], self.z_dim, 1, 1).to(x.device)
        cn = ops.to_nhwc(code) if code is not None else None
        outs = self.run(xn, zn, cn, is_baseline)
        return tuple(ops.to_nchw(o) for o in outs)


def _z_to_nhwc(z):
    if z is None:
        return None
    if isinstance(z, (list, tuple)):
        return [ops.to_nhwc(t) for t in z]
    return ops.to_nhwc(z)


class HighResolutionNetEDz(HighResolutionNet):
    """Posterior net q(z | xt, x3t) -> (mu | logvar) (enc_hrnet.py:984-1122)."""

    def __init__(self, config, **kwargs):
        extra = config.MODEL.EXTRA
        super().__init__(config, **kwargs, enable_random_code=False)
        self.extra = extra
        L = self.clip_length
        self.conv1 = nn.Conv2d(3 * L * 3 if extra.IS_BASELINE else 3 * L * 2, 64, kernel_size=3,
                               stride=1, padding=1, bias=False)
        self.conv2 = nn.Conv2d(64, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.last_layer = self._make_z_layer()
        self.last_layer_1 = None
        self.last_layer_2 = None
        self.last_layer_3 = None

    def _make_z_layer(self):
        if self.hd_z:
            mods = []
            for c in self.last_stage_channels:
                if c != self.z_dim * 2:
                    mods.append(nn.Sequential(nn.Conv2d(c, self.z_dim * 2, kernel_size=1, stride=1,
                                                        padding=0, bias=False)))
                else:
                    mods.append(None)
            return nn.ModuleList(mods)
        return nn.Sequential(
            nn.AdaptiveAvgPool2d((1, 1)),
            nn.Conv2d(sum(self.last_stage_channels), 512, kernel_size=1, stride=1, padding=0),
            _bn(512),
            nn.ReLU(inplace=True),
            nn.Conv2d(512, 2 * self.z_dim, kernel_size=1, stride=1, padding=0))

    def _expand_pretrained(self, upd):
        L = self.clip_length
        if "conv1.weight" in upd:
            return {"conv1.weight": upd["conv1.weight"].repeat(
                [1, L * 3 if self.extra.IS_BASELINE else L * 2, 1, 1])}
        return {}

    def run(self, x):
        """x: (N,H,W,6L) NHWC -> (N,1,1,2z) or, with HD_Z, a list of (N,h_b,w_b,2z)."""
        # its gradient buckets start as soon as its backward is done (vae2.dist)
        x = vdist.anchor_reduce(x, getattr(self, "_vae2_flat", None))
        xs = self._trunk_to_stage4_inputs("", x)
        ys = run_stage(self.stage4, xs)
        if self.hd_z:
            out = []
            for b, y in enumerate(ys):
                m = self.last_layer[b]
                if m is None:
                    raise ValueError("HD_Z branch with 2*Z_DIM channels has no projection "
                                     "(the reference fails here too)")
                out.append(ops.conv(y, m[0]))
            return out
        h = ops.up_avgpool(ys)  # avgpool(cat(y0, up(y1), ...)): enc_hrnet.py:1022-1025
        h = ops.conv_bn(h, self.last_layer[1], self.last_layer[2], relu=True)
        return ops.conv(h, self.last_layer[4])

    def forward(self, x, *args, **kwargs):
        out = self.run(ops.to_nhwc(x))
        if isinstance(out, list):
            return [ops.to_nchw(o) for o in out]
        return ops.to_nchw(out)


class HighResolutionNetDsc(HighResolutionNet):
    """GAN discriminator (enc_hrnet.py:1125-1154): the shared trunk with stride-1 stems
    and one 1-channel head on the upsampled 270-channel concatenation, i.e.
    HighResolutionNet.forward (:464-510).  Sequence D sees the 3L-channel x2t clip,
    frame D one RGB frame; the output is a per-pixel score map (N, H, W, 1)."""

    def __init__(self, config, is_sequence, **kwargs):
        extra = config.MODEL.EXTRA
        super().__init__(config, **kwargs, enable_random_code=False)
        self.is_sequence = is_sequence
        L = self.clip_length
        self.conv1 = nn.Conv2d(3 * L if is_sequence else 3, 64, kernel_size=3, stride=1,
                               padding=1, bias=False)
        self.conv2 = nn.Conv2d(64, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.last_layer = nn.Sequential(
            nn.Conv2d(self.last_inp_channels, self.last_inp_channels, kernel_size=1, stride=1,
                      padding=0),
            _bn(self.last_inp_channels),
            nn.ReLU(inplace=True),
            nn.Conv2d(self.last_inp_channels, 1, kernel_size=extra.FINAL_CONV_KERNEL, stride=1,
                      padding=1 if extra.FINAL_CONV_KERNEL == 3 else 0))
        self.last_layer_1 = None
        self.last_layer_2 = None
        self.last_layer_3 = None
        vheads.mark_split([self.last_layer], self.last_stage_channels)

    def _expand_pretrained(self, upd):
        if self.is_sequence and "conv1.weight" in upd:
            return {"conv1.weight": upd["conv1.weight"].repeat([1, self.clip_length, 1, 1])}
        return {}

    def run(self, x):
        """x: (N,H,W,3L) or (N,H,W,3) NHWC -> D score map (N,H,W,1)."""
        xs = self._trunk_to_stage4_inputs("", x)
        ys = run_stage(self.stage4, xs)
        if vheads.supported([self.last_layer], [int(y.shape[3]) for y in ys]):
            return vheads.run([self.last_layer], ys)
        return run_head(self.last_layer, ops.up_cat(ys))

    def forward(self, x, *args, **kwargs):
        """Reference-compatible call on an NCHW tensor -> (N, 1, H, W)."""
        return ops.to_nchw(self.run(ops.to_nhwc(x)))


def get_encdec_model(cfg, **kwargs):
    model = HighResolutionNetED(cfg, **kwargs)
    model.init_weights(cfg.MODEL.PRETRAINED)
    return model


def get_D_sequence_model(cfg, **kwargs):
    model = HighResolutionNetDsc(config=cfg, is_sequence=True, **kwargs)
    model.init_weights(cfg.MODEL.PRETRAINED)
    return model


def get_D_frame_model(cfg, **kwargs):
    model = HighResolutionNetDsc(config=cfg, is_sequence=False, **kwargs)
    model.init_weights(cfg.MODEL.PRETRAINED)
    return model


def get_encz_model(cfg, **kwargs):
    model = HighResolutionNetEDz(cfg, **kwargs)
    model.init_weights(cfg.MODEL.PRETRAINED)
    return model

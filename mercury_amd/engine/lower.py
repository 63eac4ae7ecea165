"""Lower a reference-architecture ``nn.Module`` to the native engine's unit graph.

The engine does not trace anything: it walks the known module trees of the
model zoo (``models/resnet.py`` = `pytorch_model.py:14-113`, ``models/vgg.py`` =
`pytorch_model.py:117-153`, and ``models/mobilenetv2.py``) and emits

* ``Unit``  -- one conv (implicit-GEMM or depthwise) + its BatchNorm + activation;
* ``Block`` -- main-path units, an optional shortcut unit or identity skip, the
  final activation and an optional max-pool (ImageNet stem);
* the classifier head (global average pool + linear, or -- speech VGG -- flatten +
  two linears).

Parameters are laid out in ONE flat fp32 buffer in module registration order
(so the flat order matches ``named_parameters()``, and backward produces
gradients from the end of the buffer towards the start); conv weights are
stored [K][R][S][C] in the flat buffer -- the layout the weight-gradient kernel
writes coalesced -- and converted to/from torch's [K][C][R][S] at the
state-dict boundary.  Every segment starts on a 4-element boundary so the
optimizer's float4 sweep never straddles two parameters.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import torch.nn as nn

from ..models.mobilenetv2 import InvertedResidual, MobileNetV2
from ..models.resnet import BasicBlock, Bottleneck, ResNet
from ..models.vgg import VGG


@dataclass
class Seg:
    name: str
    param: nn.Parameter
    off: int
    numel: int
    kind: str            # 'conv' (KRSC master), 'dw' ([C][9]), 'vec', 'fc'


@dataclass
class Unit:
    name: str
    conv: nn.Conv2d
    bn: nn.BatchNorm2d
    act: str                     # 'relu' | 'relu6' | 'none' (only for non-final units)
    depthwise: bool = False
    w_seg: Optional[Seg] = None
    b_seg: Optional[Seg] = None  # conv bias (VGG) if any
    g_seg: Optional[Seg] = None
    beta_seg: Optional[Seg] = None
    need_dgrad: bool = True

    @property
    def K(self):
        return self.conv.out_channels

    @property
    def C(self):
        return self.conv.in_channels

    @property
    def R(self):
        return self.conv.kernel_size[0]

    @property
    def stride(self):
        return self.conv.stride[0]

    @property
    def pad(self):
        return self.conv.padding[0]


@dataclass
class Block:
    name: str
    units: List[Unit]
    shortcut: Optional[Unit] = None
    identity: bool = False
    final_act: str = 'relu'
    pool: Optional[tuple] = None     # (k, stride, pad) max-pool after the block (ImageNet stem)
    need_dx: bool = True


@dataclass
class Lowered:
    blocks: List[Block]
    fc: nn.Linear
    segs: List[Seg] = field(default_factory=list)
    total: int = 0
    in_channels: int = 3
    num_classes: int = 10
    head_pool: str = 'avg'           # 'avg': global avg-pool + fc;  'mlp2': flatten + fc1 + fc2
    fc1: Optional[nn.Linear] = None  # first layer of the 'mlp2' head (VGG)


def supports(net):
    return isinstance(net, (ResNet, MobileNetV2, VGG))


def _bn_unit(name, conv, bn, act, depthwise=False):
    return Unit(name, conv, bn, act, depthwise)


def lower(net) -> Lowered:
    blocks = []
    if isinstance(net, ResNet):
        stem = Block('stem', [_bn_unit('conv1', net.conv1, net.bn1, 'relu')], final_act='relu',
                     need_dx=False)
        stem.units[0].need_dgrad = False
        if net.stem == 'imagenet':
            stem.pool = (3, 2, 1)
        blocks.append(stem)
        for li in range(1, 5):
            layer = getattr(net, 'layer%d' % li)
            for bi, b in enumerate(layer):
                pre = 'layer%d.%d' % (li, bi)
                if isinstance(b, BasicBlock):
                    units = [_bn_unit(pre + '.conv1', b.conv1, b.bn1, 'relu'),
                             _bn_unit(pre + '.conv2', b.conv2, b.bn2, 'none')]
                elif isinstance(b, Bottleneck):
                    units = [_bn_unit(pre + '.conv1', b.conv1, b.bn1, 'relu'),
                             _bn_unit(pre + '.conv2', b.conv2, b.bn2, 'relu'),
                             _bn_unit(pre + '.conv3', b.conv3, b.bn3, 'none')]
                else:
                    raise TypeError(type(b))
                sc = None
                if len(b.shortcut) > 0:
                    sc = _bn_unit(pre + '.shortcut', b.shortcut[0], b.shortcut[1], 'none')
                blocks.append(Block(pre, units, sc, identity=sc is None, final_act='relu'))
        fc = net.linear
        in_ch = net.conv1.in_channels
    elif isinstance(net, MobileNetV2):
        stem = Block('stem', [_bn_unit('conv1', net.conv1, net.bn1, 'relu6')], final_act='relu6',
                     need_dx=False)
        stem.units[0].need_dgrad = False
        blocks.append(stem)
        for i, b in enumerate(net.layers):
            assert isinstance(b, InvertedResidual)
            pre = 'layers.%d' % i
            units = [_bn_unit(pre + '.conv1', b.conv1, b.bn1, 'relu6'),
                     _bn_unit(pre + '.conv2', b.conv2, b.bn2, 'relu6', depthwise=True),
                     _bn_unit(pre + '.conv3', b.conv3, b.bn3, 'none')]
            sc, ident = None, False
            if b.stride == 1:
                if len(b.shortcut) > 0:
                    sc = _bn_unit(pre + '.shortcut', b.shortcut[0], b.shortcut[1], 'none')
                else:
                    ident = True
            blocks.append(Block(pre, units, sc, identity=ident, final_act='none'))
        blocks.append(Block('conv2', [_bn_unit('conv2', net.conv2, net.bn2, 'relu6')],
                            final_act='relu6'))
        fc = net.linear
        in_ch = 3
    elif isinstance(net, VGG):
        # speech VGG (`pytorch_model.py:117-153`): conv3x3(+bias)-BN-ReLU units, a 2x2 max-pool
        # after the units the config marks 'M', trailing AvgPool2d(1,1) (identity), then
        # flatten -> fc1 -> fc2 -> log_softmax.  Each conv is a one-unit block.
        feats = list(net.features)
        i = 0
        while i < len(feats):
            mod = feats[i]
            if isinstance(mod, nn.Conv2d):
                name = 'features.%d' % i
                u = _bn_unit(name, mod, feats[i + 1], 'relu')
                first = not blocks
                blk = Block(name, [u], None, identity=False, final_act='relu', need_dx=not first)
                if first:
                    u.need_dgrad = False
                i += 3
                if i < len(feats) and isinstance(feats[i], nn.MaxPool2d):
                    mp = feats[i]
                    blk.pool = (int(mp.kernel_size if isinstance(mp.kernel_size, int)
                                    else mp.kernel_size[0]),
                                int(mp.stride if isinstance(mp.stride, int) else mp.stride[0]), 0)
                    i += 1
                blocks.append(blk)
            elif isinstance(mod, nn.AvgPool2d) and mod.kernel_size in (1, (1, 1)):
                i += 1
            else:
                raise TypeError('unexpected VGG feature module %s' % type(mod).__name__)
        fc = net.fc2
        in_ch = feats[0].in_channels
    else:
        raise TypeError('native engine does not support %s' % type(net).__name__)

    lw = Lowered(blocks, fc, in_channels=in_ch, num_classes=fc.out_features)
    if isinstance(net, VGG):
        lw.head_pool = 'mlp2'
        lw.fc1 = net.fc1
    # flat layout in registration order
    unit_of = {}
    for blk in blocks:
        for u in blk.units + ([blk.shortcut] if blk.shortcut else []):
            unit_of[id(u.conv.weight)] = ('w', u)
            if u.conv.bias is not None:
                unit_of[id(u.conv.bias)] = ('b', u)
            unit_of[id(u.bn.weight)] = ('g', u)
            unit_of[id(u.bn.bias)] = ('beta', u)
    off = 0
    for name, p in net.named_parameters():
        role = unit_of.get(id(p))
        if role is not None and role[0] == 'w':
            kind = 'dw' if role[1].depthwise else 'conv'
        elif p is fc.weight or (lw.fc1 is not None and p is lw.fc1.weight):
            kind = 'fc'
        else:
            kind = 'vec'
        s = Seg(name, p, off, p.numel(), kind)
        lw.segs.append(s)
        if role is not None:
            r, u = role
            if r == 'w':
                u.w_seg = s
            elif r == 'b':
                u.b_seg = s
            elif r == 'g':
                u.g_seg = s
            else:
                u.beta_seg = s
        off += (p.numel() + 3) // 4 * 4
    lw.total = off
    lw.fc_w = next(s for s in lw.segs if s.param is fc.weight)
    lw.fc_b = next(s for s in lw.segs if s.param is fc.bias)
    if lw.fc1 is not None:
        lw.fc1_w = next(s for s in lw.segs if s.param is lw.fc1.weight)
        lw.fc1_b = next(s for s in lw.segs if s.param is lw.fc1.bias)
    return lw

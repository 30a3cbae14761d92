"""Inception-v3 image net of ``Torch_multi/myNet.py:17-330`` (the frozen feature extractor of
the reference's VIDEO_QUERY, ``main_run.py:228-256``), built from a layer table.

It is off the audio separation path -- the audio drivers construct VIDEO_QUERY
(``main_run.py:407``) but never call it -- so it is plain torch (nn.Conv2d / BatchNorm2d),
not a HIP kernel.  What a driver needs from it is that it CONSTRUCTS and that a
reference / torchvision ``inception_v3_google-1a9a5a14.pth`` loads by name: the
parameter names here are the reference's (``Conv2d_1a_3x3.conv.weight``,
``Mixed_5b.branch1x1.bn.running_mean``, ``AuxLogits.fc.weight``, ...).  Differences:

* the init draws truncated normals with torch (``trunc_normal_``, +-2 std, std 0.1 /
  0.01 conv1 of the aux head / 0.001 its fc) into the weight's own shape -- the
  reference copies a flat scipy draw into an N-d weight (``myNet.py:66-67``), which
  raises in every torch since 0.4;
* ``inception_v3(pretrained=True)`` loads the local ``inception_v3_google-1a9a5a14.pth``
  with ``weights_only=True`` when the file exists and keeps the random init otherwise
  (the reference raises; nothing is downloaded either way).
"""
import os

import torch
import torch.nn.functional as F
from torch import nn

PRETRAINED_FILE = "inception_v3_google-1a9a5a14.pth"


class BasicConv2d(nn.Module):
    """conv (no bias) -> BatchNorm(eps 1e-3) -> ReLU (myNet.py:319-329)."""

    def __init__(self, cin, cout, k, s=1, p=0, std=0.1):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride=s, padding=p, bias=False)
        self.bn = nn.BatchNorm2d(cout, eps=0.001)
        self.conv.stddev = std

    def forward(self, x):
        return F.relu(self.bn(self.conv(x)), inplace=True)


# A branch is a list of steps: ("c", name, cout, kernel, stride, pad) conv, or a pool
# ("avg3" 3x3/1 pad 1, "max3s2" 3x3/2) applied to the branch input.  Pools carry no
# parameters.  Each mixed block concatenates its branches in table order.
def _blockA(pool):
    return [[("c", "branch1x1", 64, 1, 1, 0)],
            [("c", "branch5x5_1", 48, 1, 1, 0), ("c", "branch5x5_2", 64, 5, 1, 2)],
            [("c", "branch3x3dbl_1", 64, 1, 1, 0), ("c", "branch3x3dbl_2", 96, 3, 1, 1),
             ("c", "branch3x3dbl_3", 96, 3, 1, 1)],
            [("avg3",), ("c", "branch_pool", pool, 1, 1, 0)]]


_blockB = [[("c", "branch3x3", 384, 3, 2, 0)],
           [("c", "branch3x3dbl_1", 64, 1, 1, 0), ("c", "branch3x3dbl_2", 96, 3, 1, 1),
            ("c", "branch3x3dbl_3", 96, 3, 2, 0)],
           [("max3s2",)]]


def _blockC(c7):
    r, c = (1, 7), (7, 1)
    pr, pc = (0, 3), (3, 0)
    return [[("c", "branch1x1", 192, 1, 1, 0)],
            [("c", "branch7x7_1", c7, 1, 1, 0), ("c", "branch7x7_2", c7, r, 1, pr), ("c", "branch7x7_3", 192, c, 1, pc)],
            [("c", "branch7x7dbl_1", c7, 1, 1, 0), ("c", "branch7x7dbl_2", c7, c, 1, pc),
             ("c", "branch7x7dbl_3", c7, r, 1, pr), ("c", "branch7x7dbl_4", c7, c, 1, pc),
             ("c", "branch7x7dbl_5", 192, r, 1, pr)],
            [("avg3",), ("c", "branch_pool", 192, 1, 1, 0)]]


_blockD = [[("c", "branch3x3_1", 192, 1, 1, 0), ("c", "branch3x3_2", 320, 3, 2, 0)],
           [("c", "branch7x7x3_1", 192, 1, 1, 0), ("c", "branch7x7x3_2", 192, (1, 7), 1, (0, 3)),
            ("c", "branch7x7x3_3", 192, (7, 1), 1, (3, 0)), ("c", "branch7x7x3_4", 192, 3, 2, 0)],
           [("max3s2",)]]

# InceptionE: two branches end in a (1x3 | 3x1) fork whose outputs are concatenated
_blockE = [[("c", "branch1x1", 320, 1, 1, 0)],
           [("c", "branch3x3_1", 384, 1, 1, 0), ("fork", ("branch3x3_2a", 384, (1, 3), 1, (0, 1)),
                                                  ("branch3x3_2b", 384, (3, 1), 1, (1, 0)))],
           [("c", "branch3x3dbl_1", 448, 1, 1, 0), ("c", "branch3x3dbl_2", 384, 3, 1, 1),
            ("fork", ("branch3x3dbl_3a", 384, (1, 3), 1, (0, 1)), ("branch3x3dbl_3b", 384, (3, 1), 1, (1, 0)))],
           [("avg3",), ("c", "branch_pool", 192, 1, 1, 0)]]


class Mixed(nn.Module):
    def __init__(self, cin, table):
        super().__init__()
        self.table = table
        for branch in table:
            c = cin
            for st in branch:
                if st[0] == "c":
                    setattr(self, st[1], BasicConv2d(c, *st[2:]))
                    c = st[2]
                elif st[0] == "fork":
                    for name, cout, k, s, p in st[1:]:
                        setattr(self, name, BasicConv2d(c, cout, k, s, p))

    def forward(self, x):
        outs = []
        for branch in self.table:
            y = x
            for st in branch:
                if st[0] == "c":
                    y = getattr(self, st[1])(y)
                elif st[0] == "avg3":
                    y = F.avg_pool2d(y, kernel_size=3, stride=1, padding=1)
                elif st[0] == "max3s2":
                    y = F.max_pool2d(y, kernel_size=3, stride=2)
                else:  # fork
                    y = torch.cat([getattr(self, f[0])(y) for f in st[1:]], 1)
            outs.append(y)
        return torch.cat(outs, 1)


class InceptionAux(nn.Module):
    def __init__(self, cin, num_classes):
        super().__init__()
        self.conv0 = BasicConv2d(cin, 128, 1)
        self.conv1 = BasicConv2d(128, 768, 5, std=0.01)
        self.fc = nn.Linear(768, num_classes)
        self.fc.stddev = 0.001

    def forward(self, x):
        x = self.conv1(self.conv0(F.avg_pool2d(x, kernel_size=5, stride=3)))
        return self.fc(x.flatten(1))


# the stem (name, cin, cout, kernel, stride, pad), max-pools after 2b and 4a
_STEM = [("Conv2d_1a_3x3", 3, 32, 3, 2, 0), ("Conv2d_2a_3x3", 32, 32, 3, 1, 0), ("Conv2d_2b_3x3", 32, 64, 3, 1, 1),
         ("Conv2d_3b_1x1", 64, 80, 1, 1, 0), ("Conv2d_4a_3x3", 80, 192, 3, 1, 0)]
_POOL_AFTER = {"Conv2d_2b_3x3", "Conv2d_4a_3x3"}
_MIXED = [("Mixed_5b", 192, _blockA(32)), ("Mixed_5c", 256, _blockA(64)), ("Mixed_5d", 288, _blockA(64)),
          ("Mixed_6a", 288, _blockB), ("Mixed_6b", 768, _blockC(128)), ("Mixed_6c", 768, _blockC(160)),
          ("Mixed_6d", 768, _blockC(160)), ("Mixed_6e", 768, _blockC(192)),
          ("Mixed_7a", 768, _blockD), ("Mixed_7b", 1280, _blockE), ("Mixed_7c", 2048, _blockE)]


class Inception3(nn.Module):
    """forward (training, aux_logits): (logits, aux logits, 2048-d pooled feature) -- the
    reference's third output, which VIDEO_QUERY reads as ``images_net(x)[2]``
    (myNet.py:123-128); otherwise the logits."""

    def __init__(self, num_classes=1000, aux_logits=True, transform_input=False):
        super().__init__()
        self.aux_logits, self.transform_input = aux_logits, transform_input
        for name, cin, cout, k, s, p in _STEM:
            setattr(self, name, BasicConv2d(cin, cout, k, s, p))
        for name, cin, table in _MIXED:
            setattr(self, name, Mixed(cin, table))
            if name == "Mixed_6e" and aux_logits:
                self.AuxLogits = InceptionAux(768, num_classes)
        self.fc = nn.Linear(2048, num_classes)
        with torch.no_grad():
            for m in self.modules():
                if isinstance(m, (nn.Conv2d, nn.Linear)):
                    std = getattr(m, "stddev", None)
                    if std is None:  # BasicConv2d carries it on its conv; the top fc uses 0.1
                        std = 0.1
                    nn.init.trunc_normal_(m.weight, std=std, a=-2 * std, b=2 * std)
                elif isinstance(m, nn.BatchNorm2d):
                    m.weight.fill_(1)
                    m.bias.zero_()

    def forward(self, x):
        if self.transform_input:  # ImageNet normalisation -> the TF model's [-1, 1] inputs
            x = x.clone()
            for c, (sd, mu) in enumerate(((0.229, 0.485), (0.224, 0.456), (0.225, 0.406))):
                x[:, c] = x[:, c] * (sd / 0.5) + (mu - 0.5) / 0.5
        for name, *_ in _STEM:
            x = getattr(self, name)(x)
            if name in _POOL_AFTER:
                x = F.max_pool2d(x, kernel_size=3, stride=2)
        aux = None
        for name, _, _ in _MIXED:
            x = getattr(self, name)(x)
            if name == "Mixed_6e" and self.training and self.aux_logits:
                aux = self.AuxLogits(x)
        feat = F.dropout(F.avg_pool2d(x, kernel_size=8), training=self.training).flatten(1)
        logits = self.fc(feat)
        if self.training and self.aux_logits:
            return logits, aux, feat
        return logits


def inception_v3(pretrained=False, **kwargs):
    """myNet.py:17-32: with ``pretrained`` the input transform is on and the local
    ImageNet weights file is loaded (weights_only) if it exists."""
    if pretrained:
        kwargs.setdefault("transform_input", True)
    model = Inception3(**kwargs)
    if pretrained and os.path.exists(PRETRAINED_FILE):
        model.load_state_dict(torch.load(PRETRAINED_FILE, map_location="cpu", weights_only=True))
    return model

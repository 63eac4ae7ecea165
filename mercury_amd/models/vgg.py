"""VGG for Google-Speech-Commands spectrograms (`pytorch_model.py:117-153`).

Input is 1x101x161 (F9): five 2x2 max-pools leave 512x3x5 = 7680 features,
which is ``fc1``'s in-width.  Module names (``features``, ``fc1``, ``fc2``)
match the reference so state dicts interchange.  ``in_channels`` is exposed
(reference hard-codes 1 with a comment that SVHN would use 3).
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

cfg = {
    'VGG11': [64, 'M', 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
    'VGG13': [64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
    'VGG16': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M',
              512, 512, 512, 'M'],
    'VGG19': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 256, 'M', 512, 512, 512, 512, 'M',
              512, 512, 512, 512, 'M'],
}


def _make_layers(spec, in_channels=1):
    layers = []
    for v in spec:
        if v == 'M':
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers += [nn.Conv2d(in_channels, v, 3, padding=1), nn.BatchNorm2d(v),
                       nn.ReLU(inplace=True)]
            in_channels = v
    layers.append(nn.AvgPool2d(1, 1))
    return nn.Sequential(*layers)


class VGG(nn.Module):
    def __init__(self, vgg_name, num_classes, in_channels=1, in_features=7680):
        super().__init__()
        self.features = _make_layers(cfg[vgg_name], in_channels)
        self.fc1 = nn.Linear(in_features, 128)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x):
        out = self.features(x).flatten(1)
        return F.log_softmax(self.fc2(self.fc1(out)), dim=1)

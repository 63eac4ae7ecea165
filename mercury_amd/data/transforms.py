"""Self-contained image transforms (torchvision is not installed).

Semantics follow the transforms the reference composes in
`cifar10/data_loader.py:78-111` and `exp_dataset.py:22-29,63-67`.  Inputs are
HWC uint8 ``numpy`` arrays (what ``CIFAR10_truncated.data`` holds) or CHW float
tensors after ``ToTensor``.  The randomness uses numpy's global RNG (like
torchvision uses torch's) so seeded runs are reproducible.

On the GPU hot path none of these run: ``mercury_amd.ops.augment_pool`` does
crop+flip+normalize for a whole presample pool in one HIP kernel from the
HBM-resident uint8 shard.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

CIFAR_MEAN = [0.49139968, 0.48215827, 0.44653124]
CIFAR_STD = [0.24703233, 0.24348505, 0.26158768]


class Compose(object):
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class ToPILImage(object):
    """Identity on HWC uint8 arrays (kept so reference pipelines read the same)."""

    def __call__(self, x):
        return np.asarray(x)


class ToNumpy(object):
    """PIL image / array -> ndarray (`util.py:73-91`)."""

    def __call__(self, pic):
        return np.array(pic)

    def __repr__(self):
        return self.__class__.__name__ + '()'


def _as_hwc(x):
    if torch.is_tensor(x):
        return x
    x = np.asarray(x)
    if x.ndim == 2:
        x = x[:, :, None]
    return x


class RandomCrop(object):
    def __init__(self, size, padding=0):
        self.size = size
        self.padding = padding

    def __call__(self, x):
        x = _as_hwc(x)
        if torch.is_tensor(x):  # CHW tensor
            p = self.padding
            if p:
                x = F.pad(x, (p, p, p, p))
            h, w = x.shape[-2:]
            i = np.random.randint(0, h - self.size + 1)
            j = np.random.randint(0, w - self.size + 1)
            return x[..., i:i + self.size, j:j + self.size]
        p = self.padding
        if p:
            x = np.pad(x, ((p, p), (p, p), (0, 0)))
        h, w = x.shape[:2]
        i = np.random.randint(0, h - self.size + 1)
        j = np.random.randint(0, w - self.size + 1)
        return x[i:i + self.size, j:j + self.size]


class RandomHorizontalFlip(object):
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, x):
        if np.random.rand() < self.p:
            if torch.is_tensor(x):
                return x.flip(-1)
            return _as_hwc(x)[:, ::-1]
        return x


class ToTensor(object):
    def __call__(self, x):
        if torch.is_tensor(x):
            return x
        x = np.ascontiguousarray(_as_hwc(x))
        t = torch.from_numpy(x).permute(2, 0, 1).contiguous()
        return t.float().div_(255.0) if t.dtype == torch.uint8 else t.float()


class Normalize(object):
    def __init__(self, mean, std):
        self.mean = torch.tensor(mean, dtype=torch.float32).view(-1, 1, 1)
        self.std = torch.tensor(std, dtype=torch.float32).view(-1, 1, 1)

    def __call__(self, t):
        return (t - self.mean) / self.std


class Resize(object):
    """Resize the shorter side to ``size`` (bilinear) like torchvision."""

    def __init__(self, size):
        self.size = size

    def __call__(self, x):
        t = x if torch.is_tensor(x) else torch.from_numpy(
            np.ascontiguousarray(_as_hwc(x))).permute(2, 0, 1).float()
        h, w = t.shape[-2:]
        if h <= w:
            nh, nw = self.size, int(self.size * w / h)
        else:
            nh, nw = int(self.size * h / w), self.size
        out = F.interpolate(t[None], size=(nh, nw), mode='bilinear', align_corners=False)[0]
        if torch.is_tensor(x):
            return out
        return out.clamp(0, 255).round().byte().permute(1, 2, 0).numpy()


class RandomAffine(object):
    """Rotation + isotropic scale about the centre (the subset used by `exp_dataset.py:27`)."""

    def __init__(self, degrees, scale=None):
        self.degrees = (-degrees, degrees) if np.isscalar(degrees) else degrees
        self.scale = scale

    def __call__(self, x):
        is_np = not torch.is_tensor(x)
        t = torch.from_numpy(np.ascontiguousarray(_as_hwc(x))).permute(2, 0, 1).float() \
            if is_np else x.float()
        ang = math.radians(np.random.uniform(*self.degrees))
        sc = np.random.uniform(*self.scale) if self.scale else 1.0
        c, s = math.cos(ang) / sc, math.sin(ang) / sc
        theta = torch.tensor([[c, -s, 0.0], [s, c, 0.0]], dtype=torch.float32)[None]
        grid = F.affine_grid(theta, [1] + list(t.shape), align_corners=False)
        out = F.grid_sample(t[None], grid, align_corners=False)[0]
        if is_np:
            return out.clamp(0, 255).round().byte().permute(1, 2, 0).numpy()
        return out


class Cutout(object):
    """Zero a random square (`cifar10/data_loader.py:57-75`)."""

    def __init__(self, length):
        self.length = length

    def __call__(self, img):
        h, w = img.size(1), img.size(2)
        mask = np.ones((h, w), np.float32)
        y = np.random.randint(h)
        x = np.random.randint(w)
        y1, y2 = np.clip(y - self.length // 2, 0, h), np.clip(y + self.length // 2, 0, h)
        x1, x2 = np.clip(x - self.length // 2, 0, w), np.clip(x + self.length // 2, 0, w)
        mask[y1:y2, x1:x2] = 0.
        return img * torch.from_numpy(mask).expand_as(img)


def cifar_train_transform():
    return Compose([ToPILImage(), RandomCrop(32, padding=4), RandomHorizontalFlip(),
                    ToTensor(), Normalize(CIFAR_MEAN, CIFAR_STD)])


def cifar_test_transform():
    return Compose([ToPILImage(), ToTensor(), Normalize(CIFAR_MEAN, CIFAR_STD)])


def _data_transforms_cifar10():
    return cifar_train_transform(), cifar_test_transform()

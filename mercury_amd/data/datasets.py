"""Index-returning datasets (`cifar10/datasets.py`, `util.py:162-181,240-273`).

Every dataset yields ``(index, img, target)`` -- the contract the importance
sampler relies on.  Real CIFAR downloads are impossible offline,
so ``load_cifar_arrays`` reads ``<root>/cifar{10,100}.npz`` (keys ``x_train``,
``y_train``, ``x_test``, ``y_test``; loaded with ``allow_pickle=False``) when it
exists and otherwise builds a deterministic *synthetic* CIFAR-shaped set:
uint8 HWC 32x32x3 images with exactly N/K samples per class whose pixels are a
per-class template plus noise, so a model can actually learn it (loss falls,
which keeps time-to-accuracy experiments meaningful).
"""
from __future__ import annotations

import logging
import os

import numpy as np
import torch
import torch.utils.data as data

IMG_EXTENSIONS = ('.jpg', '.jpeg', '.png', '.ppm', '.bmp', '.pgm', '.tif', '.tiff', '.webp')

_CACHE = {}


def synthetic_arrays(n, num_classes, shape=(32, 32, 3), seed=0, noise=48, template_seed=None):
    """Class-conditional synthetic images: template[class] + uniform noise.

    The class templates come from ``template_seed`` (default: fixed per class count and
    shape), NOT from ``seed`` -- so a train set and a test set drawn with different seeds share
    the same classes and only their noise/labels differ."""
    key = (n, num_classes, tuple(shape), seed, noise, template_seed)
    if key in _CACHE:
        return _CACHE[key]
    rng = np.random.RandomState(seed)
    per = n // num_classes
    y = np.repeat(np.arange(num_classes), per)
    y = np.concatenate([y, rng.randint(0, num_classes, n - len(y))]).astype(np.int64)
    rng.shuffle(y)
    # low-frequency templates so crops/flips keep the class signal
    h, w, c = shape
    tseed = template_seed if template_seed is not None else 0xC1A55 + 131 * num_classes + c
    small = np.random.RandomState(tseed).randint(
        40, 216, size=(num_classes, 4, 4, c)).astype(np.float32)
    tmpl = torch.nn.functional.interpolate(
        torch.from_numpy(small).permute(0, 3, 1, 2), size=(h, w), mode='bilinear',
        align_corners=False).permute(0, 2, 3, 1).numpy()
    x = np.empty((n,) + tuple(shape), dtype=np.uint8)
    chunk = max(1, (64 << 20) // (int(np.prod(shape)) * 4))   # ~64 MB of fp32 noise per chunk
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        nz = rng.randint(-noise, noise + 1, size=(e - s,) + tuple(shape)).astype(np.float32)
        x[s:e] = np.clip(tmpl[y[s:e]] + nz, 0, 255).astype(np.uint8)
    _CACHE[key] = (x, y)
    return x, y


def load_cifar_arrays(root, train=True, num_classes=10):
    """(X uint8 [N,32,32,3], y int64 [N]) from ``root/cifar{K}.npz`` or synthetic."""
    path = os.path.join(root or '.', 'cifar%d.npz' % num_classes)
    if os.path.exists(path):
        with np.load(path, allow_pickle=False) as z:
            if train:
                return z['x_train'], z['y_train'].astype(np.int64)
            return z['x_test'], z['y_test'].astype(np.int64)
    n = 50000 if train else 10000
    return synthetic_arrays(n, num_classes, seed=(1 if train else 2) + 7 * num_classes)


class CIFAR10_truncated(data.Dataset):
    """CIFAR subset by ``dataidxs`` (`cifar10/datasets.py:37-96`).

    ``index`` returned by ``__getitem__`` is local to the subset, as in the
    reference.  ``download`` is accepted and ignored (offline).
    """

    num_classes = 10

    def __init__(self, root, dataidxs=None, train=True, transform=None, target_transform=None,
                 download=False):
        self.root = root
        self.dataidxs = dataidxs
        self.train = train
        self.transform = transform
        self.target_transform = target_transform
        self.download = download
        self.data, self.target = self.__build_truncated_dataset__()

    def __build_truncated_dataset__(self):
        x, y = load_cifar_arrays(self.root, self.train, self.num_classes)
        if self.dataidxs is not None:
            idx = np.asarray(self.dataidxs, dtype=np.int64)
            x, y = x[idx], y[idx]
        return x, y

    def truncate_channel(self, index):
        for gs_index in np.asarray(index):
            self.data[gs_index, :, :, 1] = 0
            self.data[gs_index, :, :, 2] = 0

    def __getitem__(self, index):
        img, target = self.data[index], self.target[index]
        if self.transform is not None:
            img = self.transform(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return index, img, target

    def __len__(self):
        return len(self.data)


class CIFAR100_truncated(CIFAR10_truncated):
    num_classes = 100


class My_CIFAR10(data.Dataset):
    """Whole CIFAR-10 returning ``(index, img, target)`` + ``get_slice`` (`util.py:240-273`)."""

    num_classes = 10

    def __init__(self, root, train=True, transform=None, target_transform=None, download=False):
        self.root = root
        self.train = train
        self.transform = transform
        self.target_transform = target_transform
        self.data, targets = load_cifar_arrays(root, train, self.num_classes)
        self.targets = targets.tolist()

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        img, target = self.data[index], self.targets[index]
        if self.transform is not None:
            img = self.transform(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return index, img, target

    def get_slice(self, start, end):
        imgs, targets = [], []
        for i in range(start, end):
            _, img, target = self[i]
            imgs.append(img if torch.is_tensor(img) else torch.as_tensor(np.asarray(img)))
            targets.append(target)
        return torch.stack(imgs), torch.LongTensor(targets)


class SyntheticImageDataset(data.Dataset):
    """Generic synthetic (index, img, target) set, e.g. ImageNet-shaped 224x224."""

    def __init__(self, n, num_classes, shape=(224, 224, 3), transform=None, seed=0):
        self.data, self.target = synthetic_arrays(n, num_classes, shape, seed)
        self.transform = transform

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        img = self.data[index]
        if self.transform is not None:
            img = self.transform(img)
        return index, img, int(self.target[index])

    def get_slice(self, start, end):
        imgs = [torch.as_tensor(np.asarray(self[i][1])) for i in range(start, end)]
        return torch.stack(imgs), torch.as_tensor(self.target[start:end])


def pil_loader(path):
    from PIL import Image
    with open(path, 'rb') as f:
        img = Image.open(f)
        return img.convert('RGB')


def accimage_loader(path):
    try:
        import accimage  # noqa: F401
        return accimage.Image(path)
    except (ImportError, IOError):
        return pil_loader(path)


def default_loader(path):
    return pil_loader(path)


class SampleImageFolder(data.Dataset):
    """ImageFolder returning ``(index, sample, target)`` (`util.py:162-181`)."""

    def __init__(self, root, transform=None, target_transform=None, loader=default_loader,
                 extensions=IMG_EXTENSIONS):
        self.root = root
        self.transform = transform
        self.target_transform = target_transform
        self.loader = loader
        classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
        self.classes = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        samples = []
        for c in classes:
            for dirpath, _, files in sorted(os.walk(os.path.join(root, c))):
                for fn in sorted(files):
                    if fn.lower().endswith(extensions):
                        samples.append((os.path.join(dirpath, fn), self.class_to_idx[c]))
        self.samples = samples
        self.targets = [s[1] for s in samples]

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, index):
        path, target = self.samples[index]
        sample = self.loader(path)
        if self.transform is not None:
            sample = self.transform(sample)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return index, sample, target


logging.getLogger(__name__).addHandler(logging.NullHandler())

"""Non-IID partitioning and loader factories (`cifar10/data_loader.py`, `exp_dataset.py`).

``partition_data`` reproduces the reference's numpy RNG consumption exactly,
so with ``np.random.seed(102)`` the Dirichlet(0.5) shard sizes match SURVEY F7
(W=4 -> [13081, 7794, 13324, 15801]).  Loader factories return the same tuple
shapes as the reference.  Differences: W=1 is allowed
(`exp_dataset.py:10` asserts ``split_num > 1``), ``num_classes`` is a
parameter (reference hard-codes K=10), and CIFAR-100 is supported.
"""
from __future__ import annotations

import logging

import numpy as np
import torch.utils.data as data

from .datasets import (CIFAR10_truncated, CIFAR100_truncated, My_CIFAR10, load_cifar_arrays)
from .transforms import (Compose, RandomAffine, RandomCrop, RandomHorizontalFlip, Resize,
                         ToTensor, _data_transforms_cifar10)

log = logging.getLogger(__name__)


def read_data_distribution(filename='./data_preprocessing/non-iid-distribution/CIFAR10/distribution.txt'):
    """Parse the brace-text ``{client: {class: count}}`` file (`data_loader.py:16-29`)."""
    distribution = {}
    first = None
    with open(filename, 'r') as f:
        for x in f.readlines():
            if not x.strip() or x[0] in '{}':
                continue
            tmp = x.split(':')
            if tmp[1].strip() == '{':
                first = int(tmp[0])
                distribution[first] = {}
            else:
                distribution[first][int(tmp[0])] = int(tmp[1].strip().replace(',', ''))
    return distribution


def read_net_dataidx_map(filename='./data_preprocessing/non-iid-distribution/CIFAR10/net_dataidx_map.txt'):
    """Parse ``{client: [idx, idx, ...]}`` brace text (`data_loader.py:32-43`)."""
    net_dataidx_map = {}
    key = None
    with open(filename, 'r') as f:
        for x in f.readlines():
            if not x.strip() or x[0] in '{}]':
                continue
            tmp = x.split(':')
            if tmp[-1].strip() == '[':
                key = int(tmp[0])
                net_dataidx_map[key] = []
            else:
                net_dataidx_map[key] += [int(i.strip()) for i in x.split(',') if i.strip()]
    return net_dataidx_map


def record_net_data_stats(y_train, net_dataidx_map):
    net_cls_counts = {}
    for net_i, dataidx in net_dataidx_map.items():
        unq, unq_cnt = np.unique(y_train[dataidx], return_counts=True)
        net_cls_counts[net_i] = {int(unq[i]): int(unq_cnt[i]) for i in range(len(unq))}
    log.debug('Data statistics: %s', net_cls_counts)
    return net_cls_counts


def load_cifar10_data(datadir, num_classes=10):
    X_train, y_train = load_cifar_arrays(datadir, True, num_classes)
    X_test, y_test = load_cifar_arrays(datadir, False, num_classes)
    return X_train, y_train, X_test, y_test


def dirichlet_partition(y_train, n_nets, alpha, num_classes=None, min_require=10):
    """The reference 'hetero' loop (`data_loader.py:138-161`), RNG-order exact."""
    K = int(num_classes or (int(y_train.max()) + 1))
    N = y_train.shape[0]
    min_size = 0
    idx_batch = [[] for _ in range(n_nets)]
    while min_size < min_require:
        idx_batch = [[] for _ in range(n_nets)]
        for k in range(K):
            idx_k = np.where(y_train == k)[0]
            np.random.shuffle(idx_k)
            proportions = np.random.dirichlet(np.repeat(alpha, n_nets))
            proportions = np.array([p * (len(idx_j) < N / n_nets)
                                    for p, idx_j in zip(proportions, idx_batch)])
            proportions = proportions / proportions.sum()
            proportions = (np.cumsum(proportions) * len(idx_k)).astype(int)[:-1]
            idx_batch = [idx_j + idx.tolist()
                         for idx_j, idx in zip(idx_batch, np.split(idx_k, proportions))]
            min_size = min(len(idx_j) for idx_j in idx_batch)
        if n_nets == 1:
            break
    net_dataidx_map = {}
    for j in range(n_nets):
        np.random.shuffle(idx_batch[j])
        net_dataidx_map[j] = idx_batch[j]
    return net_dataidx_map


def partition_data(dataset, datadir, partition, n_nets, alpha, num_classes=10):
    """Returns ``(X_train, y_train, X_test, y_test, net_dataidx_map, traindata_cls_counts)``."""
    log.info('*********partition data***************')
    X_train, y_train, X_test, y_test = load_cifar10_data(datadir, num_classes)
    n_train = X_train.shape[0]
    if partition == 'homo':
        idxs = np.random.permutation(n_train)
        batch_idxs = np.array_split(idxs, n_nets)
        net_dataidx_map = {i: batch_idxs[i] for i in range(n_nets)}
    elif partition == 'hetero':
        net_dataidx_map = dirichlet_partition(y_train, n_nets, alpha, num_classes)
    elif partition == 'hetero-fix':
        net_dataidx_map = read_net_dataidx_map(
            './data_preprocessing/non-iid-distribution/CIFAR10/net_dataidx_map.txt')
    else:
        raise ValueError(partition)
    if partition == 'hetero-fix':
        traindata_cls_counts = read_data_distribution(
            './data_preprocessing/non-iid-distribution/CIFAR10/distribution.txt')
    else:
        traindata_cls_counts = record_net_data_stats(y_train, net_dataidx_map)
    return X_train, y_train, X_test, y_test, net_dataidx_map, traindata_cls_counts


def _truncated_cls(num_classes):
    return CIFAR100_truncated if num_classes == 100 else CIFAR10_truncated


def get_dataloader_CIFAR10(datadir, train_bs, test_bs, dataidxs=None, num_classes=10):
    dl_obj = _truncated_cls(num_classes)
    transform_train, transform_test = _data_transforms_cifar10()
    train_ds = dl_obj(datadir, dataidxs=dataidxs, train=True, transform=transform_train)
    test_ds = dl_obj(datadir, train=False, transform=transform_test)
    train_dl = data.DataLoader(train_ds, batch_size=train_bs, shuffle=True, drop_last=True)
    test_dl = data.DataLoader(test_ds, batch_size=test_bs, shuffle=False, drop_last=True)
    return train_dl, test_dl


def get_dataloader_test_CIFAR10(datadir, train_bs, test_bs, dataidxs_train=None,
                                dataidxs_test=None, num_classes=10):
    dl_obj = _truncated_cls(num_classes)
    transform_train, transform_test = _data_transforms_cifar10()
    train_ds = dl_obj(datadir, dataidxs=dataidxs_train, train=True, transform=transform_train)
    test_ds = dl_obj(datadir, dataidxs=dataidxs_test, train=False, transform=transform_test)
    train_dl = data.DataLoader(train_ds, batch_size=train_bs, shuffle=True, drop_last=True)
    test_dl = data.DataLoader(test_ds, batch_size=test_bs, shuffle=False, drop_last=True)
    return train_dl, test_dl


def get_dataloader(dataset, datadir, train_bs, test_bs, dataidxs=None):
    nc = 100 if str(dataset).lower() == 'cifar100' else 10
    return get_dataloader_CIFAR10(datadir, train_bs, test_bs, dataidxs, nc)


def get_dataloader_test(dataset, datadir, train_bs, test_bs, dataidxs_train, dataidxs_test):
    nc = 100 if str(dataset).lower() == 'cifar100' else 10
    return get_dataloader_test_CIFAR10(datadir, train_bs, test_bs, dataidxs_train,
                                       dataidxs_test, nc)


def load_partition_data_cifar10(dataset, data_dir, partition_method, partition_alpha,
                                client_number, batch_size):
    """8-tuple of `data_loader.py:248-282`."""
    nc = 100 if str(dataset).lower() == 'cifar100' else 10
    X_train, y_train, X_test, y_test, net_dataidx_map, traindata_cls_counts = partition_data(
        dataset, data_dir, partition_method, client_number, partition_alpha, nc)
    class_num = len(np.unique(y_train))
    train_data_num = sum(len(net_dataidx_map[r]) for r in range(client_number))
    train_data_global, test_data_global = get_dataloader(dataset, data_dir, batch_size, batch_size)
    test_data_num = len(test_data_global)
    data_local_num_dict, train_data_local_dict, test_data_local_dict = {}, {}, {}
    for client_idx in range(client_number):
        dataidxs = net_dataidx_map[client_idx]
        data_local_num_dict[client_idx] = len(dataidxs)
        tr, te = get_dataloader(dataset, data_dir, batch_size, batch_size, dataidxs)
        train_data_local_dict[client_idx] = tr
        test_data_local_dict[client_idx] = te
    return (train_data_num, test_data_num, train_data_global, test_data_global,
            data_local_num_dict, train_data_local_dict, test_data_local_dict, class_num)


def load_partition_data_distributed_cifar10(process_id, dataset, data_dir, partition_method,
                                            partition_alpha, client_number, batch_size):
    """7-tuple of `data_loader.py:208-245`: process 0 global, process k shard k-1."""
    nc = 100 if str(dataset).lower() == 'cifar100' else 10
    X_train, y_train, X_test, y_test, net_dataidx_map, _ = partition_data(
        dataset, data_dir, partition_method, client_number, partition_alpha, nc)
    class_num = len(np.unique(y_train))
    train_data_num = sum(len(net_dataidx_map[r]) for r in range(client_number))
    if process_id == 0:
        train_data_global, test_data_global = get_dataloader(dataset, data_dir, batch_size,
                                                             batch_size)
        train_data_local = test_data_local = None
        local_data_num = 0
    else:
        dataidxs = net_dataidx_map[process_id - 1]
        local_data_num = len(dataidxs)
        train_data_local, test_data_local = get_dataloader(dataset, data_dir, batch_size,
                                                           batch_size, dataidxs)
        train_data_global = test_data_global = None
    return (train_data_num, train_data_global, test_data_global, local_data_num,
            train_data_local, test_data_local, class_num)


# ---- exp_dataset.py equivalents -------------------------------------------------------

def load_cifar10_noniid(split_num, alpha, batch_size=32, data_dir='./data/cifar10',
                        dataset='cifar10'):
    """``(presam_loaders[list], train_loader, test_loader)`` (`exp_dataset.py:9-18`).

    W=1 is allowed (the reference asserts ``split_num > 1``)."""
    out = load_partition_data_cifar10(dataset, data_dir, 'hetero', alpha, split_num, batch_size)
    train_data_local_dict = out[5]
    presam_loaders = [train_data_local_dict[i] for i in range(split_num)]
    return presam_loaders, out[2], out[3]


def load_cifar10(split_num=1, batch_size=32, root='datasets/cifar10'):
    """IID variant (`exp_dataset.py:21-77`) -> ``(train_loader, presam_loader, test_loader)``."""
    import torch
    train_set = My_CIFAR10(root, train=True, transform=Compose([
        Resize(35), RandomCrop(32), RandomHorizontalFlip(),
        RandomAffine(degrees=10, scale=(0.9, 1.1)), ToTensor()]))
    if split_num > 1:
        subsets = np.array_split(np.arange(len(train_set)), split_num)
        train_loader = data.DataLoader(train_set, batch_size=batch_size, shuffle=True)
        parts = torch.utils.data.random_split(train_set, [len(s) for s in subsets])
        presam_loader = [data.DataLoader(ds, batch_size=batch_size, shuffle=True) for ds in parts]
    else:
        train_loader = data.DataLoader(train_set, batch_size=batch_size, shuffle=True)
        presam_loader = data.DataLoader(train_set, batch_size=batch_size, shuffle=False)
    test_set = My_CIFAR10(root, train=False, transform=Compose([
        Resize(33), RandomCrop(32), ToTensor()]))
    test_loader = data.DataLoader(test_set, batch_size=batch_size, shuffle=True)
    return train_loader, presam_loader, test_loader

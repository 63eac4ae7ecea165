"""Data: index-returning datasets, transforms, non-IID partitioner, loader factories,
and the HBM-resident device pool used by the native engine."""
from .datasets import (CIFAR10_truncated, CIFAR100_truncated, My_CIFAR10, SampleImageFolder,
                       SyntheticImageDataset, load_cifar_arrays, synthetic_arrays)
from .transforms import (CIFAR_MEAN, CIFAR_STD, Compose, Cutout, Normalize, RandomCrop,
                         RandomHorizontalFlip, ToNumpy, ToPILImage, ToTensor,
                         _data_transforms_cifar10)
from .partition import (partition_data, dirichlet_partition, record_net_data_stats,
                        read_data_distribution, read_net_dataidx_map, get_dataloader,
                        get_dataloader_test, get_dataloader_CIFAR10,
                        load_partition_data_cifar10, load_partition_data_distributed_cifar10,
                        load_cifar10_noniid, load_cifar10)

__all__ = [n for n in dir() if not n.startswith('__')]

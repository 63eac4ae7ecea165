import numpy as np
import pytest

from mercury_amd.data import (CIFAR10_truncated, dirichlet_partition, load_cifar10_noniid,
                              partition_data, record_net_data_stats)


@pytest.mark.parametrize('W,sizes', [
    (4, [13081, 7794, 13324, 15801]),
    (2, [22485, 27515]),
    (8, [5585, 7200, 6656, 6725, 8800, 3473, 6800, 4761])])
def test_dirichlet_shard_sizes_match_reference(W, sizes):
    # seed 102, alpha 0.5, 5000 samples per class
    y = np.repeat(np.arange(10), 5000)
    np.random.seed(102)
    m = dirichlet_partition(y, W, 0.5, 10)
    assert [len(m[i]) for i in range(W)] == sizes
    allidx = np.concatenate([m[i] for i in range(W)])
    assert len(np.unique(allidx)) == 50000


def test_partition_data_synthetic_counts():
    np.random.seed(102)
    X, y, Xt, yt, m, counts = partition_data('cifar10', '/nonexistent', 'hetero', 4, 0.5)
    assert X.shape == (50000, 32, 32, 3) and X.dtype == np.uint8
    assert [len(m[i]) for i in range(4)] == [13081, 7794, 13324, 15801]
    assert sum(sum(c.values()) for c in counts.values()) == 50000
    np.random.seed(0)
    _, _, _, _, mh, _ = partition_data('cifar10', '/nonexistent', 'homo', 3, 0.5)
    assert sorted(len(v) for v in mh.values()) == [16666, 16667, 16667]


def test_truncated_returns_index_img_target():
    ds = CIFAR10_truncated('/nonexistent', dataidxs=[5, 7, 9], train=True)
    assert len(ds) == 3
    i, img, t = ds[1]
    assert i == 1 and img.shape == (32, 32, 3)


def test_noniid_loaders_world1_allowed():
    np.random.seed(102)
    pres, train, test = load_cifar10_noniid(1, 0.5, data_dir='/nonexistent')
    assert len(pres) == 1 and len(train) == 50000 // 32
    idx, data, label = next(iter(pres[0]))
    assert data.shape == (32, 3, 32, 32) and idx.shape == (32,)
    assert abs(float(data.mean())) < 3.0


def test_synthetic_train_test_share_classes():
    """Train and test synthetic CIFAR arrays come from different seeds but the SAME class
    templates (otherwise held-out accuracy is meaningless)."""
    from mercury_amd.data.datasets import load_cifar_arrays
    xa, ya = load_cifar_arrays('/nonexistent', train=True)
    xb, yb = load_cifar_arrays('/nonexistent', train=False)
    assert not np.array_equal(xa[:100], xb[:100])
    ma = np.stack([xa[ya == k][:500].mean(0) for k in range(10)])
    mb = np.stack([xb[yb == k][:500].mean(0) for k in range(10)])
    same = np.abs(ma - mb).mean()
    cross = np.abs(ma - np.roll(mb, 1, axis=0)).mean()
    assert same < 0.2 * cross, (same, cross)

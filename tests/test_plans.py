"""Host-side plan logic (no GPU): the halo conv's padded row tiles, the measured padded and
prologue plans, and the persistent plans' launch constraints."""
import pytest

from mercury_amd.ops import hconv as H
from mercury_amd.ops.conv import MEASURED_PRO, ConvSpec, pro_ok, pro_plan


def _spec(N, Hh, C, K, st=1, gi=None):
    sp = ConvSpec(N, Hh, Hh, C, K, 3, 3, st, 1)
    if gi:
        sp.group_rows = gi * sp.P * sp.Q
    return sp


@pytest.mark.parametrize('N,Hh,C,bm,img,tr', [
    (1280, 56, 64, 128, 1, 2),     # 2 x 56 = 112 of 128
    (1280, 56, 64, 256, 1, 4),     # 4 x 56 = 224 of 256
    (1280, 28, 128, 128, 1, 4),    # 4 x 28 = 112
    (1280, 28, 128, 256, 1, 7),    # 7 x 28 = 196 (28 % 8, 28 % 9 != 0)
    (1280, 14, 256, 128, 1, 7),    # 7 x 14 = 98
    (1280, 7, 512, 128, 2, 7),     # two 49-pixel images = 98
])
def test_padded_tile_shapes(N, Hh, C, bm, img, tr):
    sp = _spec(N, Hh, C, C, gi=128)
    assert H._tile_shape(sp, bm) is None            # no whole-row tile fills bm exactly
    assert H._tile_shape(sp, bm, pad=True) == (img, tr)
    vr = img * tr * sp.Q
    assert vr >= H.PAD_MIN * bm and sp.M % vr == 0 and sp.group_rows % vr == 0
    assert H.persistent_ok(sp, bm, 64)


def test_exact_tiles_unchanged_by_padding():
    # the CIFAR shapes tile exactly: the padded search returns the same shape
    for N, Hh, C, bm in ((320, 32, 64, 256), (320, 16, 128, 256), (320, 8, 256, 128),
                         (320, 4, 512, 64), (32, 32, 64, 256)):
        sp = _spec(N, Hh, C, C, gi=32)
        assert H._tile_shape(sp, bm) == H._tile_shape(sp, bm, pad=True) is not None


def test_padding_below_the_floor_is_refused():
    # 1 x 80 of 128 (62.5 %) and 2 x 80 of 256 would waste too many MFMA rows
    sp = ConvSpec(320, 50, 80, 128, 128, 3, 3, 1, 1)
    assert H._tile_shape(sp, 128, pad=True) is None
    assert H._tile_shape(sp, 256, pad=True) is None


def test_padded_geometry_fits_and_row_kernels_reject_it():
    sp = _spec(1280, 56, 64, 64, gi=128)
    g = H.geometry(sp, 256, 64, pad=True)
    assert g is not None and g['IMG'] * g['TR'] * g['Q'] == 224
    assert H.lds_bytes(g, 256, 64, 0) <= H.LDS_MAX
    assert g['PGRID'] == 0
    assert H.geometry(sp, 256, 64) is None          # per-tile / row-step kernels: exact only
    assert not H.row_ok(sp, 256, 64)


def test_measured_pad_plans_are_launchable():
    for (N, Hh, C, K), (p, fold) in H.MEASURED_PAD.items():
        sp = _spec(N, Hh, C, K, gi=128)
        assert p[2] == 0 and len(p) == 4 and 0 < p[3] <= 4096
        g = H.geometry(sp, p[0], p[1], pad=True)
        assert g is not None and H.lds_bytes(g, p[0], p[1], 0) <= H.LDS_MAX
        assert H.persistent_ok(sp, p[0], p[1])
        if fold:
            pro = dict(stats=True, group_imgs=128)
            assert H.lds_bytes(g, p[0], p[1], 0) + H.persist_table_bytes(sp, pro) <= H.LDS_MAX
        assert H.engine_plan(sp, train=N <= 128) == p


def test_pad_plans_follow_the_switch():
    sp = _spec(1280, 56, 64, 64, gi=128)
    old = H._CFG['pad']
    try:
        H._CFG['pad'] = False
        p = H.engine_plan(sp, train=False)
        assert p is None or len(p) < 4              # no padded plan with the switch off
        H._CFG['pad'] = True
        assert H.engine_plan(sp, train=False) == H.MEASURED_PAD[(1280, 56, 64, 64)][0]
        assert H.persist_bn_plan(sp, 128, row_only=True) == H.MEASURED_PAD[(1280, 56, 64, 64)][0]
    finally:
        H._CFG['pad'] = old


def test_measured_prologue_plans_take_the_prologue():
    for (N, Hh, C, K), p in MEASURED_PRO.items():
        sp = ConvSpec(N, Hh, Hh, C, K, 1, 1, 1, 0)
        assert pro_plan(sp) == p
        assert pro_ok(sp, p, keep=True), (N, Hh, C, K, p)
    # ghost-BN groups (the scoring batch) and 3x3 convs are not in the table's scope
    sp = ConvSpec(32, 8, 8, 576, 96, 1, 1, 1, 0)
    sp.group_rows = 16 * 64
    assert pro_plan(sp) is None
    assert pro_plan(ConvSpec(32, 8, 8, 576, 96, 3, 3, 1, 1)) is None

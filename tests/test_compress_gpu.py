"""Ternary-compressed gradient wire on the GPU: the HIP pack / decode kernels (csrc/misc.hip)
against the torch layout of parallel/compress.py, unbiasedness of the Philox draws, and the
native engine's forced-bucket RCCL path with grad_compress='ternary'."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n', [1, 16, 1001, 65536 + 5])
def test_pack_kernel_message(n):
    from mercury_amd import ops
    from mercury_amd.parallel.compress import decode_sum_torch, tern_words
    ops.lib()
    g = torch.Generator(device='cpu').manual_seed(n)
    x = (torch.randn(n, generator=g) * 0.3).cuda()
    x[0] = 0.0
    if n > 3:
        x[3] = 2.5                                   # the maximum: always kept
    words = torch.zeros(tern_words(n), dtype=torch.int32, device='cuda')
    ws = torch.zeros(1, device='cuda')
    ops.tern_pack(x, words, ws, seed=11, counter=4)
    torch.cuda.synchronize()
    m = float(x.abs().max())
    dec = decode_sum_torch(words.view(1, -1).cpu(), n, avg=False)
    assert torch.allclose(words[:1].view(torch.float32).cpu(), torch.tensor([m]))
    nz = dec != 0
    assert torch.allclose(dec[nz].abs(), torch.full_like(dec[nz], m))
    assert (torch.sign(dec[nz]) == torch.sign(x.cpu()[nz])).all()
    assert dec[0] == 0
    if n > 3:
        assert dec[3] == m


def test_unpack_kernel_matches_torch_decode():
    from mercury_amd import ops
    from mercury_amd.parallel.compress import decode_sum_torch, encode_torch, tern_words
    ops.lib()
    g = torch.Generator().manual_seed(2)
    n, W = 4099, 3
    msgs = torch.stack([encode_torch(torch.randint(-1, 2, (n,), generator=g).to(torch.int8),
                                     0.5 + r) for r in range(W)])
    out = torch.empty(n, device='cuda')
    ops.tern_unpack(msgs.cuda(), W, n, out)
    torch.cuda.synchronize()
    assert torch.allclose(out.cpu(), decode_sum_torch(msgs, n))
    assert msgs.shape[1] == tern_words(n)


def test_pack_unbiased_over_counters():
    from mercury_amd import ops
    from mercury_amd.parallel.compress import tern_words
    ops.lib()
    n = 4096
    x = torch.linspace(-1.0, 1.0, n, device='cuda')
    words = torch.zeros(tern_words(n), dtype=torch.int32, device='cuda')
    ws = torch.zeros(1, device='cuda')
    acc = torch.zeros(n, device='cuda')
    out = torch.empty(n, device='cuda')
    reps = 400
    for c in range(reps):
        ops.tern_pack(x, words, ws, seed=3, counter=c)
        ops.tern_unpack(words, 1, n, out)
        acc += out
    torch.cuda.synchronize()
    err = (acc / reps - x).abs()
    assert float(err.max()) < 6 / reps ** 0.5          # var <= |x| max|x| <= 1
    assert abs(float((acc / reps - x).mean())) < 0.01


def test_engine_ternary_world1():
    import torch.distributed as dist
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    from mercury_amd.parallel.dist import free_port
    if dist.is_initialized():
        dist.destroy_process_group()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % free_port(), rank=0,
                            world_size=1, device_id=torch.device('cuda', 0))
    try:
        x, y = synthetic_arrays(3000, 10, seed=5)
        torch.manual_seed(7)
        e = NativeEngine(ResNet18(10).cuda(), 'cuda', 32, 10, bucket_bytes=4 << 20, seed=3,
                         force_buckets=True, comm='rccl', grad_compress='ternary')
        assert e.tern is not None and len(e.bucket_plan()) > 1
        e.set_shard(x, y)
        e.prime()
        p0 = e.opt.p.clone()
        e.step()
        e.build_graphs()
        for _ in range(20):
            e.step()
        torch.cuda.synchronize()
        m = e.read_meters()
        assert torch.isfinite(e.opt.p).all() and float((e.opt.p - p0).abs().max()) > 0
        assert m['count'] == 32 * 21 and m['loss_sum'] == m['loss_sum']
    finally:
        dist.destroy_process_group()

"""Host-dataset pipeline (data/host.py + csrc/loader.cpp + csrc/image.hip): the native prefetcher
delivers every sampled row exactly once per epoch in sampler order with reproducible flips, and
the on-device transform matches the torch implementation of Resize -> Flip -> ToTensor ->
Normalize (REF/data_and_toy_model.py:8-38). torchvision itself is not importable here: parity
with PIL's resize is unpinned (the kernel implements its upsampling filter + uint8 rounding)."""
import pytest
import torch

from tutorial_torch_distributed_data_parallel_amd.data import (CIFAR_MEAN, CIFAR_STD,
                                                                DistributedSampler,
                                                                HostImageDataset, ImageTransform,
                                                                PrefetchLoader, cifar_like_uint8)
from tutorial_torch_distributed_data_parallel_amd.data.host import reference_transform


def _ds(n=101, hw=8):
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (n, hw, hw, 3), generator=g, dtype=torch.uint8)
    return HostImageDataset(img, torch.arange(n))


@pytest.mark.parametrize("drop_last", [False, True])
def test_prefetcher_order_and_coverage_cpu(drop_last):
    ds = _ds()
    sampler = DistributedSampler(ds, num_replicas=1, rank=0, shuffle=True)
    tf = ImageTransform(size=8, flip_p=0.0, mean=(0, 0, 0), std=(1 / 255,) * 3, round_u8=True)
    loader = PrefetchLoader(ds, 16, sampler=sampler, drop_last=drop_last, transform=tf,
                            depth=3, threads=3)
    for epoch in range(3):
        sampler.set_epoch(epoch)
        order = list(sampler)
        seen = []
        for x, y in loader:
            seen += y.tolist()
            # identity transform at the source size: the gathered pixels come back unchanged
            torch.testing.assert_close(x, ds.images[y].permute(0, 3, 1, 2).float())
        want = order[: len(order) // 16 * 16] if drop_last else order
        assert seen == want
        assert len(seen) // 16 == len(loader) or not drop_last


def test_flip_bits_reproducible_and_epoch_dependent():
    ds = _ds(64, 4)
    tf = ImageTransform(size=4, flip_p=0.5, mean=(0, 0, 0), std=(1 / 255,) * 3)
    sampler = DistributedSampler(ds, num_replicas=1, rank=0, shuffle=False)

    def flips(epoch):
        sampler.set_epoch(epoch)
        loader = PrefetchLoader(ds, 8, sampler=sampler, transform=tf, seed=3)
        out = []
        for x, y in loader:
            ref = ds.images[y].permute(0, 3, 1, 2).float()
            out += [bool((x[i] - ref[i].flip(-1)).abs().max() < 1e-3 and
                         (x[i] - ref[i]).abs().max() > 1e-3) for i in range(len(y))]
        return out
    a, b, c = flips(0), flips(0), flips(1)
    assert a == b and a != c
    assert 16 < sum(a) < 48  # ~ half flipped


def test_cifar_like_uint8_shape():
    ds = cifar_like_uint8(n=50, seed=1)
    assert ds.images.shape == (50, 32, 32, 3) and ds.images.dtype == torch.uint8
    assert ds.labels.dtype == torch.int64


@pytest.mark.gpu
@pytest.mark.parametrize("channels_last", [True, False])
@pytest.mark.parametrize("round_u8", [True, False])
def test_image_transform_kernel_matches_torch(channels_last, round_u8):
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 256, (5, 32, 32, 3), generator=g, dtype=torch.uint8)
    flip = torch.tensor([0, 1, 1, 0, 1], dtype=torch.uint8)
    tf = ImageTransform(size=224, flip_p=0.5, round_u8=round_u8, channels_last=channels_last)
    out = tf(x.cuda(), flip.cuda())
    ref = reference_transform(x.cuda(), flip.cuda(), (224, 224), CIFAR_MEAN, CIFAR_STD, round_u8)
    assert out.is_contiguous(memory_format=torch.channels_last) == channels_last
    # rounding: the kernel's bilinear may land on the other side of .5 than torch's (fp32 order)
    atol = (1.0 / 255 / 0.199) if round_u8 else 1e-4
    torch.testing.assert_close(out, ref, atol=atol, rtol=0)
    if round_u8:
        assert (out - ref).abs().gt(1e-4).float().mean() < 1e-3


@pytest.mark.gpu
def test_prefetch_loader_gpu_trains():
    """A cifar_like uint8 host set through the native prefetcher into a small CNN on the GPU."""
    import tutorial_torch_distributed_data_parallel_amd as tdp

    ds = cifar_like_uint8(n=512, seed=0)
    loader = PrefetchLoader(ds, 64, transform=ImageTransform(size=64), device="cuda")
    torch.manual_seed(0)
    model = torch.nn.Sequential(tdp.nn.Conv2d(3, 16, 3, stride=2, padding=1, relu=True),
                                tdp.nn.AdaptiveAvgPool2d((1, 1)), torch.nn.Flatten(),
                                tdp.nn.Linear(16, 10)).cuda()
    opt = tdp.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    losses = []
    for epoch in range(3):
        for x, y in loader:
            assert x.is_cuda and x.shape == (len(y), 3, 64, 64)
            opt.zero_grad()
            loss = tdp.ops.cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            losses.append(float(loss))
    assert losses[-1] < losses[0]


def test_cifar10_binary_reader_roundtrip(tmp_path):
    """The CIFAR-10 binary record layout (label byte + R/G/B 32x32 planes) read by memmap into
    HostImageDataset, through PrefetchLoader + the transform, against reference_transform.
    A fixture in the real layout (no download here); parity with torchvision is unpinned."""
    from tutorial_torch_distributed_data_parallel_amd.data import (load_cifar10_bin,
                                                                    write_cifar10_bin)

    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    g = torch.Generator().manual_seed(5)
    parts = []
    for name in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        img = torch.randint(0, 256, (7, 32, 32, 3), generator=g, dtype=torch.uint8)
        lab = torch.randint(0, 10, (7,), generator=g)
        write_cifar10_bin(str(d / name), img, lab)
        parts.append((img, lab))
    # the on-disk bytes really are CHW planes after the label
    raw = (d / "data_batch_1.bin").read_bytes()
    assert len(raw) == 7 * 3073 and raw[0] == int(parts[0][1][0])
    assert raw[1] == int(parts[0][0][0, 0, 0, 0]) and raw[1 + 1024] == int(parts[0][0][0, 0, 0, 1])
    train = load_cifar10_bin(str(tmp_path), train=True)
    test = load_cifar10_bin(str(d), train=False)
    assert train.images.shape == (35, 32, 32, 3) and len(test) == 7
    assert torch.equal(train.images, torch.cat([p[0] for p in parts[:5]]))
    assert torch.equal(train.labels, torch.cat([p[1] for p in parts[:5]]))
    assert torch.equal(test.images, parts[5][0])
    tf = ImageTransform(size=64, flip_p=0.0)
    loader = PrefetchLoader(train, 8, transform=tf)
    for x, y in loader:
        # no sampler: the first batch is rows 0..7 in order
        assert torch.equal(y, train.labels[: len(y)])
        want = reference_transform(train.images[: len(y)], None, (64, 64), CIFAR_MEAN, CIFAR_STD)
        torch.testing.assert_close(x, want)
        break
    with pytest.raises(FileNotFoundError):
        load_cifar10_bin(str(tmp_path / "missing"))


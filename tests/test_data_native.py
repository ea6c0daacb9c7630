"""Native data pipeline: sample index, token ring loader, native collate."""
import numpy as np
import pytest

import paddle_ray_amd as paddle
from paddle_ray_amd.io import GPTDataset, NativeTokenLoader, write_token_dataset


def _ref_sample_idx(lens, doc_idx, seq, epochs, tpe):
    n = (epochs * tpe - 1) // seq
    out = np.zeros((n + 1, 2), dtype=np.int64)
    pos, off = 0, 0
    for s in range(1, n + 1):
        rem = seq + 1
        while rem:
            dl = lens[doc_idx[pos]] - off
            rem -= dl
            if rem <= 0:
                off += rem + dl - 1
                rem = 0
            else:
                pos += 1
                off = 0
        out[s] = (pos, off)
    return out


@pytest.fixture
def token_ds(tmp_path):
    rs = np.random.RandomState(0)
    docs = [rs.randint(0, 60000, rs.randint(3, 40)) for _ in range(50)]
    prefix = str(tmp_path / 'corpus')
    write_token_dataset(prefix, docs)
    return prefix, docs


def test_sample_idx_matches_reference(token_ds):
    prefix, docs = token_ds
    ds = GPTDataset(prefix, seq_len=16)
    tpe = int(ds.lens.sum())
    epochs = len(ds.doc_idx) // len(ds.lens)
    ref = _ref_sample_idx(ds.lens, ds.doc_idx, 16, epochs, tpe)
    np.testing.assert_array_equal(ds.sample_idx, ref)


def test_samples_are_contiguous_stream_windows(token_ds):
    prefix, docs = token_ds
    ds = GPTDataset(prefix, seq_len=16, seed=3)
    stream = np.concatenate([docs[d] for d in ds.doc_idx]).astype(np.int64)
    for i in range(10):
        s = int(ds.shuffle_idx[i])
        np.testing.assert_array_equal(ds[i], stream[s * 16: s * 16 + 17])


def test_native_loader_matches_dataset(token_ds):
    prefix, _ = token_ds
    ds = GPTDataset(prefix, seq_len=16, seed=5)
    loader = NativeTokenLoader(ds, batch_size=4, num_slots=3, num_threads=3, device='cpu')
    n = 0
    for b, (x, y) in enumerate(loader):
        ref = np.stack([ds[b * 4 + i] for i in range(4)])
        np.testing.assert_array_equal(x.numpy(), ref[:, :-1])
        np.testing.assert_array_equal(y.numpy(), ref[:, 1:])
        n += 1
    assert n == len(loader) == len(ds) // 4
    # resume from batch 2
    x, _ = next(iter(loader.resume_from(2)))
    np.testing.assert_array_equal(x.numpy(), np.stack([ds[8 + i] for i in range(4)])[:, :-1])


def test_native_loader_rank_sharding(token_ds):
    prefix, _ = token_ds
    ds = GPTDataset(prefix, seq_len=8, seed=1)
    a = [x.numpy() for x, _ in NativeTokenLoader(ds, 2, device='cpu', rank=0, world_size=2)]
    b = [x.numpy() for x, _ in NativeTokenLoader(ds, 2, device='cpu', rank=1, world_size=2)]
    assert len(a) == len(b)
    assert not np.array_equal(a[0], b[0])


def test_native_collate_large_batch():
    from paddle_ray_amd.io import default_collate_fn
    arrs = [np.random.rand(256, 1024).astype('float32') for _ in range(8)]  # 8 MB
    np.testing.assert_array_equal(default_collate_fn(arrs), np.stack(arrs))

"""paddle.audio (windows, mel filterbank, DCT, features, WAV I/O) and paddle.text (Viterbi,
file-based datasets) against independent numpy / brute-force references."""
import itertools
import math
import os

import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd.audio import functional as AF


def test_windows_match_scipy():
    import scipy.signal
    for w in ['hann', 'hamming', 'blackman', 'bohman', 'cosine', 'triang', ('tukey', 0.3),
              ('gaussian', 7.0), ('taylor', 4, 30)]:
        for fftbins in (True, False):
            ours = AF.get_window(w, 64, fftbins=fftbins).numpy()
            ref = scipy.signal.get_window(w, 64, fftbins=fftbins)
            np.testing.assert_allclose(ours, ref, rtol=1e-10, atol=1e-12)
    with pytest.raises(ValueError):
        AF.get_window('gaussian', 10)


def _np_mel(f, htk):
    f = np.asarray(f, np.float64)
    if htk:
        return 2595.0 * np.log10(1.0 + f / 700.0)
    lin = f / (200.0 / 3)
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-9) / 1000.0) / (np.log(6.4) / 27.0), lin)


def test_mel_scale_and_fbank():
    f = np.array([0.0, 300.0, 999.0, 1000.0, 4000.0, 8000.0])
    for htk in (False, True):
        np.testing.assert_allclose(AF.hz_to_mel(paddle.to_tensor(f), htk).numpy(),
                                   _np_mel(f, htk), rtol=1e-6)
        back = AF.mel_to_hz(AF.hz_to_mel(paddle.to_tensor(f), htk), htk).numpy()
        np.testing.assert_allclose(back, f, rtol=1e-6, atol=1e-6)
        assert abs(AF.hz_to_mel(440.0, htk) - float(_np_mel(440.0, htk))) < 1e-9
    sr, n_fft, n_mels = 16000, 512, 40
    fb = AF.compute_fbank_matrix(sr, n_fft, n_mels, f_min=0.0, dtype='float64').numpy()
    # independent reference: triangles between consecutive mel points, Slaney area norm
    mpts = np.linspace(_np_mel(0.0, False), _np_mel(sr / 2, False), n_mels + 2)
    hz = np.where(mpts >= 15.0, 1000.0 * np.exp((np.log(6.4) / 27.0) * (mpts - 15.0)),
                  mpts * 200.0 / 3)
    bins = np.linspace(0, sr / 2, n_fft // 2 + 1)
    ref = np.zeros((n_mels, bins.size))
    for m in range(n_mels):
        lo, c, hi = hz[m], hz[m + 1], hz[m + 2]
        up = (bins - lo) / (c - lo)
        down = (hi - bins) / (hi - c)
        ref[m] = np.maximum(0, np.minimum(up, down)) * 2.0 / (hi - lo)
    np.testing.assert_allclose(fb, ref, rtol=1e-6, atol=1e-9)


def test_dct_and_power_to_db():
    d = AF.create_dct(13, 40, dtype='float64').numpy()
    import scipy.fft
    ref = scipy.fft.dct(np.eye(40), type=2, norm='ortho')[:, :13]
    np.testing.assert_allclose(d, ref, rtol=1e-9, atol=1e-12)
    s = np.array([1e-12, 1e-3, 1.0, 100.0])
    db = AF.power_to_db(paddle.to_tensor(s), top_db=None).numpy()
    np.testing.assert_allclose(db, 10 * np.log10(np.maximum(s, 1e-10)), rtol=1e-6)
    db2 = AF.power_to_db(paddle.to_tensor(s), top_db=30.0).numpy()
    assert db2.min() >= 20.0 - 30.0 - 1e-6


def test_feature_layers_shapes_and_mfcc_consistency():
    from paddle_ray_amd.audio import features as F
    x = paddle.to_tensor(np.sin(np.linspace(0, 200 * np.pi, 8000)).astype(np.float32)[None])
    spec = F.Spectrogram(n_fft=256, hop_length=64, power=2.0)(x)
    assert spec.shape == [1, 129, 126]
    # peak bin at the tone frequency: 100 cycles over 8000 samples -> bin 100/8000*256 = 3.2
    assert int(spec.numpy()[0].mean(-1).argmax()) in (3, 4)
    lm = F.LogMelSpectrogram(sr=8000, n_fft=256, hop_length=64, n_mels=32, f_min=0.0)(x)
    mf = F.MFCC(sr=8000, n_mfcc=13, n_fft=256, hop_length=64, n_mels=32, f_min=0.0)(x)
    dct = AF.create_dct(13, 32).numpy()
    np.testing.assert_allclose(mf.numpy()[0], dct.T @ lm.numpy()[0], rtol=1e-4, atol=1e-3)


def test_wav_roundtrip(tmp_path):
    sr = 8000
    wav = (0.5 * np.sin(np.linspace(0, 20 * np.pi, 4000))).astype(np.float32)
    p = str(tmp_path / 'a.wav')
    paddle.audio.save(p, paddle.to_tensor(np.stack([wav, -wav])), sr)
    info = paddle.audio.info(p)
    assert (info.sample_rate, info.num_frames, info.num_channels, info.bits_per_sample) == \
        (sr, 4000, 2, 16)
    x, sr2 = paddle.audio.load(p)
    assert sr2 == sr and x.shape == [2, 4000]
    np.testing.assert_allclose(x.numpy()[0], wav, atol=1.0 / 16384)
    y, _ = paddle.audio.load(p, frame_offset=100, num_frames=50, normalize=False)
    assert y.shape == [2, 50] and y.numpy().dtype == np.int16
    assert paddle.audio.backends.get_current_backend() == 'wave_backend'


def _brute_viterbi(em, tr, n, bos):
    N = em.shape[-1]
    best, arg = -np.inf, None
    for seq in itertools.product(range(N), repeat=n):
        s = em[np.arange(n), list(seq)].sum() + sum(tr[seq[i - 1], seq[i]] for i in range(1, n))
        if bos:
            s += tr[N - 1, seq[0]] + tr[N - 2, seq[-1]]
        if s > best:
            best, arg = s, seq
    return best, arg


@pytest.mark.parametrize('bos', [False, True])
def test_viterbi_decode_brute_force(bos):
    rng = np.random.RandomState(3)
    B, L, N = 4, 5, 4
    em = rng.randn(B, L, N).astype(np.float64)
    tr = rng.randn(N, N).astype(np.float64)
    lens = np.array([5, 3, 1, 4], np.int64)
    scores, path = paddle.text.viterbi_decode(paddle.to_tensor(em), paddle.to_tensor(tr),
                                              paddle.to_tensor(lens), bos)
    assert path.shape == [B, 5]
    for b in range(B):
        ref_s, ref_p = _brute_viterbi(em[b], tr, lens[b], bos)
        assert abs(float(scores.numpy()[b]) - ref_s) < 1e-9
        assert list(path.numpy()[b][:lens[b]]) == list(ref_p)
        assert (path.numpy()[b][lens[b]:] == 0).all()
    dec = paddle.text.ViterbiDecoder(paddle.to_tensor(tr), bos)
    s2, p2 = dec(paddle.to_tensor(em), paddle.to_tensor(lens))
    np.testing.assert_allclose(s2.numpy(), scores.numpy())


def test_uci_housing_from_file(tmp_path):
    rng = np.random.RandomState(0)
    data = rng.rand(50, 14) * 10
    p = tmp_path / 'housing.data'
    np.savetxt(p, data)
    tr = paddle.text.UCIHousing(data_file=str(p), mode='train')
    te = paddle.text.UCIHousing(data_file=str(p), mode='test')
    assert len(tr) == 40 and len(te) == 10
    x, y = tr[0]
    assert x.shape == (13,) and y.shape == (1,)
    assert abs(float(y[0]) - data[0, 13]) < 1e-5
    with pytest.raises(ValueError):
        paddle.text.UCIHousing()


def test_imdb_from_tar(tmp_path):
    import io
    import tarfile
    p = str(tmp_path / 'aclImdb.tar.gz')
    docs = {'aclImdb/train/pos/0.txt': b'good good movie!', 'aclImdb/train/neg/0.txt':
            b'bad, bad movie.', 'aclImdb/test/pos/0.txt': b'good film'}
    with tarfile.open(p, 'w:gz') as tf:
        for name, body in docs.items():
            ti = tarfile.TarInfo(name)
            ti.size = len(body)
            tf.addfile(ti, io.BytesIO(body))
    ds = paddle.text.Imdb(data_file=p, mode='train', cutoff=0)
    assert len(ds) == 2
    doc, lab = ds[0]
    w = ds.word_idx
    assert list(doc) == [w[b'good'], w[b'good'], w[b'movie']] and int(lab[0]) == 0
    assert int(ds[1][1][0]) == 1

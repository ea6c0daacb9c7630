"""Audio classification datasets (parity: python/paddle/audio/datasets/{dataset,esc50,tess}.py).

No downloads exist in this environment: point ``data_dir`` at an extracted copy of the
corpus (the same directory layout the public archives unpack to)."""
import collections
import os

import numpy as np

from ...io import Dataset
from .. import backends, features

feat_funcs = {
    'raw': None,
    'melspectrogram': features.MelSpectrogram,
    'mfcc': features.MFCC,
    'logmelspectrogram': features.LogMelSpectrogram,
    'spectrogram': features.Spectrogram,
}


class AudioClassificationDataset(Dataset):
    """(waveform or feature, label) pairs from a list of wav files."""

    def __init__(self, files, labels, feat_type='raw', sample_rate=None, **kwargs):
        super().__init__()
        if feat_type not in feat_funcs:
            raise RuntimeError(f"Unknown feat_type: {feat_type}, it must be one in "
                               f"{list(feat_funcs.keys())}")
        self.files, self.labels = files, labels
        self.feat_type = feat_type
        self.sample_rate = sample_rate
        self.feat_config = kwargs

    def _convert_to_record(self, idx):
        import torch
        from ...framework.core import Tensor
        file, label = self.files[idx], self.labels[idx]
        waveform, sr = backends.load(file)
        w = waveform._t if hasattr(waveform, '_t') else torch.as_tensor(waveform)
        w = w[0] if w.dim() > 1 else w
        if self.sample_rate is None:
            self.sample_rate = sr
        fn = feat_funcs[self.feat_type]
        if fn is None:
            return w.numpy(), label
        f = fn(sr=sr, **self.feat_config) if self.feat_type != 'spectrogram' else \
            fn(**self.feat_config)
        return f(Tensor(w[None])).numpy()[0], label

    def __getitem__(self, idx):
        rec, label = self._convert_to_record(idx)
        return np.asarray(rec), np.array(label, dtype=np.int64)

    def __len__(self):
        return len(self.files)


class ESC50(AudioClassificationDataset):
    """ESC-50 (2000 clips, 50 classes, 5 folds). ``data_dir`` holds ``audio/`` and
    ``meta/esc50.csv``; ``split`` is the held-out fold for ``mode='dev'``."""

    meta_info = collections.namedtuple('META_INFO', ('filename', 'fold', 'target', 'category',
                                                     'esc10', 'src_file', 'take'))
    audio_path = 'audio'
    meta = os.path.join('meta', 'esc50.csv')

    def __init__(self, mode='train', split=1, feat_type='raw', data_dir=None, **kwargs):
        if data_dir is None:
            raise ValueError("ESC50: no download in this environment; pass data_dir")
        if mode not in ('train', 'dev'):
            raise ValueError("mode must be 'train' or 'dev'")
        files, labels = [], []
        with open(os.path.join(data_dir, self.meta)) as rf:
            for line in rf.readlines()[1:]:
                m = self.meta_info(*line.strip().split(','))
                fold, target = int(m.fold), int(m.target)
                if (mode == 'train' and fold != split) or (mode == 'dev' and fold == split):
                    files.append(os.path.join(data_dir, self.audio_path, m.filename))
                    labels.append(target)
        super().__init__(files, labels, feat_type, **kwargs)


class TESS(AudioClassificationDataset):
    """Toronto emotional speech set (7 emotions). ``data_dir`` holds the wav files
    named ``<speaker>_<word>_<emotion>.wav`` (any nesting)."""

    label_list = ['angry', 'disgust', 'fear', 'happy', 'neutral', 'ps', 'sad']

    def __init__(self, mode='train', n_folds=5, split=1, feat_type='raw', data_dir=None,
                 **kwargs):
        if data_dir is None:
            raise ValueError("TESS: no download in this environment; pass data_dir")
        if not (1 <= split <= n_folds):
            raise ValueError(f"split must be in [1, {n_folds}]")
        wavs = []
        for root, _, fs in os.walk(data_dir):
            wavs += [os.path.join(root, f) for f in fs if f.endswith('.wav')]
        wavs.sort()
        files, labels = [], []
        for i, f in enumerate(wavs):
            emotion = os.path.basename(f)[:-4].split('_')[-1].lower()
            if emotion not in self.label_list:
                continue
            fold = i % n_folds + 1
            if (mode == 'train' and fold != split) or (mode != 'train' and fold == split):
                files.append(f)
                labels.append(self.label_list.index(emotion))
        super().__init__(files, labels, feat_type, **kwargs)


__all__ = ['AudioClassificationDataset', 'ESC50', 'TESS']

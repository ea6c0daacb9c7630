"""Vision datasets (parity: python/paddle/vision/datasets/{mnist,cifar,flowers,voc2012,
folder}.py).

There is no network here, so nothing is downloaded: every dataset reads the reference's
on-disk formats from a path you pass (or from ``$PADDLE_DATA_HOME/<name>/``). MNIST /
FashionMNIST / Cifar10 / Cifar100 fall back to ``SyntheticImageDataset`` samples of the
same shapes when no file is available (used by the benches and CPU tests); Flowers and
VOC2012 require their files.
"""
import gzip
import os
import struct
import tarfile
import warnings

import numpy as np

from ...io import Dataset
from ._common import check_backend, decode_image, find_local, load_numpy_pickle, require


class SyntheticImageDataset(Dataset):
    def __init__(self, num_samples=1024, shape=(1, 28, 28), num_classes=10, seed=0,
                 transform=None):
        rng = np.random.RandomState(seed)
        self.images = rng.rand(num_samples, *shape).astype(np.float32)
        self.labels = rng.randint(0, num_classes, (num_samples, 1)).astype(np.int64)
        self.transform = transform

    def __getitem__(self, i):
        img = self.images[i]
        if self.transform is not None:
            img = self.transform(img)
        return img, self.labels[i]

    def __len__(self):
        return len(self.images)


def _open_maybe_gz(path):
    with open(path, 'rb') as f:
        head = f.read(2)
    return gzip.open(path, 'rb') if head == b'\x1f\x8b' else open(path, 'rb')


def _read_idx(path):
    """IDX (MNIST) file -> uint8 ndarray of its declared shape."""
    with _open_maybe_gz(path) as f:
        buf = f.read()
    magic = struct.unpack_from('>I', buf, 0)[0]
    ndim = magic & 0xff
    dims = struct.unpack_from('>' + 'I' * ndim, buf, 4)
    return np.frombuffer(buf, np.uint8, offset=4 + 4 * ndim).reshape(dims)


class MNIST(Dataset):
    """MNIST from the IDX files (gzip or raw): items are (image, label[1] int64); image is a
    [28, 28] float32 array ('cv2' backend) or a PIL image ('pil'), before ``transform``."""

    NAME = 'mnist'
    FILES = {'train': ('train-images-idx3-ubyte.gz', 'train-labels-idx1-ubyte.gz'),
             'test': ('t10k-images-idx3-ubyte.gz', 't10k-labels-idx1-ubyte.gz')}

    def __init__(self, image_path=None, label_path=None, mode='train', transform=None,
                 download=True, backend=None):
        mode = mode.lower()
        if mode not in ('train', 'test'):
            raise ValueError(f"mode should be 'train' or 'test', but got {mode}")
        self.mode, self.transform = mode, transform
        self.backend = check_backend(backend)
        image_path = image_path or find_local(self.NAME, self.FILES[mode][0])
        label_path = label_path or find_local(self.NAME, self.FILES[mode][1])
        self.synthetic = image_path is None or label_path is None
        if self.synthetic:
            warnings.warn(f"{type(self).__name__}: no local IDX files (no network to download "
                          f"them); using synthetic samples of the same shape")
            n = 60000 if mode == 'train' else 10000
            self._syn = SyntheticImageDataset(n, (1, 28, 28), 10, 0 if mode == 'train' else 1,
                                              transform)
            return
        self.images = _read_idx(image_path)
        self.labels = _read_idx(label_path).astype(np.int64).reshape(-1, 1)
        if len(self.images) != len(self.labels):
            raise ValueError("image / label count mismatch")

    def __getitem__(self, idx):
        if self.synthetic:
            return self._syn[idx]
        image = self.images[idx]
        if self.backend == 'pil':
            from PIL import Image
            image = Image.fromarray(image, mode='L')
        else:
            image = image.astype(np.float32)
        if self.transform is not None:
            image = self.transform(image)
        return image, self.labels[idx]

    def __len__(self):
        return len(self._syn) if self.synthetic else len(self.labels)


class FashionMNIST(MNIST):
    NAME = 'fashion-mnist'


class Cifar10(Dataset):
    """CIFAR-10 from the python-version tar.gz (batches decoded with a numpy-only
    unpickler): items are (HWC uint8-valued image, label int64)."""

    NAME, ARCHIVE, NUM_CLASSES = 'cifar', 'cifar-10-python.tar.gz', 10
    FLAGS = {'train': 'data_batch', 'test': 'test_batch'}

    def __init__(self, data_file=None, mode='train', transform=None, download=True,
                 backend=None):
        mode = mode.lower()
        if mode not in ('train', 'test'):
            raise ValueError(f"mode should be 'train' or 'test', but got {mode}")
        self.mode, self.transform = mode, transform
        self.backend = check_backend(backend)
        data_file = data_file or find_local(self.NAME, self.ARCHIVE)
        self.synthetic = data_file is None
        if self.synthetic:
            warnings.warn(f"{type(self).__name__}: no local archive (no network to download "
                          f"it); using synthetic samples of the same shape")
            self._syn = SyntheticImageDataset(50000 if mode == 'train' else 10000, (3, 32, 32),
                                              self.NUM_CLASSES, 0 if mode == 'train' else 1,
                                              transform)
            return
        flag = self.FLAGS[mode]
        data, labels = [], []
        with tarfile.open(data_file, mode='r') as tf:
            names = sorted(m.name for m in tf.getmembers()
                           if m.isfile() and os.path.basename(m.name).startswith(flag))
            for name in names:
                batch = load_numpy_pickle(tf.extractfile(name))
                data.append(np.asarray(batch[b'data'], np.uint8))
                lab = batch.get(b'labels', batch.get(b'fine_labels'))
                labels.append(np.asarray(lab, np.int64))
        self.data = np.concatenate(data).reshape(-1, 3, 32, 32)
        self.labels = np.concatenate(labels)

    def __getitem__(self, idx):
        if self.synthetic:
            return self._syn[idx]
        image = self.data[idx].transpose(1, 2, 0)
        if self.backend == 'pil':
            from PIL import Image
            image = Image.fromarray(image)
        if self.transform is not None:
            image = self.transform(image)
        if self.backend != 'pil' and isinstance(image, np.ndarray):
            image = image.astype(np.float32)
        return image, np.array(self.labels[idx], np.int64)

    def __len__(self):
        return len(self._syn) if self.synthetic else len(self.labels)


class Cifar100(Cifar10):
    NAME, ARCHIVE, NUM_CLASSES = 'cifar', 'cifar-100-python.tar.gz', 100
    FLAGS = {'train': 'train', 'test': 'test'}


class Flowers(Dataset):
    """Oxford 102 Flowers: the image tgz (jpg/image_%05d.jpg) + imagelabels.mat +
    setid.mat (read with scipy.io.loadmat). mode train/test/valid -> tstid/trnid/valid as
    in the reference."""

    MODE_FLAG = {'train': 'tstid', 'test': 'trnid', 'valid': 'valid'}

    def __init__(self, data_file=None, label_file=None, setid_file=None, mode='train',
                 transform=None, download=True, backend=None):
        import scipy.io as scio
        mode = mode.lower()
        if mode not in self.MODE_FLAG:
            raise ValueError(f"mode should be one of {list(self.MODE_FLAG)}, got {mode}")
        self.transform, self.backend = transform, check_backend(backend)
        data_file = require(data_file or find_local('flowers', '102flowers.tgz'), 'Flowers',
                            download)
        label_file = require(label_file or find_local('flowers', 'imagelabels.mat'),
                             'Flowers labels', download)
        setid_file = require(setid_file or find_local('flowers', 'setid.mat'),
                             'Flowers setid', download)
        self.labels = scio.loadmat(label_file)['labels'][0]
        self.indexes = scio.loadmat(setid_file)[self.MODE_FLAG[mode]][0]
        self._tar = tarfile.open(data_file)
        self._members = {m.name: m for m in self._tar.getmembers() if m.isfile()}

    def __getitem__(self, idx):
        index = int(self.indexes[idx])
        name = 'jpg/image_%05d.jpg' % index
        raw = self._tar.extractfile(self._members[name]).read()
        image = decode_image(raw, self.backend)
        if self.transform is not None:
            image = self.transform(image)
        label = np.array([self.labels[index - 1]], np.int64)
        if self.backend != 'pil' and isinstance(image, np.ndarray):
            image = image.astype(np.float32)
        return image, label

    def __len__(self):
        return len(self.indexes)


class VOC2012(Dataset):
    """VOC2012 segmentation pairs from VOCtrainval_11-May-2012.tar: (image, label mask);
    mode train/test/valid -> trainval/train/val split lists as in the reference."""

    MODE_FLAG = {'train': 'trainval', 'test': 'train', 'valid': 'val'}
    ROOT = 'VOCdevkit/VOC2012/'

    def __init__(self, data_file=None, mode='train', transform=None, download=True,
                 backend=None):
        mode = mode.lower()
        if mode not in self.MODE_FLAG:
            raise ValueError(f"mode should be one of {list(self.MODE_FLAG)}, got {mode}")
        self.transform, self.backend = transform, check_backend(backend)
        data_file = require(data_file or find_local('voc2012', 'VOCtrainval_11-May-2012.tar'),
                            'VOC2012', download)
        self._tar = tarfile.open(data_file)
        self._members = {m.name: m for m in self._tar.getmembers() if m.isfile()}
        lst = self.ROOT + f'ImageSets/Segmentation/{self.MODE_FLAG[mode]}.txt'
        names = self._tar.extractfile(self._members[lst]).read().decode().split()
        self.names = [n.strip() for n in names if n.strip()]

    def __getitem__(self, idx):
        n = self.names[idx]
        img = self._tar.extractfile(self._members[self.ROOT + f'JPEGImages/{n}.jpg']).read()
        lab = self._tar.extractfile(self._members[self.ROOT + f'SegmentationClass/{n}.png'])
        image = decode_image(img, self.backend)
        label = decode_image(lab.read(), 'pil', mode=None)
        if self.backend != 'pil':
            label = np.asarray(label)
        if self.transform is not None:
            image = self.transform(image)
        if self.backend != 'pil':
            return np.asarray(image).astype(np.float32), label.astype(np.float32)
        return image, label

    def __len__(self):
        return len(self.names)


IMG_EXTENSIONS = ('.jpg', '.jpeg', '.png', '.ppm', '.bmp', '.pgm', '.tif', '.tiff', '.webp')


def has_valid_extension(filename, extensions):
    return filename.lower().endswith(tuple(extensions))


def pil_loader(path):
    from PIL import Image
    with open(path, 'rb') as f:
        return Image.open(f).convert('RGB')


def cv2_loader(path):
    """RGB HWC uint8 array (the reference's cv2 loader converts BGR -> RGB)."""
    return np.asarray(pil_loader(path))


def default_loader(path):
    from .. import get_image_backend
    return cv2_loader(path) if get_image_backend() == 'cv2' else pil_loader(path)


class DatasetFolder(Dataset):
    """root/class_x/xxx.ext -> (sample, class_index); classes sorted by name."""

    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root, self.transform = root, transform
        self.loader = loader or default_loader
        if extensions is None and is_valid_file is None:
            extensions = IMG_EXTENSIONS
        if extensions is not None and is_valid_file is not None:
            raise ValueError("extensions and is_valid_file cannot both be passed")
        valid = is_valid_file or (lambda p: has_valid_extension(p, extensions))
        self.classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        self.samples = []
        for c in self.classes:
            for dirpath, _, files in sorted(os.walk(os.path.join(root, c), followlinks=True)):
                for fn in sorted(files):
                    p = os.path.join(dirpath, fn)
                    if valid(p):
                        self.samples.append((p, self.class_to_idx[c]))
        if not self.samples:
            raise RuntimeError(f"Found 0 files in subfolders of: {root}")
        self.targets = [s[1] for s in self.samples]

    def __getitem__(self, index):
        path, target = self.samples[index]
        sample = self.loader(path)
        if self.transform is not None:
            sample = self.transform(sample)
        return sample, target

    def __len__(self):
        return len(self.samples)


class ImageFolder(Dataset):
    """Every image file under ``root`` (recursively, no labels) -> [sample]."""

    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root, self.transform = root, transform
        self.loader = loader or default_loader
        if extensions is None and is_valid_file is None:
            extensions = IMG_EXTENSIONS
        valid = is_valid_file or (lambda p: has_valid_extension(p, extensions))
        self.samples = []
        for dirpath, _, files in sorted(os.walk(root, followlinks=True)):
            for fn in sorted(files):
                p = os.path.join(dirpath, fn)
                if valid(p):
                    self.samples.append(p)
        if not self.samples:
            raise RuntimeError(f"Found 0 files in: {root}")

    def __getitem__(self, index):
        sample = self.loader(self.samples[index])
        if self.transform is not None:
            sample = self.transform(sample)
        return [sample]

    def __len__(self):
        return len(self.samples)

"""Vision datasets. No network here: MNIST/Cifar read local files when present,
else ``Synthetic*`` datasets of the same shapes are used (documented)."""
import numpy as np

from ...io import Dataset


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


class MNIST(SyntheticImageDataset):
    def __init__(self, image_path=None, label_path=None, mode='train', transform=None,
                 download=False, backend=None):
        super().__init__(60000 if mode == 'train' else 10000, (1, 28, 28), 10,
                         0 if mode == 'train' else 1, transform)


FashionMNIST = MNIST


class Cifar10(SyntheticImageDataset):
    def __init__(self, data_file=None, mode='train', transform=None, download=False,
                 backend=None):
        super().__init__(50000 if mode == 'train' else 10000, (3, 32, 32), 10,
                         0 if mode == 'train' else 1, transform)


class Cifar100(SyntheticImageDataset):
    def __init__(self, data_file=None, mode='train', transform=None, download=False,
                 backend=None):
        super().__init__(50000 if mode == 'train' else 10000, (3, 32, 32), 100,
                         0 if mode == 'train' else 1, transform)

"""Legacy dataset helpers (parity: python/paddle/dataset/common.py). No network: download()
only resolves files already under DATA_HOME."""
import glob
import hashlib
import os
import pickle

from ..vision.datasets._common import DATA_HOME

__all__ = []


def must_mkdirs(path):
    os.makedirs(path, exist_ok=True)


def md5file(fname):
    h = hashlib.md5()
    with open(fname, 'rb') as f:
        for chunk in iter(lambda: f.read(4096), b''):
            h.update(chunk)
    return h.hexdigest()


def download(url, module_name, md5sum, save_name=None):
    """Return the local copy ``DATA_HOME/module_name/<file>`` (checked against md5sum when
    given); there is no network, so a missing file is an error."""
    d = os.path.join(DATA_HOME, module_name)
    fn = os.path.join(d, save_name or url.split('/')[-1])
    if not os.path.exists(fn):
        raise RuntimeError(f"{fn} is not available locally and this environment cannot "
                           f"download {url}")
    if md5sum and md5file(fn) != md5sum:
        raise RuntimeError(f"md5 mismatch for {fn}")
    return fn


def fetch_all():
    raise RuntimeError("fetch_all needs network access, which this environment does not have")


def split(reader, line_count, suffix="%05d.pickle", dumper=pickle.dump):
    """Write the reader's samples into files of ``line_count`` samples each."""
    if not callable(dumper):
        raise TypeError("dumper should be callable.")
    buf, idx = [], 0
    for d in reader():
        buf.append(d)
        if len(buf) == line_count:
            with open(suffix % idx, 'wb') as f:
                dumper(buf, f)
            buf, idx = [], idx + 1
    if buf:
        with open(suffix % idx, 'wb') as f:
            dumper(buf, f)


def cluster_files_reader(files_pattern, trainer_count, trainer_id, loader=pickle.load):
    """Reader over the files (of ``split``) assigned round-robin to this trainer. The
    default loader unpickles: only use it on files you wrote yourself."""
    def reader():
        if not callable(loader):
            raise TypeError("loader should be callable.")
        files = sorted(glob.glob(files_pattern))
        for i, fn in enumerate(files):
            if i % trainer_count == trainer_id:
                with open(fn, 'rb') as f:
                    yield from loader(f)
    return reader


def _check_exists_and_download(path, url, md5, module_name, download_flag=True):
    if path and os.path.exists(path):
        return path
    if download_flag:
        return download(url, module_name, md5)
    raise ValueError(f'{path} not exists and auto download disabled')

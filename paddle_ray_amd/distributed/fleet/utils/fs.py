"""File-system clients (parity: python/paddle/distributed/fleet/utils/fs.py)."""
import os
import shutil


class LocalFS:
    def ls_dir(self, fs_path):
        if not os.path.exists(fs_path):
            return [], []
        dirs, files = [], []
        for f in os.listdir(fs_path):
            (dirs if os.path.isdir(os.path.join(fs_path, f)) else files).append(f)
        return dirs, files

    def mkdirs(self, fs_path):
        os.makedirs(fs_path, exist_ok=True)

    def delete(self, fs_path):
        if os.path.isdir(fs_path):
            shutil.rmtree(fs_path)
        elif os.path.exists(fs_path):
            os.remove(fs_path)

    def is_exist(self, fs_path):
        return os.path.exists(fs_path)

    def is_file(self, fs_path):
        return os.path.isfile(fs_path)

    def is_dir(self, fs_path):
        return os.path.isdir(fs_path)

    def rename(self, a, b):
        os.rename(a, b)

    def mv(self, a, b, overwrite=False):
        if overwrite and os.path.exists(b):
            self.delete(b)
        shutil.move(a, b)

    def touch(self, fs_path, exist_ok=True):
        open(fs_path, 'a').close()

    def list_dirs(self, fs_path):
        return self.ls_dir(fs_path)[0]

    def upload(self, local, remote):
        shutil.copy(local, remote)

    def download(self, remote, local):
        shutil.copy(remote, local)


class HDFSClient(LocalFS):
    def __init__(self, hadoop_home=None, configs=None, *a, **k):
        raise RuntimeError("HDFS is not reachable from this environment")

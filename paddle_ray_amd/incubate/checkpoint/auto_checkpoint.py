"""Auto checkpoint / resume by epoch range (parity: python/paddle/fluid/incubate/checkpoint/
auto_checkpoint.py, exported as paddle.incubate.checkpoint.auto_checkpoint).

The reference saves executor state to HDFS under an EDL job. Here checkpoints go to a
(shared) filesystem directory: ``PADDLE_CHECKPOINT_PATH`` (or
``PADDLE_EDL_HDFS_CHECKPOINT_PATH`` used as a path) / ``PADDLE_JOB_ID`` / range name.
Objects with state_dict/set_state_dict (layers, optimizers, LR schedulers, GradScaler)
are registered with ``register``; ``train_epoch_range`` yields the remaining epochs,
restores the registered state when a previous run of the same job left a checkpoint, and
saves after an epoch once ``save_checkpoint_inter`` seconds have passed since the last
save (and after the final epoch). Writes are atomic (temp dir + rename); rank 0 writes.
"""
import json
import os
import shutil
import time

_registered = {}
_current = [None]


def register(name, obj):
    """Include ``obj`` (has state_dict / set_state_dict) in every auto checkpoint."""
    if not (hasattr(obj, 'state_dict') and hasattr(obj, 'set_state_dict')):
        raise TypeError("registered objects need state_dict() and set_state_dict()")
    _registered[name] = obj


def unregister(name=None):
    if name is None:
        _registered.clear()
    else:
        _registered.pop(name, None)


class AutoCheckpointChecker:
    def __init__(self):
        env = os.environ
        self._job_id = env.get('PADDLE_JOB_ID')
        self._path = env.get('PADDLE_CHECKPOINT_PATH') or env.get('PADDLE_EDL_HDFS_CHECKPOINT_PATH')
        self._trainer_id = int(env.get('PADDLE_TRAINER_ID', env.get('RANK', '0')))
        self._inter = int(env.get('PADDLE_EDL_SAVE_CHECKPOINT_INTER', '900'))

    def valid(self):
        return bool(self._job_id and self._path)

    @property
    def trainer_id(self):
        return self._trainer_id

    @property
    def job_id(self):
        return self._job_id

    def save_checkpoint_inter(self):
        return self._inter

    def get_range_checkpoint_path(self, name):
        return os.path.join(self._path, self._job_id, name)

    def __str__(self):
        return f"AutoCheckpointChecker(job={self._job_id}, path={self._path}, " \
               f"trainer={self._trainer_id}, inter={self._inter}s)"


class TrainEpochRange:
    def __init__(self, max_epoch_num, name, checkpoint_inter=None, checker=None):
        self._max = int(max_epoch_num)
        self.name = name
        self._checker = checker or AutoCheckpointChecker()
        self._inter = checkpoint_inter if checkpoint_inter is not None \
            else self._checker.save_checkpoint_inter()
        self._epoch_no = -1  # last finished epoch
        self._last_save = time.time()
        self._restored_from = None
        self._dir = self._checker.get_range_checkpoint_path(name) if self._checker.valid() \
            else None
        if self._dir:
            self._restore()

    @property
    def restored_from(self):
        return self._restored_from

    def _status_file(self):
        return os.path.join(self._dir, 'status.json')

    def _restore(self):
        if not os.path.exists(self._status_file()):
            return
        with open(self._status_file()) as f:
            st = json.load(f)
        ck = os.path.join(self._dir, st['checkpoint'])
        from ...framework.io import load
        for name, obj in _registered.items():
            p = os.path.join(ck, name + '.pdstate')
            if os.path.exists(p):
                obj.set_state_dict(load(p))
        self._epoch_no = int(st['epoch_no'])
        self._restored_from = ck

    def save_checkpoint(self):
        if not self._dir or self._checker.trainer_id != 0:
            return
        from ...framework.io import save
        os.makedirs(self._dir, exist_ok=True)
        tag = f'epoch_{self._epoch_no}'
        tmp = os.path.join(self._dir, f'.{tag}.tmp')
        shutil.rmtree(tmp, ignore_errors=True)
        os.makedirs(tmp)
        for name, obj in _registered.items():
            save(obj.state_dict(), os.path.join(tmp, name + '.pdstate'))
        final = os.path.join(self._dir, tag)
        shutil.rmtree(final, ignore_errors=True)
        os.replace(tmp, final)
        st_tmp = self._status_file() + '.tmp'
        with open(st_tmp, 'w') as f:
            json.dump({'epoch_no': self._epoch_no, 'checkpoint': tag, 'time': time.time(),
                       'max_epoch_num': self._max}, f)
        os.replace(st_tmp, self._status_file())
        for d in os.listdir(self._dir):  # keep only the newest checkpoint
            if d.startswith('epoch_') and d != tag:
                shutil.rmtree(os.path.join(self._dir, d), ignore_errors=True)
        self._last_save = time.time()

    def get(self):
        return self._epoch_no

    def next(self):
        for e in range(self._epoch_no + 1, self._max):
            yield e
            self._epoch_no = e
            last = e == self._max - 1
            if self._dir and (last or time.time() - self._last_save >= self._inter):
                self.save_checkpoint()


def _get_train_epoch_range():
    return _current[0]


def train_epoch_range(max_epoch_num, save_checkpoint_inter=None):
    """for epoch in train_epoch_range(N): ... -- resumes after a restart of the same job."""
    checker = AutoCheckpointChecker()
    if not checker.valid():
        yield from range(max_epoch_num)
        return
    r = TrainEpochRange(max_epoch_num, 'train_epoch_range', save_checkpoint_inter, checker)
    _current[0] = r
    try:
        yield from r.next()
    finally:
        _current[0] = None

"""paddle.distributed.io (parity: python/paddle/distributed/io.py): persistables save/load."""
import os

from ..framework.io import save as _save, load as _load


def save_persistables(executor, dirname, main_program=None, filename=None):
    from ..static import default_main_program
    prog = main_program or default_main_program()
    os.makedirs(dirname, exist_ok=True)
    _save(prog.state_dict(), os.path.join(dirname, filename or 'persistables.pdparams'))


def load_persistables(executor, dirname, main_program=None, filename=None):
    from ..static import default_main_program
    prog = main_program or default_main_program()
    prog.set_state_dict(_load(os.path.join(dirname, filename or 'persistables.pdparams')))


def is_persistable(var):
    return getattr(var, 'persistable', False)

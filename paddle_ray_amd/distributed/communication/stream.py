"""paddle.distributed.communication.stream (parity: python/paddle/distributed/communication/
stream/*.py): collectives with ``use_calc_stream``.

On MI355X the RCCL kernels run on the process group's own stream. ``use_calc_stream=True`` asks
for the result to be ordered on the CALCULATION stream as if the collective ran there: the op is
issued synchronously (the current stream waits on the RCCL stream -- a device-side dependency,
no host block) and returns no task. ``use_calc_stream=False`` with ``sync_op=False`` returns the
task to ``wait()`` on."""
from .. import collective as C
from ..collective import ReduceOp

__all__ = ['all_gather', 'all_reduce', 'alltoall', 'alltoall_single', 'broadcast', 'reduce', 'reduce_scatter',
           'recv', 'scatter', 'send']


def _check(sync_op, use_calc_stream):
    if use_calc_stream and not sync_op:
        raise RuntimeError("use_calc_stream can only be true in sync op behavior.")
    return sync_op or use_calc_stream


def _ret(task, use_calc_stream):
    return None if use_calc_stream else task


def all_reduce(tensor, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    return _ret(C.all_reduce(tensor, op, group, _check(sync_op, use_calc_stream)), use_calc_stream)


def all_gather(tensor_or_tensor_list, tensor, group=None, sync_op=True, use_calc_stream=False):
    return _ret(C.all_gather(tensor_or_tensor_list, tensor, group, _check(sync_op, use_calc_stream)),
                use_calc_stream)


def alltoall(out_tensor_or_tensor_list, in_tensor_or_tensor_list, group=None, sync_op=True, use_calc_stream=False):
    # (stream.alltoall takes the output first, unlike distributed.alltoall)
    return _ret(C.alltoall(in_tensor_or_tensor_list, out_tensor_or_tensor_list, group,
                           _check(sync_op, use_calc_stream)), use_calc_stream)


def alltoall_single(out_tensor, in_tensor, out_split_sizes=None, in_split_sizes=None, group=None, sync_op=True,
                    use_calc_stream=False):
    return _ret(C.alltoall_single(in_tensor, out_tensor, in_split_sizes, out_split_sizes, group,
                                  _check(sync_op, use_calc_stream)), use_calc_stream)


def broadcast(tensor, src=0, group=None, sync_op=True, use_calc_stream=False):
    return _ret(C.broadcast(tensor, src, group, _check(sync_op, use_calc_stream)), use_calc_stream)


def reduce(tensor, dst=0, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    return _ret(C.reduce(tensor, dst, op, group, _check(sync_op, use_calc_stream)), use_calc_stream)


def reduce_scatter(tensor, tensor_or_tensor_list, op=ReduceOp.SUM, group=None, sync_op=True,
                   use_calc_stream=False):
    return _ret(C.reduce_scatter(tensor, tensor_or_tensor_list, op, group, _check(sync_op, use_calc_stream)),
                use_calc_stream)


def scatter(tensor, tensor_or_tensor_list=None, src=0, group=None, sync_op=True, use_calc_stream=False):
    return _ret(C.scatter(tensor, tensor_or_tensor_list, src, group, _check(sync_op, use_calc_stream)),
                use_calc_stream)


def send(tensor, dst=0, group=None, sync_op=True, use_calc_stream=False):
    return _ret(C.send(tensor, dst, group, _check(sync_op, use_calc_stream)), use_calc_stream)


def recv(tensor, src=0, group=None, sync_op=True, use_calc_stream=False):
    return _ret(C.recv(tensor, src, group, _check(sync_op, use_calc_stream)), use_calc_stream)

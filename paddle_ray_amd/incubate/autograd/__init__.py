from ...autograd import jacobian as Jacobian, hessian as Hessian  # noqa


def enable_prim():
    pass


def disable_prim():
    pass


def prim_enabled():
    return False

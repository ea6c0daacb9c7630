"""paddle.device.xpu: there is no XPU on an MI355X build; ``synchronize`` says so."""

__all__ = ['synchronize']


def synchronize(device=None):
    raise RuntimeError("paddle.device.xpu.synchronize: no XPU device in the MI355X build")

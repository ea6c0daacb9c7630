"""Times the channels-last max pool forward / backward at ResNet-50's stem-pool shape
(bs 256, 112x112x64 bf16, 3x3 / s2 / p1) and checks them against torch's fp32 pool."""
import torch
from paddle_ray_amd.ops import fused


def main():
    torch.manual_seed(0)
    x = torch.randn(256, 112, 112, 64, device='cuda', dtype=torch.bfloat16).requires_grad_()
    y = fused.max_pool2d_nhwc(x, (3, 3), (2, 2), (1, 1))
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    yr = torch.nn.functional.max_pool2d(xr, 3, 2, 1)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    print('fwd err', float((y.float().permute(0, 3, 1, 2) - yr).abs().max()),
          'bwd err', float((x.grad.float().permute(0, 3, 1, 2) - xr.grad).abs().max()))
    x.grad = None
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for it in range(3):
        ev[0].record()
        for _ in range(20):
            y = fused.max_pool2d_nhwc(x, (3, 3), (2, 2), (1, 1))
        ev[1].record()
        for _ in range(20):
            torch.autograd.grad(y, x, dy, retain_graph=True)
        ev[2].record()
        torch.cuda.synchronize()
        print(f'fwd {ev[0].elapsed_time(ev[1]) / 20 * 1e3:.1f} us  bwd {ev[1].elapsed_time(ev[2]) / 20 * 1e3:.1f} us')


if __name__ == '__main__':
    main()

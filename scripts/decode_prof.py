"""Decode-step kernel profile: 24x2048 FusedMultiTransformer, batch 8, ctx 1024, eager steps
(for rocprofv3 --kernel-trace --stats). usage: python -m scripts.decode_prof [graph]"""
import sys

import torch


def main():
    import paddle_ray_amd as paddle
    from paddle_ray_amd.incubate.nn import FusedMultiTransformer, FusedMultiTransformerDecoder
    paddle.set_device('gpu')
    E, H, L, B, ctx = 2048, 16, 24, 8, 1024
    m = FusedMultiTransformer(E, H, 4 * E, num_layers=L)
    m.eval()
    m.to(dtype='bfloat16')
    dec = FusedMultiTransformerDecoder(m, B, ctx + 64, use_graph=len(sys.argv) > 1)
    dec.t.fill_(ctx)
    xt = torch.randn(B, 1, E, device='cuda', dtype=torch.bfloat16)
    for _ in range(10):
        dec.step(xt)
        dec.t.fill_(ctx)
    torch.cuda.synchronize()
    print('done')


if __name__ == '__main__':
    main()

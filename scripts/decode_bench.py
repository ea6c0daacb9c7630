"""Decode-attention bandwidth: the HIP split-K kernel (K.mmha_decode) vs torch SDPA over
the same KV cache, and end-to-end FusedMultiTransformer decode steps/s.

usage: python scripts/decode_bench.py [--quick]"""
import argparse
import json
import math
import time

import torch


def bench(fn, iters=50, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--quick', action='store_true')
    a = ap.parse_args()
    from paddle_ray_amd.ops import fused as K
    rows = []
    shapes = [(1, 32, 128, 4095), (8, 32, 128, 4095), (32, 16, 128, 2047), (64, 32, 128, 1023),
              (8, 16, 64, 8191)]
    if a.quick:
        shapes = shapes[:2]
    for B, H, D, t in shapes:
        L = t + 1
        qkv = torch.randn(B, 3, H, D, device='cuda', dtype=torch.bfloat16)
        cache = torch.randn(2, B, H, L, D, device='cuda', dtype=torch.bfloat16)
        hip = bench(lambda: K.mmha_decode(qkv, cache, t))
        q = qkv[:, 0].unsqueeze(2)                                 # [B, H, 1, D]

        def sdpa():
            cache[0, :, :, t] = qkv[:, 1]
            cache[1, :, :, t] = qkv[:, 2]
            return torch.nn.functional.scaled_dot_product_attention(q, cache[0], cache[1])
        ref = bench(sdpa)
        gb = 2 * B * H * (t + 1) * D * 2 / 1e9
        rows.append(dict(B=B, H=H, D=D, ctx=t + 1, hip_us=round(hip * 1e6, 1),
                         sdpa_us=round(ref * 1e6, 1), hip_TBps=round(gb / hip / 1e3, 2),
                         sdpa_TBps=round(gb / ref / 1e3, 2), splits=K._native.lib().mmha_splits(B, H, t)))
        print(json.dumps(rows[-1]), flush=True)
    # end-to-end decode: 24-layer 2048-wide model (GPT-3 1.3B shape), batch 8
    import paddle_ray_amd as paddle
    from paddle_ray_amd.incubate.nn import FusedMultiTransformer
    paddle.set_device('gpu')
    E, H, L, B, ctx = 2048, 16, (4 if a.quick else 24), 8, 1024
    m = FusedMultiTransformer(E, H, 4 * E, num_layers=L)
    m.eval()
    m.to(dtype='bfloat16')
    caches = [paddle.Tensor(torch.zeros(2, B, H, ctx + 64, E // H, device='cuda',
                                        dtype=torch.bfloat16)) for _ in range(L)]
    x = paddle.Tensor(torch.randn(B, 1, E, device='cuda', dtype=torch.bfloat16))
    step = [ctx]

    def one():
        with paddle.no_grad():
            m(x, caches=caches, time_step=step[0])
    dt = bench(one, iters=20, warmup=3)
    print(json.dumps(dict(model=f'{L}x{E} FusedMultiTransformer decode', batch=B, ctx=ctx,
                          ms_per_token_step=round(dt * 1e3, 3),
                          tokens_per_s=round(B / dt, 1))), flush=True)
    # the same step replayed from one captured HIP graph (device-side position counter)
    from paddle_ray_amd.incubate.nn import FusedMultiTransformerDecoder
    dec = FusedMultiTransformerDecoder(m, B, ctx + 256)
    dec.t.fill_(ctx)
    xt = torch.randn(B, 1, E, device='cuda', dtype=torch.bfloat16)

    def gstep():
        dec.step(xt)
        dec.t.fill_(ctx)  # keep the context length fixed for the measurement
    dg = bench(gstep, iters=50, warmup=3)
    print(json.dumps(dict(model=f'{L}x{E} FusedMultiTransformerDecoder (HIP graph)', batch=B,
                          ctx=ctx, ms_per_token_step=round(dg * 1e3, 3),
                          tokens_per_s=round(B / dg, 1))), flush=True)


if __name__ == '__main__':
    main()

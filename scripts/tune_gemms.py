"""Tune the flagship GEMM shapes with TunableOp on the MI355X and write the results CSV.

    python scripts/tune_gemms.py --out gpurun_out/tune/gemm_gfx950.csv [--model gpt3-1.3b]

Runs a few GPT-3 1.3B training steps (the bench.py config) with tuning on, then writes the
solutions; copy the CSV to paddle_ray_amd/tuning/gemm_gfx950.csv to make bench/smoke use it.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--model', default='gpt3-1.3b')
    ap.add_argument('--micro-batch', type=int, default=16)
    ap.add_argument('--seq', type=int, default=1024)
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--max-ms', type=int, default=30)
    a = ap.parse_args()
    import threading

    def heartbeat():  # tuning one GEMM can take minutes with no other output
        t0 = time.time()
        while True:
            time.sleep(30)
            live = a.out + '.live'
            n = sum(1 for _ in open(live)) if os.path.exists(live) else 0
            print(f"[tune] {time.time() - t0:.0f}s, {n} lines in {live}", flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    import torch
    import paddle_ray_amd as paddle
    from paddle_ray_amd.incubate import autotune
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    autotune.enable_gemm_tuning(filename=a.out + '.live', tune=True, max_duration_ms=a.max_ms,
                                max_iterations=200)
    paddle.set_device('gpu:0')
    paddle.set_default_dtype('bfloat16')
    cfg = gpt_config(a.model, max_seq_len=max(a.seq, 1024), hidden_dropout=0.1)
    model = GPTForPretraining(cfg)
    paddle.set_default_dtype('float32')
    opt = paddle.optimizer.AdamW(1e-4, parameters=model.parameters(), weight_decay=0.01,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0),
                                 multi_precision=True)
    model, opt, _ = group_sharded_parallel(model, opt, 'p_g_os')
    tok = torch.randint(0, cfg.vocab_size, (a.micro_batch, a.seq + 1), device='cuda')
    inp, lab = paddle.Tensor(tok[:, :-1].contiguous()), paddle.Tensor(tok[:, 1:].contiguous())
    for i in range(a.steps):
        t0 = time.time()
        loss = model(inp, lab)
        loss.backward()
        opt.step()
        opt.clear_grad()
        torch.cuda.synchronize()
        print(f"step {i} loss {float(loss):.4f} {time.time() - t0:.1f}s "
              f"tuned={len(torch.cuda.tunable.get_results())}", flush=True)
    print("validators:", torch.cuda.tunable.get_validators(), flush=True)
    n = autotune.write_gemm_results(a.out)
    print(f"wrote {n} GEMM solutions to {a.out}", flush=True)


if __name__ == '__main__':
    main()

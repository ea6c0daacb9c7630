#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): GPT-3 1.3B pretraining step with Fleet sharding
stage 3 ('p_g_os') over N MI355X GPUs (one process per GPU, RCCL over xGMI), bf16
compute, fp32 master weights + AdamW moments (sharded), synthetic token data,
random-init weights. Weak scaling: ``--micro-batch`` sequences of ``--seq`` tokens
per GPU per step.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Prints ONE JSON line on rank 0. ``--model resnet50`` runs the secondary headline
(ResNet50 bf16 images/s, DP).
"""
import argparse
import json
import math
import os
import sys
import time

BASELINE = None  # BASELINE.json "published" is empty: no reference number to divide by


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=10)
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--model', default='gpt3-1.3b')
    p.add_argument('--micro-batch', type=int, default=16)
    p.add_argument('--seq', type=int, default=1024)
    p.add_argument('--level', default='p_g_os')
    p.add_argument('--dropout', type=float, default=0.1)
    p.add_argument('--recompute', action='store_true')
    p.add_argument('--zero3-release', action='store_true',
                   help='release gathered ZeRO-3 units after forward (reference schedule)')
    p.add_argument('--no-graph', action='store_true',
                   help='BERT: run the static Executor op by op (no HIP-graph replay)')
    p.add_argument('--profile-dir', default=None)
    p.add_argument('--tuned-gemms', action='store_true',
                   help='load the committed MI355X TunableOp solutions for the library GEMMs (off by '
                        'default: measured 126.93 vs 126.93 ms per GPT step, profiles/r6/tunableop_ab.md)')
    p.add_argument('--no-tuned-gemms', action='store_true', help=argparse.SUPPRESS)  # (the old default)
    return p.parse_args()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _supervise(procs, limit_s, poll_s=0.2, grace_s=10.0):
    """Wait for every rank; the FIRST non-zero exit (or the wall-clock limit) terminates the
    siblings (SIGTERM, then SIGKILL after ``grace_s``) so one dead rank cannot leave the others
    blocked inside a collective. Returns the first failing status (124 on the time limit)."""
    import signal
    t_end = time.monotonic() + limit_s
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                print(f"bench.py: rank pid {p.pid} exited with {c}; stopping {len(live)} sibling(s)",
                      file=sys.stderr, flush=True)
        if live and (rc != 0 or time.monotonic() > t_end):
            if rc == 0:
                rc = 124
                print(f"bench.py: wall-clock limit {limit_s:.0f}s reached; stopping the ranks",
                      file=sys.stderr, flush=True)
            for p in live:
                p.send_signal(signal.SIGTERM)
            t_kill = time.monotonic() + grace_s
            while live and time.monotonic() < t_kill:
                live = [p for p in live if p.poll() is None]
                time.sleep(poll_s)
            for p in live:
                p.kill()
                p.wait()
            live = []
        time.sleep(poll_s)
    return rc


def _spawn_ranks(n):
    """``--gpus N`` without a launcher: start N fresh rank processes (one per GPU) and
    exit with the first failing child status (siblings are stopped, see ``_supervise``).
    Runs before this process imports torch or touches the GPU, so every rank initialises
    HIP in a clean process (no fork after HIP init, no exec from a GPU process)."""
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1', MASTER_PORT=port,
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '0'))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    return _supervise(procs, float(os.environ.get('PRA_BENCH_TIMEOUT', 570)))


def main():
    a = parse()
    if a.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(_spawn_ranks(a.gpus))
    if os.environ.get('PRA_BENCH_TRACE'):
        # diagnosing a stuck rank: every rank dumps all its threads' stacks periodically
        import faulthandler
        v = float(os.environ['PRA_BENCH_TRACE'])
        faulthandler.dump_traceback_later(v if v > 1 else 120.0, repeat=True)
    import torch
    import torch.distributed as dist
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import collective as C

    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; launch one rank per GPU "
                         f"(torchrun --nproc-per-node {a.gpus}) or drop WORLD_SIZE to self-spawn")
    if world > 1:
        # a rank stuck in a collective fails within 5 minutes (the default watchdog budget is
        # 30), well inside the driver's bench limit, so a broken run still reports
        os.environ.setdefault('PRA_COMM_TIMEOUT', '300')
        C.init_parallel_env()
    rank = C.get_rank()
    dev = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device('cpu')
    if dev.type == 'cuda':
        paddle.set_device(f'gpu:{dev.index}')
    paddle.seed(1234 + rank)
    if dev.type == 'cuda' and a.tuned_gemms:
        from paddle_ray_amd.incubate import autotune
        autotune.use_tuned_gemms()  # paddle_ray_amd/tuning/gemm_gfx950.csv (if present)

    if a.model.startswith('gpt'):
        result = bench_gpt(a, paddle, torch, dist, C, world, rank, dev)
    elif a.model.startswith('bert'):
        result = bench_bert(a, paddle, torch, dist, C, world, rank, dev)
    elif a.model.startswith('ernie'):
        result = bench_ernie(a, paddle, torch, dist, C, world, rank, dev)
    else:
        result = bench_resnet(a, paddle, torch, dist, C, world, rank, dev)
    result['backend'] = dist.get_backend() if world > 1 else 'none'
    result['world_size'] = world
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _timed(step_fn, a, torch, dist, world, dev):
    for _ in range(a.warmup):
        step_fn()
    if world > 1:
        dist.barrier()
    if dev.type == 'cuda':
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step_fn()
    if dev.type == 'cuda':
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def _op_profile(step_fn, a, torch, rank):
    """One extra (untimed) step under torch.profiler with Python stacks: per-op tables grouped
    by call site (which layer issues each fill / copy / reduce kernel)."""
    os.makedirs(a.profile_dir, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        step_fn()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_stack_n=6)
    with open(os.path.join(a.profile_dir, f'ops_by_stack_rank{rank}.txt'), 'w') as f:
        f.write(ka.table(sort_by='self_cuda_time_total', row_limit=120, max_name_column_width=60))
    with open(os.path.join(a.profile_dir, f'ops_rank{rank}.txt'), 'w') as f:
        f.write(prof.key_averages(group_by_input_shape=True).table(
            sort_by='self_cuda_time_total', row_limit=150, max_name_column_width=60))


def bench_gpt(a, paddle, torch, dist, C, world, rank, dev):
    from paddle_ray_amd.models import gpt_config, GPTForPretraining, gpt_flops_per_token
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    paddle.set_default_dtype('bfloat16')
    cfg = gpt_config(a.model, max_seq_len=max(a.seq, 1024), hidden_dropout=a.dropout,
                     recompute=a.recompute)
    model = GPTForPretraining(cfg)
    paddle.set_default_dtype('float32')
    clip = paddle.nn.ClipGradByGlobalNorm(1.0)
    sched = paddle.optimizer.lr.CosineAnnealingDecay(1e-4, T_max=100000)
    opt = paddle.optimizer.AdamW(learning_rate=sched, parameters=model.parameters(),
                                 weight_decay=0.01, grad_clip=clip, multi_precision=True,
                                 apply_decay_param_fun=lambda n: not ('norm' in n or '.b' in n))
    # stage 3 with the gathered units kept resident from forward to backward (288 GB
    # of HBM hold the 2.6 GB of gathered bf16 weights, so the backward re-gather is skipped);
    # --zero3-release restores the reference's release-after-forward schedule
    model, opt, _ = group_sharded_parallel(model, opt, a.level,
                                           release_after_forward=bool(a.zero3_release))
    g = torch.Generator(device=dev).manual_seed(rank)
    tokens = torch.randint(0, cfg.vocab_size, (a.micro_batch, a.seq + 1), device=dev, generator=g)
    inp = paddle.Tensor(tokens[:, :-1].contiguous())
    lab = paddle.Tensor(tokens[:, 1:].contiguous())
    losses = []

    def step():
        loss = model(inp, lab)
        loss.backward()
        opt.step()
        opt.clear_grad()
        sched.step()
        losses.append(loss.detach())

    dt = _timed(step, a, torch, dist, world, dev)
    if a.profile_dir:
        _op_profile(step, a, torch, rank)
    last_loss = float(losses[-1].item())
    tok = a.micro_batch * a.seq * world * a.steps
    tps = tok / dt
    fpt = gpt_flops_per_token(cfg, a.seq)
    mfu = tps / world * fpt / 2.5e15
    return {"metric": "tokens/sec GPT-3-1.3B Fleet sharding-3", "value": round(tps, 2),
            "unit": "tokens/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1000, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None if BASELINE is None else tps / BASELINE,
            "dtype": "bf16", "data": "synthetic (random tokens, random-init weights)",
            "config": {"model": "GPT-3-1.3B" if a.model == 'gpt3-1.3b' else a.model,
                       "global_batch": a.micro_batch * world, "seq_len": a.seq,
                       "parallelism": f"sharding{ {'os': 1, 'os_g': 2, 'p_g_os': 3}[a.level] }"
                                      f"_dp{world}",
                       "micro_batch_per_gpu": a.micro_batch, "hidden_dropout": a.dropout,
                       "optimizer": "AdamW fp32-master, global-norm clip",
                       # at world 1 there is nothing to shard (parallel/sharding.py turns the
                       # stage off, as the reference would): the step is plain training
                       "zero3_active": bool(world > 1 and a.level == 'p_g_os'),
                       "zero3_params": ("released after forward" if a.zero3_release
                                        else "gathered units resident forward->backward (non-default)")
                       if world > 1 and a.level == 'p_g_os' else "n/a (world 1)"},
            "tokens_per_sec_per_gpu": round(tps / world, 2),
            "mfu_bf16_dense": round(mfu, 4), "final_loss": round(last_loss, 4)}


def bench_resnet(a, paddle, torch, dist, C, world, rank, dev):
    from paddle_ray_amd.vision.models import resnet50
    model = resnet50(data_format='NHWC')
    model = paddle.amp.decorate(model, level='O2', dtype='bfloat16')
    opt = paddle.optimizer.Momentum(0.1, 0.9, parameters=model.parameters(), weight_decay=1e-4,
                                    multi_precision=True)
    if world > 1:
        model = paddle.DataParallel(model)
    elif dev.type == 'cuda' and not a.no_graph and os.environ.get('PRA_RESNET_GRAPH', '0') == '1':
        # (opt-in, PRA_RESNET_GRAPH=1) jit.to_static training capture: forward and backward of the
        # dygraph model replayed as two HIP graphs (jit/api.py _TrainGraph, accumulate mode).
        # Measured slower than eager on the same box: 9300 / 9291 vs 9546 / 9590 img/s
        # (profiles/r5/resnet_graph_ab.log) -- the eager queue already keeps the GPU busy
        st = paddle.static.BuildStrategy()
        st.use_hip_graph = True
        model = paddle.jit.to_static(model, build_strategy=st)
    bs = a.micro_batch if a.micro_batch != 16 else 256
    x = paddle.Tensor(torch.randn(bs, 224, 224, 3, device=dev, dtype=torch.bfloat16))
    y = paddle.Tensor(torch.randint(0, 1000, (bs,), device=dev))
    ce = paddle.nn.CrossEntropyLoss()

    def step():
        loss = ce(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()

    dt = _timed(step, a, torch, dist, world, dev)
    if a.profile_dir:
        _op_profile(step, a, torch, rank)
    graphed = hasattr(model, 'forward') and hasattr(model.forward, 'graph_status')
    if graphed:
        st_ = model.forward.graph_status()
        graphed = bool(st_) and all(v == 'graph' for v in st_.values())
        if not graphed and rank == 0:
            print(f"resnet: HIP-graph capture fell back to eager: {st_}", file=sys.stderr)
    ips = bs * world * a.steps / dt
    return {"metric": "samples/sec ResNet50 bf16", "value": round(ips, 2), "unit": "images/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1000, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"model": "ResNet50", "global_batch": bs * world, "seq_len": None,
                       "parallelism": f"dp{world}",
                       "executor": "HIP graph (jit.to_static capture)" if graphed else "eager"},
            "samples_per_sec_per_gpu": round(ips / world, 2)}


def bench_ernie(a, paddle, torch, dist, C, world, rank, dev):
    """BASELINE config 5: ERNIE-3.0 10B MLM pretraining, Fleet hybrid TP=2 x PP=world/2 (TP=2 x
    PP=4 on 8 GPUs: Megatron column/row-parallel layers with RCCL all-reduce inside each stage,
    1F1B micro-batch schedule over RCCL send/recv between stages); one GPU trains the whole
    10B model (bf16 params, fp32 AdamW master/moments: ~160 GB of 288). Tokens/s of the job."""
    import numpy as np
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.models import ernie_config, ernie_pipe
    mp = 2 if world % 2 == 0 else 1
    pp = world // mp
    S = a.seq if a.seq != 1024 else 512
    micro = a.micro_batch if a.micro_batch != 16 else 8
    acc = max(8, 2 * pp)
    name = 'ernie-3.0-10b' if a.model in ('ernie', 'ernie-10b', 'ernie-3.0-10b') else a.model
    cfg = ernie_config(name, mp_degree=mp, hidden_dropout_prob=a.dropout,
                       attention_probs_dropout_prob=0.0, max_position_embeddings=max(S, 512))
    if world > 1:
        st = fleet.DistributedStrategy()
        st.hybrid_configs = {'dp_degree': 1, 'mp_degree': mp, 'pp_degree': pp}
        st.pipeline_configs = {'micro_batch_size': micro, 'accumulate_steps': acc}
        fleet.init(is_collective=True, strategy=st)
    paddle.seed(1234)
    pl = ernie_pipe(cfg)
    pl = paddle.amp.decorate(pl, level='O2', dtype='bfloat16')
    opt = paddle.optimizer.AdamW(1e-4, parameters=pl.parameters(), multi_precision=True)
    rs = np.random.RandomState(rank)
    B = micro * acc
    ids = paddle.to_tensor(rs.randint(5, cfg.vocab_size, (B, S)))
    labels = paddle.to_tensor(rs.randint(5, cfg.vocab_size, (B, S)))
    if world > 1:
        model = fleet.distributed_model(pl)
        opt = fleet.distributed_optimizer(opt)

        def step():
            model.train_batch([ids, labels], opt)
    else:
        idc, lbc = ids.split(acc, 0), labels.split(acc, 0)

        def step():
            for i in range(acc):
                loss = pl._loss_fn(pl(idc[i]), lbc[i]) / acc
                loss.backward()
            opt.step()
            opt.clear_grad()

    dt = _timed(step, a, torch, dist, world, dev)
    tps = B * S * a.steps / dt
    n_params = sum(int(np.prod(p.shape)) for p in pl.parameters()) * mp
    return {"metric": "tokens/sec ERNIE-3.0-10B Fleet TP x PP", "value": round(tps, 2),
            "unit": "tokens/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1000, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random tokens, random-init weights)",
            "config": {"model": "ERNIE-3.0-10B" if name == "ernie-3.0-10b" else name, "global_batch": B, "seq_len": S,
                       "parallelism": f"tp{mp}_pp{pp}", "micro_batch": micro,
                       "accumulate_steps": acc, "params_per_stage_x_tp": n_params}}


def bench_bert(a, paddle, torch, dist, C, world, rank, dev):
    """BASELINE config 3: BERT-base pretraining through the STATIC-graph Executor with AMP
    (static.amp.decorate, bf16): per-op grad ops, fwd+bwd replayed as one HIP graph, AdamW.
    MLM as in the reference's BERT pretraining data (max_predictions_per_seq = 80 at seq 512,
    20 at 128): the prediction head and its softmax-CE run on the masked positions only."""
    import numpy as np
    from paddle_ray_amd import static
    from paddle_ray_amd.models import bert_config, BertForPretraining
    name = 'bert-base-uncased' if a.model in ('bert', 'bert-base') else a.model
    cfg = bert_config(name)
    bs = a.micro_batch if a.micro_batch != 16 else 32
    S = a.seq if a.seq != 1024 else 512
    paddle.seed(1234)
    # AMP O2 (the reference's use_pure_fp16 with bf16): bf16 parameters, fp32 master weights and
    # moments in the optimizer, so every op runs the bf16 fused kernels with no per-op casts
    paddle.set_default_dtype('bfloat16')
    model = BertForPretraining(cfg)
    paddle.set_default_dtype('float32')
    paddle.enable_static()
    main_p, startup = static.Program(), static.Program()
    P = max(1, int(round(S * 0.15625)))  # masked positions per sequence (80 at 512)
    with static.program_guard(main_p, startup):
        ids_v = static.data('ids', [bs, S], 'int64')
        pos_v = static.data('pos', [bs * P], 'int64')
        lab_v = static.data('lab', [bs * P], 'int64')
        nsp_v = static.data('nsp', [bs], 'int64')
        loss_v = model(ids_v, masked_positions=pos_v, labels=lab_v, next_sentence_label=nsp_v)
        opt = static.amp.decorate(paddle.optimizer.AdamW(1e-4, parameters=model.parameters(),
                                                         multi_precision=True),
                                  use_bf16=True, use_pure_fp16=True)
        if world > 1:
            # static-mode fleet data parallel: bucketed async gradient all-reduce inside the
            # backward (distributed/fleet/meta_optimizers.py)
            from paddle_ray_amd.distributed import fleet
            fleet.init(is_collective=True)
            opt = fleet.distributed_optimizer(opt)
        opt.minimize(loss_v)
    exe = static.Executor()
    exe.run(startup)
    prog = main_p
    if dev.type == 'cuda' and not a.no_graph:
        prog = static.CompiledProgram(main_p)
        prog._build_strategy.use_hip_graph = True
    rs = np.random.RandomState(rank)
    ids = rs.randint(5, cfg.vocab_size, (bs, S))
    pos = np.stack([np.sort(rs.choice(S, P, replace=False)) + i * S for i in range(bs)]).reshape(-1)
    lab = ids.reshape(-1)[pos].copy()
    ids.reshape(-1)[pos] = 103  # [MASK]
    feed = {'ids': torch.from_numpy(ids.astype('int64')).to(dev),
            'pos': torch.from_numpy(pos.astype('int64')).to(dev),
            'lab': torch.from_numpy(lab.astype('int64')).to(dev),
            'nsp': torch.from_numpy(rs.randint(0, 2, (bs,)).astype('int64')).to(dev)}
    feed = {k: paddle.Tensor(v) for k, v in feed.items()}
    last = [None]

    def step():
        last[0] = exe.run(prog, feed=feed, fetch_list=[loss_v], return_numpy=False)[0]

    dt = _timed(step, a, torch, dist, world, dev)
    if a.profile_dir:
        _op_profile(step, a, torch, rank)   # per-op tables need --no-graph (a graph replay is one op)
    paddle.disable_static()
    sps = bs * world * a.steps / dt
    return {"metric": "samples/sec BERT-base static+AMP", "value": round(sps, 2),
            "unit": "sequences/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1000, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"model": name, "global_batch": bs * world, "seq_len": S,
                       "parallelism": f"dp{world}", "executor": "static Program, " + ("op by op" if a.no_graph else "HIP graph"),
                       "amp": "O2 bf16 (fp32 master weights)",
                       "masked_positions_per_seq": P},
            "tokens_per_sec": round(sps * S, 1), "final_loss": float(last[0])}


if __name__ == '__main__':
    main()

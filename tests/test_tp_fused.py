"""Tensor parallel keeps the fused path: GPT at mp=2 (fused add+dropout+LN blocks, vocab-
parallel embedding lookup and vocab-parallel softmax-CE) matches the single-process model
built from the gathered shards — losses over 3 SGD steps and the updated weights.

Parity: python/paddle/distributed/fleet/layers/mpu/mp_layers.py (Column/RowParallelLinear,
VocabParallelEmbedding, ParallelCrossEntropy), c_softmax_with_cross_entropy_op.cu."""
import numpy as np
import pytest
import torch

from dist_utils import run_ranks


def _gather(sd_mp, cfg, world):
    """Full single-process state dict from this rank's shards (all-gathered)."""
    import torch.distributed as dist
    H, nh = cfg.hidden_size, cfg.num_heads
    hd = H // nh
    full = {}
    for k, v in sd_mp.items():
        t = v._t.detach().contiguous()
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        if 'qkv_proj' in k:   # local columns are (3, heads/mp, hd): interleave per head group
            lead = t.shape[:-1]
            ps = [p.reshape(*lead, 3, nh // world, hd) for p in parts]
            full[k] = torch.cat(ps, -2).reshape(*lead, 3 * H)
        elif 'word_embeddings' in k or 'out_proj.weight' in k or 'fc2.weight' in k:
            full[k] = torch.cat(parts, 0)
        elif 'fc1' in k:
            full[k] = torch.cat(parts, -1)
        else:
            assert all(torch.equal(p, t) for p in parts), k  # replicated params agree
            full[k] = t
    return full


def _tp_gpt_worker(rank, world, dropout):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    from paddle_ray_amd.parallel import tensor_parallel as tp
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 1, 'mp_degree': world, 'pp_degree': 1}
    fleet.init(is_collective=True, strategy=st)
    tp.model_parallel_random_seed(5)
    cfg = gpt_config('gpt3-tiny', mp_degree=world, hidden_dropout=dropout, num_layers=2)
    model = GPTForPretraining(cfg)
    assert all(b.fused for b in model.gpt.layers)
    full = _gather(model.state_dict(), cfg, world)
    ref = GPTForPretraining(gpt_config('gpt3-tiny', hidden_dropout=dropout, num_layers=2))
    ref.set_state_dict({k: paddle.Tensor(v.clone()) for k, v in full.items()})
    ids = np.random.RandomState(0).randint(0, 1024, (2, 17))
    x, y = paddle.to_tensor(ids[:, :-1]), paddle.to_tensor(ids[:, 1:])
    out = {}
    for name, m in (('mp', model), ('ref', ref)):
        opt = paddle.optimizer.SGD(0.5, parameters=m.parameters())
        paddle.seed(11)  # same dropout stream for both runs (and on every mp rank)
        losses = []
        for _ in range(3):
            loss = m(x, y)
            loss.backward()
            opt.step()
            opt.clear_grad()
            losses.append(float(loss))
        out[name] = losses
    after = _gather(model.state_dict(), cfg, world)
    rsd = ref.state_dict()
    out['max_w_diff'] = max(float((after[k] - rsd[k]._t).abs().max()) for k in after)
    return out


@pytest.mark.parametrize('dropout', [0.0, 0.1])
def test_gpt_mp2_matches_single_process(tmp_path, dropout):
    res = run_ranks(_tp_gpt_worker, 2, tmp_path, (dropout,))
    for r in res:
        np.testing.assert_allclose(r['mp'], r['ref'], rtol=1e-5, atol=1e-5)
        assert r['max_w_diff'] < 1e-5
    assert res[0]['mp'] == res[1]['mp']


def test_vocab_parallel_ce_matches_full_softmax_ce(tmp_path):
    res = run_ranks(_vpce_worker, 2, tmp_path)
    for r in res:
        np.testing.assert_allclose(r['loss'], r['ref_loss'], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(r['grad'], r['ref_grad'], rtol=1e-5, atol=1e-7)


def _vpce_worker(rank, world, device='cpu', dtype=torch.float32):
    import torch.distributed as dist
    from paddle_ray_amd.ops import fused as K
    g = torch.Generator().manual_seed(0)
    T, V = 37, 96
    logits = (torch.randn(T, V, generator=g) * 3).to(dtype)
    labels = torch.randint(0, V, (T,), generator=g)
    labels[3] = -100
    labels[5] = V // world            # a label at a shard boundary
    per = V // world
    mine = logits[:, rank * per:(rank + 1) * per].clone().to(device).requires_grad_(True)
    loss = K.vocab_parallel_cross_entropy(mine, labels.to(device), None, world, rank)
    dl = torch.linspace(0.5, 1.5, T, device=device)
    (loss * dl).sum().backward()
    full = logits.float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(full, labels, ignore_index=-100, reduction='none')
    (ref * dl.cpu()).sum().backward()
    return {'loss': loss.detach().float().cpu().numpy(), 'ref_loss': ref.detach().numpy(),
            'grad': mine.grad.float().cpu().numpy(),
            'ref_grad': full.grad[:, rank * per:(rank + 1) * per].numpy()}


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_vocab_parallel_ce_hip_kernel_gpu(dtype):
    """The HIP partial/final/backward kernels against the fp32 torch reference, as one rank of
    a 4-way vocab split with the other ranks' partials computed by the same kernel."""
    from paddle_ray_amd.ops import fused as K
    from paddle_ray_amd.ops import registry as R
    g = torch.Generator().manual_seed(1)
    T, V, world = 300, 4 * 1000, 4
    per = V // world
    logits = (torch.randn(T, V, generator=g) * 4).to(dtype).cuda()
    labels = torch.randint(0, V, (T,), generator=g).cuda()
    labels[7] = -100
    parts = [R.dispatch('vp_ce_part_fwd', logits, logits[:, r * per:(r + 1) * per].contiguous(),
                        labels, r * per) for r in range(world)]
    allp = torch.stack(parts)
    loss, lse = R.dispatch('vp_ce_final', allp, allp, labels, V, -100)
    lf = logits.float()
    ref = torch.nn.functional.cross_entropy(lf, labels, ignore_index=-100, reduction='none')
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lse, torch.logsumexp(lf, -1), rtol=1e-5, atol=1e-4)
    dloss = torch.rand(T, device='cuda')
    lf.requires_grad_(True)
    (torch.nn.functional.cross_entropy(lf, labels, ignore_index=-100, reduction='none') * dloss).sum().backward()
    for r in range(world):
        sl = logits[:, r * per:(r + 1) * per].contiguous()
        gr = R.dispatch('vp_ce_bwd', sl, sl, labels, lse, dloss, r * per, V, -100)
        tol = 1e-6 if dtype == torch.float32 else 2e-3
        torch.testing.assert_close(gr.float(), lf.grad[:, r * per:(r + 1) * per], rtol=1e-2, atol=tol)
    assert K._native.lib() is not None

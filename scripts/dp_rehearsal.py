"""Multi-rank rehearsal of the data-parallel training path on ONE GPU.

    RAFT_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29561 scripts/dp_rehearsal.py [--graph] [--fp32]

``--fp32``: the fp32 model (the reference's default precision, `train_standard.sh`): the DP
gradient must match the mean of the ranks' single-process slice gradients (same shapes, same
kernels) to rel 1e-5 -- what remains is the all-reduce's own summation, so this pins the DP
arithmetic rather than bf16 noise -- and the full-batch gradient to 1e-3.  Without a RAFT_DIST_BACKEND the
ranks use RCCL, one GPU each (needs as many visible GPUs as ranks).

Every rank runs the fused HIP training path on cuda:0 with its half of a batch; GradSync
all-reduces the gradients (bucketed, side stream, post-accumulate-grad hooks).  Rank 0 then
recomputes the full-batch gradient in a single process and checks that the averaged DP gradient
matches it (BatchNorm frozen, as in every stage after chairs, so per-replica batch statistics do
not enter).  RCCL refuses two ranks on one device, hence gloo (which reduces CUDA tensors through
the host); the launch, hook, bucket and stream logic is the code the 8-GPU RCCL run executes.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_raft_amd import RAFT  # noqa: E402
from pytorch_raft_amd.data.synthetic import make_pair_batch  # noqa: E402
from pytorch_raft_amd.engine.trainer import TrainState  # noqa: E402
from pytorch_raft_amd.parallel import dist as pdist  # noqa: E402
from pytorch_raft_amd.ops import _ext  # noqa: E402


def single_grad(args, sd, dev, i1, i2, flow, valid):
    """Flat gradient of ONE process on the given batch, from the state dict ``sd``."""
    torch.manual_seed(0)
    ref = RAFT(argparse.Namespace(**vars(args))).to(dev).train()
    ref.freeze_bn()
    ref.load_state_dict(sd)
    st = TrainState(ref, args, dev, sync=False)
    st.forward_backward(i1, i2, flow, valid)
    return torch.cat([p.grad.reshape(-1).float() for p in ref.parameters()])


def half_mean_grad(args, sd, dev, world, i1, i2, flow, valid):
    """Mean of single-process gradients of the ranks' own slices: the same batch shape (so the
    same kernels) as each rank ran -- what the all-reduce must reproduce up to its own sums."""
    gs = []
    for r in range(world):
        s = slice(2 * r, 2 * r + 2)
        gs.append(single_grad(args, sd, dev, i1[s], i2[s], flow[s], valid[s]))
    return sum(gs) / world


def graph_mode(model, args, dev, rank, world, i1, i2, flow, valid, sl, fp32=False):
    """The graphed step's DP path: eager encoders + g_dec replay -> one flat all-reduce of the
    update-block gradients overlapping the eager encoder backward, whose post-accumulate-grad
    hooks launch the encoder gradient buckets -> clip + fused AdamW."""
    from pytorch_raft_amd.engine.trainer import GraphedTrainStep
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    st = TrainState(model, args, dev, graph_ready=True)
    assert st.sync is None
    g = GraphedTrainStep(st, (i1[sl], i2[sl], flow[sl], valid[sl]), warmup=1)
    assert g.enc_sync is not None and len(g.enc_sync.buckets) > 1
    # kernel choices made once on rank 0: identical tile tables, no autotune on the other ranks
    tab = pdist.conv_tuning_table().tolist()
    tabs = [None] * world
    torch.distributed.all_gather_object(tabs, (sorted(map(tuple, tab)),
                                               int(_ext.ops().conv_autotune_runs())))
    tables_same = all(t[0] == tabs[0][0] for t in tabs) and len(tabs[0][0]) > 0
    runs = [t[1] for t in tabs]
    # one step up to the averaged gradients (weights untouched)
    g._forward_backward_sync(i1[sl], i2[sl], flow[sl], valid[sl], graphs=True)
    torch.cuda.synchronize()
    g_dp = torch.cat([p.grad.reshape(-1).float() for p in model.parameters()])
    # overlap: the first encoder bucket was launched while encoder gradients were still pending
    n_enc = len(g.enc_sync.bucket_of)
    first_bucket, fired = g.enc_sync.launch_log[0]
    assert fired < n_enc, (g.enc_sync.launch_log, n_enc)
    launched_early = sum(1 for _, f in g.enc_sync.launch_log if f < n_enc)
    # two full steps: every rank must hold bit-identical weights afterwards, and the first step
    # must match ONE single-process step of the global batch (rank 0 below)
    w0 = torch.cat([p.detach().reshape(-1).float() for p in model.parameters()])
    g.step(i1[sl], i2[sl], flow[sl], valid[sl])
    torch.cuda.synchronize()
    w1 = torch.cat([p.detach().reshape(-1).float() for p in model.parameters()])
    g.step(i1[sl], i2[sl], flow[sl], valid[sl])
    torch.cuda.synchronize()
    w = torch.cat([p.detach().reshape(-1).float() for p in model.parameters()])
    ws = [torch.empty_like(w) for _ in range(world)]
    torch.distributed.all_gather(ws, w)
    same = all(torch.equal(ws[0], x) for x in ws)
    if rank == 0:
        g_full = single_grad(args, sd, dev, i1, i2, flow, valid)
        rel = ((g_dp - g_full).norm() / g_full.norm()).item()
        g_half = half_mean_grad(args, sd, dev, world, i1, i2, flow, valid)
        rel_h = ((g_dp - g_half).norm() / g_half.norm()).item()
        # one eager single-process step of the global batch from the same weights
        torch.manual_seed(0)
        ref = RAFT(argparse.Namespace(**vars(args))).to(dev).train()
        ref.freeze_bn()
        ref.load_state_dict(sd)
        st2 = TrainState(ref, args, dev, sync=False)
        # TrainState.step would broadcast BN buffers (a collective) from rank 0 alone: the
        # single-process step is spelled out instead
        st2.optimizer.zero_grad(set_to_none=True)
        loss2, _ = st2.forward_backward(i1, i2, flow, valid)
        st2.apply_update(loss2)
        st2.scheduler.step()
        torch.cuda.synchronize()
        wr = torch.cat([p.detach().reshape(-1).float() for p in ref.parameters()])
        # AdamW's first step is lr * g / (|g| + eps) ~ lr * sign(g): it is compared where the
        # gradient's sign is resolved (|g| above 4x the DP-vs-full discrepancy) and |g| >> eps
        # (around |g| ~ eps = 1e-8 the step still depends on |g| itself, and the per-rank vs
        # global loss normalisation moves such entries by O(1) of their size); the rest is
        # rounding noise whose sign varies run to run with the kernels' reduction order
        resolved = (g_full.abs() > 4 * (g_dp - g_full).abs()) & (g_full.abs() > 100 * args.epsilon)
        d_dp, d_ref = (w1 - w0)[resolved], (wr - w0)[resolved]
        rel_w = ((d_dp - d_ref).norm() / d_ref.norm()).item()
        cos_w = torch.nn.functional.cosine_similarity(d_dp[None], d_ref[None]).item()
        print('resolved gradient entries: %.4f' % resolved.float().mean().item(), flush=True)
        print('dp rehearsal (hipgraph%s): world=%d backend=%s enc_buckets=%d launched_during_'
              'backward=%d rel_grad_err=%.3e rel_grad_err_same_shapes=%.3e step_delta_rel=%.3e '
              'step_delta_cos=%.6f ranks_identical=%s tuned_tables_identical=%s autotune_runs=%s' %
              (', fp32' if fp32 else '', world, torch.distributed.get_backend(),
               len(g.enc_sync.buckets), launched_early, rel, rel_h, rel_w, cos_w, same,
               tables_same, runs), flush=True)
        _check(fp32, rel, rel_h)
        if fp32:
            assert cos_w > 0.9999 and rel_w < 1e-2, (cos_w, rel_w)
        else:
            # bf16: observed step delta rel 1.2e-3 / cos 0.999999 at 4 ranks once entries with
            # |g| ~ eps are excluded (round 3's 0.12 / 0.993 came from those)
            assert cos_w > 0.9995 and rel_w < 3e-2, (cos_w, rel_w)
        assert same, 'weights diverged across ranks'
        assert tables_same, 'ranks run different conv kernels'
        assert all(r == 0 for r in runs[1:]), ('ranks > 0 must not autotune', runs)


def _check(fp32, rel, rel_h):
    """rel_h: DP vs the mean of single-process gradients of the ranks' own slices (same shapes,
    same kernels) -- isolates the bucketed all-reduce.  rel: DP vs one full-batch process (other
    batch shapes pick other MIOpen solvers / conv tiles, so it also carries their rounding)."""
    if fp32:
        assert rel_h < 1e-5, rel_h
        assert rel < 1e-3, rel
    else:
        assert rel_h < 1e-2, rel_h
        assert rel < 1e-2, rel


def main():
    graph = '--graph' in sys.argv
    fp32 = '--fp32' in sys.argv
    dev = pdist.init_distributed()
    rank, world = pdist.rank(), pdist.world_size()
    args = argparse.Namespace(small=False, mixed_precision=not fp32, corr_impl='hip', lr=4e-4,
                              wdecay=1e-4, epsilon=1e-8, num_steps=100, iters=4, gamma=0.8,
                              clip=1.0, add_noise=False, bucket_mb=2.0, enc_bucket_mb=1.0)
    torch.manual_seed(0)
    model = RAFT(args).to(dev).train()
    model.freeze_bn()
    pdist.broadcast_module(model)
    i1, i2, flow, valid = make_pair_batch(2 * world, 128, 160, device=dev)
    sl = slice(2 * rank, 2 * rank + 2)
    if graph:
        graph_mode(model, args, dev, rank, world, i1, i2, flow, valid, sl, fp32)
        pdist.barrier(dev)
        pdist.destroy()
        return
    st = TrainState(model, args, dev)
    assert st.sync is not None and st.sync.enabled
    st.optimizer.zero_grad(set_to_none=True)
    st.sync.prepare()
    loss, _ = st.forward_backward(i1[sl], i2[sl], flow[sl], valid[sl])
    st.sync.finish()
    g_dp = torch.cat([p.grad.reshape(-1).float() for p in model.parameters()])
    if rank == 0:
        sd = model.state_dict()
        g_full = single_grad(args, sd, dev, i1, i2, flow, valid)
        rel = ((g_dp - g_full).norm() / g_full.norm()).item()
        g_half = half_mean_grad(args, sd, dev, world, i1, i2, flow, valid)
        rel_h = ((g_dp - g_half).norm() / g_half.norm()).item()
        print('dp rehearsal%s: world=%d backend=%s buckets=%d rel_grad_err=%.3e '
              'rel_grad_err_same_shapes=%.3e loss=%.4f' %
              (' (fp32)' if fp32 else '', world, torch.distributed.get_backend(),
               len(st.sync.buckets), rel, rel_h, loss.item()), flush=True)
        _check(fp32, rel, rel_h)
    pdist.barrier(dev)
    pdist.destroy()


if __name__ == '__main__':
    main()

"""Long-horizon training parity: the HIP path vs the stock PyTorch-ROCm ops.

    python scripts/parity_train.py --impl hip   --steps 2000 --out gpurun_out/parity/hip.jsonl
    python scripts/parity_train.py --impl torch --steps 2000 --out gpurun_out/parity/torch.jsonl
    python scripts/parity_train.py --compare gpurun_out/parity/hip.jsonl gpurun_out/parity/torch.jsonl

Both runs start from the same random init (seed 1234) and see the same data in the same order:
step k trains on a fresh synthetic batch (``make_pair_batch`` seed 10007 + k, generated on the
device), so every batch is unseen when it is used and the per-step EPE of the final iteration
(measured BEFORE that batch's update) is a held-out error.  The reference loop is
`train.py:161-208` (AdamW + OneCycle, clip 1.0, gamma 0.8, bf16 autocast here).

``--impl hip`` runs the graphed native step (bench.py's path), ``--impl torch`` the stock ops
(MIOpen / ATen encoder and update block, torch correlation, torch loss, torch AdamW).  A drift
in a rarely used branch (a mis-scaled gradient, the GradScaler skip path, the correlation
backward's slab / atomic switch) shows up as a diverging curve long before 2,000 steps.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--impl', choices=['hip', 'torch'], default='hip')
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--batch', type=int, default=12)
    ap.add_argument('--size', type=int, nargs=2, default=[368, 496])
    ap.add_argument('--iters', type=int, default=12)
    ap.add_argument('--lr', type=float, default=4e-4)
    ap.add_argument('--log_every', type=int, default=50)
    ap.add_argument('--out', type=str, default=None)
    ap.add_argument('--compare', nargs=2, default=None, metavar=('A', 'B'))
    return ap.parse_args(argv)


def _window_mean(rows, key, lo, hi):
    v = [r[key] for r in rows if lo <= r['step'] < hi]
    return sum(v) / max(1, len(v))


def compare(pa, pb):
    ra = [json.loads(line) for line in open(pa) if line.strip().startswith('{"step"')]
    rb = [json.loads(line) for line in open(pb) if line.strip().startswith('{"step"')]
    n = min(ra[-1]['step'], rb[-1]['step']) + 1
    print('%8s %10s %10s %10s %10s' % ('steps', 'epe_a', 'epe_b', 'loss_a', 'loss_b'))
    w = max(1, n // 10)
    worst = 0.0
    for lo in range(0, n, w):
        ea, eb = _window_mean(ra, 'epe', lo, lo + w), _window_mean(rb, 'epe', lo, lo + w)
        la, lb = _window_mean(ra, 'loss', lo, lo + w), _window_mean(rb, 'loss', lo, lo + w)
        worst = max(worst, abs(ea - eb) / max(eb, 1e-6))
        print('%4d-%-4d %10.4f %10.4f %10.4f %10.4f' % (lo, lo + w - 1, ea, eb, la, lb))
    # final EPE: mean over the last 10 % of the steps (per-batch EPE is noisy)
    fa, fb = _window_mean(ra, 'epe', n - w, n), _window_mean(rb, 'epe', n - w, n)
    rel = abs(fa - fb) / max(fb, 1e-6)
    print('final EPE (last %d steps): %.4f vs %.4f  rel diff %.2f%%  (worst window %.2f%%)'
          % (w, fa, fb, 100 * rel, 100 * worst))
    return rel


def main(argv=None):
    a = parse(argv)
    if a.compare:
        rel = compare(*a.compare)
        sys.exit(0 if rel <= 0.05 else 1)
    import torch
    from pytorch_raft_amd.models.raft import RAFT
    from pytorch_raft_amd.engine.trainer import TrainState, GraphedTrainStep
    from pytorch_raft_amd.data.synthetic import make_pair_batch

    dev = torch.device('cuda', 0)
    torch.backends.cudnn.benchmark = True
    margs = argparse.Namespace(
        small=False, mixed_precision=True, amp_dtype='bfloat16', alternate_corr=False,
        dropout=0.0, corr_mode='auto', corr_impl='torch' if a.impl == 'torch' else 'auto',
        lr=a.lr, wdecay=1e-4, epsilon=1e-8, num_steps=a.steps, iters=a.iters, gamma=0.8,
        clip=1.0, add_noise=False)
    if a.impl == 'torch':
        import pytorch_raft_amd.ops.loss as L
        import pytorch_raft_amd.engine.trainer as T
        _orig = L.sequence_loss

        def _torch_loss(*x, **k):
            k['impl'] = 'torch'
            return _orig(*x, **k)
        T.sequence_loss = _torch_loss
    torch.manual_seed(1234)
    model = RAFT(margs).to(dev).train()
    h, w = a.size

    def batch(k):
        return make_pair_batch(a.batch, h, w, device=dev, seed=10007 + k)

    graphed = a.impl == 'hip'
    st = TrainState(model, margs, dev, graph_ready=graphed)
    stepper = GraphedTrainStep(st, batch(0), warmup=2) if graphed else st
    out = open(a.out, 'w') if a.out else sys.stdout
    out.write(json.dumps({'impl': a.impl, 'steps': a.steps, 'batch': a.batch, 'size': [h, w],
                          'iters': a.iters, 'lr': a.lr}) + '\n')
    hist = []
    t0 = time.perf_counter()
    for k in range(a.steps):
        i1, i2, fl, va = batch(k)
        loss, met = stepper.step(i1, i2, fl, va)
        hist.append(torch.stack([loss.detach().float(), met['epe'].detach().float()]))
        if (k + 1) % a.log_every == 0 or k + 1 == a.steps:
            vals = torch.stack(hist).cpu().tolist()
            base = k + 1 - len(vals)
            for j, (lv, ev) in enumerate(vals):
                out.write(json.dumps({'step': base + j, 'loss': lv, 'epe': ev}) + '\n')
            out.flush()
            hist = []
            print('parity[%s]: step %d/%d  loss %.4f epe %.4f  %.1f s' % (
                a.impl, k + 1, a.steps, vals[-1][0], vals[-1][1], time.perf_counter() - t0),
                file=sys.stderr, flush=True)
    assert stepper.check_finite(), 'non-finite loss / skipped step'
    if out is not sys.stdout:
        out.close()


if __name__ == '__main__':
    main()

"""Steady-state per-kernel time: kernel_stats(warmup+K steps) - kernel_stats(warmup only).

usage: prof_diff.py <dir_warm_only> <dir_warm_plus_steps> <steps>
       prof_diff.py --single <dir_of_timed_region_trace> <steps>
"""
import csv, glob, os, sys


def load(d):
    f = glob.glob(os.path.join(d, '**', '*kernel_stats.csv'), recursive=True)
    if not f:
        return {}
    out = {}
    for r in csv.DictReader(open(f[0])):
        out[r['Name']] = (float(r['TotalDurationNs']), int(r['Calls']))
    return out


if sys.argv[1] == '--single':   # one trace restricted to the timed region (roctx selected regions)
    a, b, steps = {}, load(sys.argv[2]), int(sys.argv[3])
else:
    a, b, steps = load(sys.argv[1]), load(sys.argv[2]), int(sys.argv[3])
rows = []
for k, (t, c) in b.items():
    t0, c0 = a.get(k, (0.0, 0))
    if c - c0 > 0 and t - t0 > 0:
        rows.append((t - t0, c - c0, k))
tot = sum(r[0] for r in rows)
print('steady-state kernel time per step: %.3f ms over %d steps (sum of kernel durations)' % (tot / 1e6 / steps, steps))
print('%7s %8s %9s %10s  %s' % ('pct', 'calls/st', 'avg_us', 'ms/step', 'kernel'))
for t, c, k in sorted(rows, reverse=True)[:400]:
    print('%6.2f%% %8.1f %9.1f %10.3f  %s' % (100 * t / tot, c / steps, t / c / 1e3, t / 1e6 / steps, k[:140]))

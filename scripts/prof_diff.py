"""Steady-state per-kernel time: kernel_stats(warmup+K steps) - kernel_stats(warmup only).

usage: prof_diff.py <dir_warm_only> <dir_warm_plus_steps> <steps>
       prof_diff.py --single <dir_of_timed_region_trace> <steps>
       prof_diff.py --markers <dir_of_full_trace> <steps>   (bench.py --trace_markers)
       prof_diff.py --phases <dir_of_full_trace> <steps>    (+ RAFT_PHASE_MARKS=1: [decode] / [encoder])
       prof_diff.py --sequence <dir_of_full_trace>          (dispatch order of the last step's tail)
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


def load_between_markers(d):
    """Kernels dispatched between the last two marker spin kernels (bench.py --trace_markers)."""
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'spin' in r['Kernel_Name'].lower() or 'sleep' in r['Kernel_Name'].lower()]
    assert len(marks) >= 2, 'no marker kernels in the trace'
    i0, i1 = marks[-2], marks[-1]
    out = {}
    for r in rows[i0 + 1:i1]:
        t, c = out.get(r['Kernel_Name'], (0.0, 0))
        out[r['Kernel_Name']] = (t + int(r['End_Timestamp']) - int(r['Start_Timestamp']), c + 1)
    return out


def load_phases(d):
    """As load_between_markers, with every kernel name prefixed by its phase: the decode replay
    (correlation, update block, upsampling, loss; forward + backward) is bracketed by
    raft_phase_marker_kernel launches (RAFT_PHASE_MARKS=1) -> '[decode] '; everything else
    (encoders forward / backward, clip, optimizer) -> '[encoder] '."""
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'spin' in r['Kernel_Name'].lower() or 'sleep' in r['Kernel_Name'].lower()]
    assert len(marks) >= 2, 'no marker kernels in the trace'
    i0, i1 = marks[-2], marks[-1]
    out = {}
    decode = False
    for r in rows[i0 + 1:i1]:
        name = r['Kernel_Name']
        if 'raft_phase_marker' in name:
            decode = not decode
            continue
        key = '[%s] %s' % ('decode' if decode else 'encoder', name)
        t, c = out.get(key, (0.0, 0))
        out[key] = (t + int(r['End_Timestamp']) - int(r['Start_Timestamp']), c + 1)
    return out


def sequence(d):
    """Dispatch-ordered kernels from the end of the second-to-last decode replay to the last
    timing marker: the previous step's encoder backward + optimizer, this step's encoder forward,
    decode replay and encoder backward (RAFT_PHASE_MARKS=1 + --trace_markers)."""
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'spin' in r['Kernel_Name'].lower() or 'sleep' in r['Kernel_Name'].lower()]
    i1 = marks[-1]
    pm = [i for i in range(i1) if 'raft_phase_marker' in rows[i]['Kernel_Name']]
    start = pm[-3] if len(pm) >= 3 else 0
    phase = 'encoder'
    for r in rows[start + 1:i1]:
        name = r['Kernel_Name']
        if 'raft_phase_marker' in name:
            phase = 'decode' if phase == 'encoder' else 'encoder'
            print('---- %s' % phase)
            continue
        us = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        print('%8.1f  [%s] %s' % (us, phase, name[:150]))


if sys.argv[1] == '--sequence':
    sequence(sys.argv[2])
    sys.exit(0)
if sys.argv[1] == '--phases':
    a, b, steps = {}, load_phases(sys.argv[2]), int(sys.argv[3])
elif sys.argv[1] == '--markers':
    a, b, steps = {}, load_between_markers(sys.argv[2]), int(sys.argv[3])
elif sys.argv[1] == '--single':   # one trace restricted to the timed region (roctx selected regions)
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

"""Host-side HIP API time inside the timed region of a traced bench run: which runtime calls the
host spends the step in (a blocking copy, a stream / event synchronize, an allocation).

    rocprofv3 --hip-trace --kernel-trace --output-format csv -d DIR -o run -- \\
        python bench.py --trace_markers ...
    python scripts/host_api_stalls.py DIR [steps]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    kf = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    hf = glob.glob(os.path.join(d, '**', '*hip_api_trace.csv'), recursive=True)
    krows = sorted(csv.DictReader(open(kf[0])), key=lambda r: int(r['Start_Timestamp']))
    marks = [r for r in krows if 'spin' in r['Kernel_Name'].lower() or 'sleep' in r['Kernel_Name'].lower()]
    assert len(marks) >= 2, 'no marker kernels (bench.py --trace_markers)'
    t0, t1 = int(marks[-2]['End_Timestamp']), int(marks[-1]['Start_Timestamp'])
    calls = {}
    long_calls = []
    for r in csv.DictReader(open(hf[0])):
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if e < t0 or s > t1:
            continue
        name = r.get('Function') or r.get('Operation') or r.get('Kind', '?')
        n, tot, mx = calls.get(name, (0, 0, 0))
        calls[name] = (n + 1, tot + e - s, max(mx, e - s))
        if e - s > 200000:
            long_calls.append((e - s, s - t0, name, r.get('Thread_Id', '?')))
    wall = t1 - t0
    print('timed region %.3f ms over %d steps; host HIP API time by call (all threads):'
          % (wall / 1e6, steps))
    print('%12s %8s %10s  %s' % ('total ms/step', 'calls', 'max us', 'function'))
    for name, (n, tot, mx) in sorted(calls.items(), key=lambda kv: -kv[1][1])[:30]:
        print('%12.3f %8d %10.1f  %s' % (tot / 1e6 / steps, n, mx / 1e3, name))
    print('calls longer than 200 us (duration us, offset ms, function, thread):')
    for dur, off, name, tid in sorted(long_calls, key=lambda x: x[1])[:60]:
        print('%10.1f %10.3f  %s  %s' % (dur / 1e3, off / 1e6, name, tid))


if __name__ == '__main__':
    main()

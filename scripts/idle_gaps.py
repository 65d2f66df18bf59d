"""GPU idle time inside the timed region of a traced bench run: the union of all kernels' busy
intervals (every stream) between the two timing markers vs the wall time between them, and the
largest gaps with the kernels on either side.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python bench.py --trace_markers ...
    python scripts/idle_gaps.py DIR [steps] [top]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows)
             if 'spin' in r['Kernel_Name'].lower() or 'sleep' in r['Kernel_Name'].lower()]
    assert len(marks) >= 2, 'no marker kernels in the trace (bench.py --trace_markers)'
    i0, i1 = marks[-2], marks[-1]
    t_begin = int(rows[i0]['End_Timestamp'])
    t_end = int(rows[i1]['Start_Timestamp'])
    ivs = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'])
           for r in rows[i0 + 1:i1]]
    ivs.sort()
    busy = 0
    gaps = []
    cur_s, cur_e, cur_name = None, None, None
    prev_name = rows[i0]['Kernel_Name']
    last_end = t_begin
    for s, e, name in ivs:
        if s > last_end:
            gaps.append((s - last_end, prev_name, name))
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= last_end:
            last_end = e
            prev_name = name
    if cur_e is not None:
        busy += cur_e - cur_s
    if t_end > last_end:
        gaps.append((t_end - last_end, prev_name, rows[i1]['Kernel_Name']))
    wall = t_end - t_begin
    idle = sum(g for g, _, _ in gaps)
    print('timed region: %.3f ms wall, %.3f ms busy (union of all streams), %.3f ms idle '
          '(%.1f %%) over %d steps -> %.3f ms idle per step; %d gaps'
          % (wall / 1e6, busy / 1e6, idle / 1e6, 100.0 * idle / max(wall, 1), steps,
             idle / 1e6 / steps, len(gaps)))
    buckets = {}
    for g, _, _ in gaps:
        k = '<2us' if g < 2000 else '2-5us' if g < 5000 else '5-20us' if g < 20000 else '>=20us'
        n, t = buckets.get(k, (0, 0))
        buckets[k] = (n + 1, t + g)
    for k in ('<2us', '2-5us', '5-20us', '>=20us'):
        n, t = buckets.get(k, (0, 0))
        print('  gaps %-7s %5d  %.3f ms' % (k, n, t / 1e6))
    print('largest gaps (us, kernel before -> kernel after):')
    for g, a, b in sorted(gaps, reverse=True)[:top]:
        print('%9.1f  %s -> %s' % (g / 1e3, a[:70], b[:70]))
    # the dispatch sequence of the last step boundary: kernels with start offsets, durations and
    # queue / stream ids around the largest gap of the last quarter of the region
    qcol = next((c for c in ('Stream_Id', 'Queue_Id') if c in rows[0]), None)
    tail = [iv for iv in ivs if iv[0] > t_begin + 0.75 * wall]
    if tail:
        best, at = 0, 0
        last = tail[0][1]
        for k in range(1, len(tail)):
            if tail[k][0] - last > best:
                best, at = tail[k][0] - last, k
            last = max(last, tail[k][1])
        lo, hi = max(0, at - 25), min(len(tail), at + 25)
        sid = {(int(r['Start_Timestamp']), r['Kernel_Name']): (r.get(qcol, '?') if qcol else '?')
               for r in rows[i0 + 1:i1]}
        print('around the largest late gap (%.1f us): start(us) dur(us) %s kernel' % (best / 1e3, qcol or ''))
        for s0, e0, name in tail[lo:hi]:
            print('%10.1f %8.1f %5s  %s' % ((s0 - t_begin) / 1e3, (e0 - s0) / 1e3,
                                           sid.get((s0, name), '?'), name[:90]))


if __name__ == '__main__':
    main()

"""Summarise rocprofv3 --stats / kernel-trace CSVs: top kernels by total time."""
import csv, glob, os, sys
root = sys.argv[1]
stats = glob.glob(os.path.join(root, '**', '*kernel_stats.csv'), recursive=True)
if stats:
    rows = list(csv.DictReader(open(stats[0])))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    print('kernel stats from', stats[0], 'total %.3f ms' % (tot / 1e6))
    rows.sort(key=lambda r: -float(r['TotalDurationNs']))
    print('%-8s %-8s %-10s %s' % ('pct', 'calls', 'avg_us', 'name'))
    for r in rows[:60]:
        print('%6.2f%% %8s %10.1f  %s' % (100 * float(r['TotalDurationNs']) / tot, r['Calls'],
                                          float(r['AverageNs']) / 1e3, r['Name'][:150]))
else:
    print('no kernel_stats.csv under', root)
    for f in glob.glob(os.path.join(root, '**', '*'), recursive=True):
        print(f)

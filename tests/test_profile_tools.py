"""CPU tests of the trace-analysis tools (scripts/idle_gaps.py, scripts/host_api_stalls.py,
scripts/grid_fill.py) on synthetic rocprofv3 CSVs: the busy-union / idle-gap arithmetic and the
marker bracketing that the round-6 host-side analysis (README, profiles/r6/host/) relies on."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, header, rows):
    with open(path, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def _kernel_trace(d):
    # two marker spins bracket the region [1000, 10000) ns; kernels on two streams overlap
    rows = [
        ('at::cuda::spin_kernel(long)', 0, 1000, 0),
        ('a', 1000, 3000, 0),         # busy 1000-3000
        ('b', 2000, 4000, 2),         # overlaps a: busy union 1000-4000
        ('c', 6000, 7000, 0),         # gap 4000-6000 (2 us)
        ('d', 9500, 9900, 2),         # gap 7000-9500 (2.5 us), then 9900-10000 (0.1 us)
        ('at::cuda::spin_kernel(long)', 10000, 11000, 0),
    ]
    _write(os.path.join(d, 'run_kernel_trace.csv'),
           ['Kernel_Name', 'Start_Timestamp', 'End_Timestamp', 'Stream_Id'], rows)


def test_idle_gaps_union_and_gaps(tmp_path):
    _kernel_trace(str(tmp_path))
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'idle_gaps.py'),
                          str(tmp_path), '1', '5'], capture_output=True, text=True, check=True).stdout
    first = out.splitlines()[0]
    # wall 9 us, busy 3 + 1 + 0.4 = 4.4 us, idle 2 + 2.5 + 0.1 = 4.6 us
    assert 'timed region: 0.009 ms wall, 0.004 ms busy' in first, first
    assert '3 gaps' in first, first
    assert '2.5  c -> d' in out, out


def test_host_api_stalls_bracketing(tmp_path):
    d = str(tmp_path)
    _kernel_trace(d)
    _write(os.path.join(d, 'run_hip_api_trace.csv'),
           ['Function', 'Start_Timestamp', 'End_Timestamp', 'Thread_Id'],
           [('hipLaunchKernel', 1200, 1300, 1), ('hipGraphLaunch', 2000, 502000, 1),
            ('hipMemcpyAsync', 50_000_000, 50_100_000, 1)])   # outside the region: ignored
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'host_api_stalls.py'), d, '1'],
                         capture_output=True, text=True, check=True).stdout
    assert 'hipGraphLaunch' in out and 'hipLaunchKernel' in out
    assert 'hipMemcpyAsync' not in out
    # the 500 us graph launch is listed among the long calls
    assert '500.0' in out.split('calls longer than 200 us')[1]


def test_grid_fill_reads_the_persisted_table():
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'grid_fill.py')],
                         capture_output=True, text=True, check=True).stdout
    lines = [l for l in out.splitlines()[1:] if l.strip()]
    assert len(lines) >= 20                     # the chairs-geometry keys of tune_db/
    assert all('%' in l for l in lines)


def test_categorize_splits_ours_by_phase_and_places_the_stem(tmp_path):
    p = tmp_path / 'summary.txt'
    p.write_text(
        '  5.00%   36.0  44.1  1.500  [decode] void conv_detail::conv_fwd_glds_kernel<3, 1, 1, 8, 2>(ConvFwdArgs)\n'
        '  1.00%    2.0  46.9  0.100  [encoder] void (anonymous namespace)::stem_conv_fwd_kernel<2, false>(x)\n'
        '  1.00%    2.0  58.9  0.120  [encoder] void (anonymous namespace)::stem_conv_wgrad_kernel<2, false>(x)\n'
        '  0.50%    2.0  23.3  0.040  [encoder] void (anonymous namespace)::stem_wgrad_reduce_kernel<false>(x)\n'
        '  0.50%    2.0  20.0  0.200  [encoder] void (anonymous namespace)::norm_bwd_stats_kernel<0>(x)\n')
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'categorize.py'), str(p)],
                         capture_output=True, text=True, check=True).stdout
    cats = {l.rsplit(None, 1)[0]: float(l.rsplit(None, 1)[1]) for l in out.splitlines()}
    assert cats['update-block dgrad'] == 1.5           # EPI 8 = dgrad, decode phase
    assert cats['encoder conv fwd'] == 0.1
    assert abs(cats['encoder wgrad'] - 0.16) < 1e-9
    assert cats['encoder norm'] == 0.2
    assert 'other' not in cats and 'reduce' not in cats
    assert abs(cats['total'] - 1.96) < 1e-9

"""Summarise a rocprofv3 --kernel-trace CSV (kernel_trace.csv): per-kernel
count / total / average device time over the last `window` of the trace (a
time window ending at the last dispatch, default: everything), and the union of
busy intervals (GPU-busy fraction) in that window.

``--timed-syrk <trace dir> <bench json>``: the headline kernel's launches of the
bench's timed region from a trace of ``bench.py --no-band --no-sparse``: the
batch-B ``syrk_kernel`` dispatches (Grid_Size_Y = B, the eta batch) are
(warmup + steps) x launches-per-step; the last steps x launches-per-step of them
are the timed ones. Prints count / average / total against the bench line's
HIP-event ``roofline.avg_launch_ms`` (JSON).

``--timed-spmm <trace dir> <bench json> [sparse4|sparse5]``: the same for a sparse
line's dominant SpMM (the launches between the timing marks; timed_spmm).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def timed_syrk(trace_dir, bench_json):
    with open(bench_json) as fh:
        line = json.loads([l for l in fh if l.startswith('{')][-1])
    roof = line['roofline']
    B = line['config']['eta_per_rank_per_step']
    steps, warm = line['steps'], line['warmup']
    files = glob.glob(os.path.join(trace_dir, '**', '*kernel_trace*.csv'), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if 'syrk_kernel' in r['Kernel_Name'] and 'band' not in r['Kernel_Name'] and \
                        int(r['Grid_Size_Y']) == B:
                    rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    rows.sort()
    per_step = roof['launches'] // steps
    # the headline curve runs first; later batch-B launches (a dense_nu25 sub-line)
    # are not part of its timed steps
    assert len(rows) >= (warm + steps) * per_step, (len(rows), warm, steps, per_step)
    timed = rows[warm * per_step:(warm + steps) * per_step]
    durs = [(e - s) / 1e6 for s, e in timed]
    avg = sum(durs) / len(durs)
    flops = roof['algorithmic_flops_per_launch']
    out = {'trace_files': [os.path.relpath(f) for f in files], 'batch': B,
           'launches_per_step': per_step, 'timed_launches': len(timed),
           'trace_avg_launch_ms': round(avg, 4), 'trace_total_ms': round(sum(durs), 3),
           'bench_avg_launch_ms': roof['avg_launch_ms'],
           'rel_diff_vs_bench': round(avg / roof['avg_launch_ms'] - 1.0, 5),
           'algorithmic_flops_per_launch': flops,
           'trace_tflops': round(flops / (avg * 1e-3) / 1e12, 3),
           'trace_frac_of_peak': round(flops / (avg * 1e-3) / 1e12 / roof['peak'], 4),
           'bench_frac': roof['frac']}
    print(json.dumps(out, indent=1))


def timed_spmm(trace_dir, bench_json, config=None):
    """The sparse line's dominant SpMM in the timed steps of a trace of
    ``bench.py --config sparseN``: the launches of that kernel instance (its block
    width) that start between the two ``timing_mark_kernel`` launches bracketing the
    timed loop (gpmi_sp_set_timing), against the bench line's in-step HIP-event
    ``roofline.avg_launch_ms``."""
    with open(bench_json) as fh:
        line = json.loads([l for l in fh if l.startswith('{')][-1])
    if config:
        line = line['sparse_modes'][config]
    roof = line['roofline']
    kern, width = re.match(r'(\w+) \(s=(\d+) columns\)', roof['kernel']).groups()
    files = glob.glob(os.path.join(trace_dir, '**', '*kernel_trace*.csv'), recursive=True)
    marks, rows = [], []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r['Kernel_Name']
                t = (int(r['Start_Timestamp']), int(r['End_Timestamp']))
                if 'timing_mark_kernel' in name:
                    marks.append(t[0])
                elif kern in name and re.search(r'%s<%s,' % (kern, width), name):
                    rows.append(t)
    marks.sort()
    # the timed window: the first on/off pair of marks (the line's set_timing(True)
    # then set_timing(False) around the timed steps; the second pair brackets the
    # isolated launches)
    assert len(marks) >= 2, marks
    lo, hi = marks[0], marks[1]
    timed = sorted(t for t in rows if lo <= t[0] <= hi)
    durs = [(e - s) / 1e6 for s, e in timed]
    avg = sum(durs) / len(durs)
    bench_n = roof['in_step_by_width'][width]['launches']
    alg = roof['algorithmic_bytes_per_launch']
    out = {'trace_files': [os.path.relpath(f) for f in files], 'kernel': '%s<%s>' % (kern, width),
           'timed_launches_trace': len(timed), 'timed_launches_bench': bench_n,
           'trace_avg_launch_ms': round(avg, 5), 'trace_total_ms': round(sum(durs), 3),
           'bench_avg_launch_ms': roof['avg_launch_ms'],
           'rel_diff_vs_bench': round(avg / roof['avg_launch_ms'] - 1.0, 5),
           'algorithmic_bytes_per_launch': round(alg),
           'trace_gbs': round(alg / (avg * 1e-3) / 1e9, 1),
           'trace_frac_of_hbm_peak': round(alg / (avg * 1e-3) / 1e9 / roof['peak'], 4),
           'bench_frac': roof['frac']}
    print(json.dumps(out, indent=1))


def main():
    if sys.argv[1] == '--timed-syrk':
        return timed_syrk(sys.argv[2], sys.argv[3])
    if sys.argv[1] == '--timed-spmm':
        return timed_spmm(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
    path = sys.argv[1]
    window_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                         r['Kernel_Name'].split('(')[0].replace('gpmi::', '')))
    rows.sort()
    t_end = max(e for _, e, _ in rows)
    t0 = t_end - window_ms * 1e6 if window_ms > 0 else rows[0][0]
    rows = [r for r in rows if r[0] >= t0]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in rows:
        agg[n][0] += 1
        agg[n][1] += e - s
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - rows[0][0]
    print('window %.3f ms, busy union %.3f ms (%.3f)' % (span / 1e6, busy / 1e6, busy / span))
    for n, (c, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print('%-28s %7d %10.3f ms %9.2f us' % (n[:28], c, tot / 1e6, tot / c / 1e3))


if __name__ == '__main__':
    main()

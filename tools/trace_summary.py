"""Summarise a rocprofv3 --kernel-trace CSV (kernel_trace.csv): per-kernel
count / total / average device time over the last `window` of the trace (a
time window ending at the last dispatch, default: everything), and the union of
busy intervals (GPU-busy fraction) in that window."""
import csv
import sys
from collections import defaultdict


def main():
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

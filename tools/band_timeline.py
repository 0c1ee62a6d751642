"""Per-panel timeline of the band reduction from a rocprofv3 --kernel-trace CSV
(`bash tools/gpu.sh <name> trace-band`): the last reduction in the trace is
split at its SYMM launches (one per panel); for each requested panel the
kernels from that panel's SYMM start to the next one's are listed with their
start offset, duration and grid, and every panel's span is summarised.

    python tools/band_timeline.py <trace dir> [panel ...]
"""
import csv
import glob
import os
import sys


def load(trace_dir):
    files = glob.glob(os.path.join(trace_dir, '**', '*kernel_trace*.csv'), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r['Kernel_Name'].split('(')[0].replace('gpmi::', '').replace('void ', '')
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), name,
                             int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])),
                             int(r.get('Grid_Size_Y', 1))))
    rows.sort()
    return rows


def main():
    rows = load(sys.argv[1])
    want = [int(a) for a in sys.argv[2:]] or [10, 60, 110]
    symm = [i for i, r in enumerate(rows) if r[2] in ('symm_kernel', 'symm_bal_kernel')]
    # the last reduction: the SYMM launches between the last two cq_top_kernel
    # launches (one per reduction, after its panels)
    tops = [r[0] for r in rows if r[2] == 'cq_top_kernel']
    if tops:
        lo = tops[-2] if len(tops) > 1 else -1
        symm = [i for i in symm if lo < rows[i][0] < tops[-1]]
    npan = len(symm)
    t0 = rows[symm[0]][0]
    spans = []
    for j in range(npan):
        a = rows[symm[j]][0]
        b = rows[symm[j + 1]][0] if j + 1 < npan else max(r[1] for r in rows[symm[j]:])
        spans.append((b - a) / 1e3)
    print('panels %d, reduction span (first SYMM to last kernel) %.3f ms' %
          (npan, (max(r[1] for r in rows[symm[0]:]) - t0) / 1e6))
    for lo in range(0, npan, 16):
        print('  panels %3d-%3d: %s us' % (lo, min(npan, lo + 16) - 1,
                                           ' '.join('%.0f' % s for s in spans[lo:lo + 16])))
    for j in want:
        if j >= npan:
            continue
        a = rows[symm[j]][0]
        b = rows[symm[j + 1]][0] if j + 1 < npan else max(r[1] for r in rows[symm[j]:])
        print('\npanel %d (span %.1f us)' % (j, (b - a) / 1e3))
        for r in rows:
            if r[0] < a - 200e3 or r[0] >= b:
                continue
            if r[1] < a:
                continue
            print('  %8.1f %8.1f  %7.1f us  %-26s grid %d x %d' %
                  ((r[0] - a) / 1e3, (r[1] - a) / 1e3, (r[1] - r[0]) / 1e3, r[2][:26], r[3], r[4]))


if __name__ == '__main__':
    main()

"""Summarize rocprofv3 --pmc CSV passes per kernel (dev tool).

usage: python tools/pmc_summary.py OUT.json NOTE dir1 [dir2 ...]
PMC_FIRST=K (environment): also report, per kernel, the mean over its first K
dispatches of each pass ('per_dispatch_first'), e.g. the timed call of a run
that makes a second, differently sized call afterwards. PMC_MARKS=1: the mean over
the dispatches between the first two timing_mark_kernel launches of each pass
('per_dispatch_timed': bench.py's timed steps).
Each dir holds one pass's *_counter_collection.csv. Per kernel name (template
and argument list stripped) it reports dispatch count, the summed counter
values and the per-dispatch mean; FETCH_SIZE / WRITE_SIZE are in KB as
rocprofv3 reports them (gfx950: FETCH_SIZE counts half the bytes of wide
coalesced streaming reads, MI355X_MICROARCH.md "HBM").

When a pass holds SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE and
SQ_INSTS_VALU_MFMA_MOPS_F64 and a kernel trace sits beside the counters, it also
derives per kernel: mfma_busy_frac = MFMA busy cycles / (4 SIMDs x 256 CUs x
GRBM_GUI_ACTIVE / 8 XCDs), the effective clock GRBM_GUI_ACTIVE / 8 / kernel
time, and the executed fp64 MFMA rate (one MOPS = 512 flop)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.split('(')[0]


def main():
    out, note, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    first_k = int(os.environ.get('PMC_FIRST', '0'))
    rows_by = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for d in dirs:
        for f in glob.glob(os.path.join(d, '*counter_collection.csv')):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row['Kernel_Name'])
                    acc[k][row['Counter_Name']] += float(row['Counter_Value'])
                    disp[k].add((f, row['Dispatch_Id']))
                    rows_by[(f, k)][int(row['Dispatch_Id'])][row['Counter_Name']] += \
                        float(row['Counter_Value'])
    first = defaultdict(lambda: defaultdict(float))
    if first_k:
        for (f, k), by in rows_by.items():
            for did in sorted(by)[:first_k]:
                for c, v in by[did].items():
                    first[k][c] += v / first_k
    last_k = int(os.environ.get('PMC_LAST', '0'))   # the same over the last K dispatches
    last = defaultdict(lambda: defaultdict(float))
    if last_k:
        for (f, k), by in rows_by.items():
            for did in sorted(by)[-last_k:]:
                for c, v in by[did].items():
                    last[k][c] += v / last_k
    # PMC_MARKS=1: the mean over the dispatches between the first two timing_mark_kernel
    # dispatches of each pass (bench.py's timed steps, gpmi_sp_set_timing)
    timed = defaultdict(lambda: defaultdict(float))
    timed_n = {}
    if os.environ.get('PMC_MARKS'):
        files = {f for f, _ in rows_by}
        for f in files:
            marks = sorted(d for (g, k), by in rows_by.items() if g == f and
                           'timing_mark_kernel' in k for d in by)
            if len(marks) < 2:
                continue
            lo, hi = marks[0], marks[1]
            for (g, k), by in rows_by.items():
                if g != f:
                    continue
                ids = [d for d in by if lo < d < hi]
                if not ids:
                    continue
                timed_n[k] = len(ids)
                for d in ids:
                    for c, v in by[d].items():
                        timed[k][c] += v / len(ids)
    res = {'note': note, 'kernels': {}}
    for k, cs in acc.items():
        nd = max(1, len(disp[k]) // max(1, len(dirs)))
        res['kernels'][k] = {'dispatches': nd,
                             'sum': {c: v for c, v in sorted(cs.items())},
                             'per_dispatch': {c: v / nd for c, v in sorted(cs.items())}}
        if first_k and k in first:
            res['kernels'][k]['first_dispatches'] = first_k
            res['kernels'][k]['per_dispatch_first'] = dict(sorted(first[k].items()))
        if k in timed:
            res['kernels'][k]['timed_dispatches'] = timed_n[k]
            res['kernels'][k]['per_dispatch_timed'] = dict(sorted(timed[k].items()))
        if last_k and k in last:
            res['kernels'][k]['last_dispatches'] = last_k
            res['kernels'][k]['per_dispatch_last'] = dict(sorted(last[k].items()))
    times = defaultdict(float)
    for d in dirs:
        for f in glob.glob(os.path.join(d, '*kernel_trace.csv')):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    times[short(row['Kernel_Name'])] += (int(row['End_Timestamp']) -
                                                         int(row['Start_Timestamp'])) * 1e-9
    for k, v in res['kernels'].items():
        cs = v['sum']
        if times.get(k) and cs.get('GRBM_GUI_ACTIVE') and 'SQ_VALU_MFMA_BUSY_CYCLES' in cs:
            per_xcd = cs['GRBM_GUI_ACTIVE'] / 8.0
            v['derived'] = {
                'kernel_time_s': times[k],
                'effective_clock_ghz': per_xcd / times[k] / 1e9,
                'mfma_busy_frac': cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * 256 * per_xcd),
                'mfma_f64_tflops_executed': cs.get('SQ_INSTS_VALU_MFMA_MOPS_F64', 0.0) * 512 / times[k] / 1e12,
            }
    with open(out, 'w') as fh:
        json.dump(res, fh, indent=1)
    for k, v in res['kernels'].items():
        print(k, v['dispatches'], {c: '%.4g' % x for c, x in v['sum'].items()})


if __name__ == '__main__':
    main()

"""Per-dispatch MFMA counters of one kernel, grouped by grid size (dev tool).

usage: python tools/pmc_per_dispatch.py OUT.json KERNEL dir [dir ...]
Each dir holds one rocprofv3 --pmc pass with SQ_VALU_MFMA_BUSY_CYCLES,
SQ_INSTS_VALU_MFMA_MOPS_F64 and GRBM_GUI_ACTIVE (*_counter_collection.csv). Per
dispatch: mfma_busy_frac = busy cycles / (4 SIMDs x 256 CUs x GRBM_GUI_ACTIVE / 8
XCDs), the effective clock GRBM_GUI_ACTIVE / 8 / dispatch time and the executed
fp64 MFMA rate (one MOPS = 512 flop), as tools/pmc_summary.py derives them for a
whole kernel; then the mean per grid size (tools/fp64_peak's three occupancy
configurations, or the SYRK's launches)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, kname, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    disp = defaultdict(dict)
    for d in dirs:
        for f in glob.glob(os.path.join(d, '*counter_collection.csv')):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    base = row['Kernel_Name'].split('(')[0].split('<')[0].split(' ')[-1]
                    if base.split('::')[-1] != kname:
                        continue
                    key = (f, int(row['Dispatch_Id']))
                    r = disp[key]
                    r['grid'] = int(row['Grid_Size'])
                    r['t'] = (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) * 1e-9
                    r[row['Counter_Name']] = r.get(row['Counter_Name'], 0.0) + \
                        float(row['Counter_Value'])
    groups = defaultdict(list)
    for r in disp.values():
        if r['t'] <= 0 or 'GRBM_GUI_ACTIVE' not in r:
            continue
        gui = r['GRBM_GUI_ACTIVE'] / 8.0
        d = {'grid': r['grid'], 'time_ms': r['t'] * 1e3,
             'effective_clock_ghz': gui / r['t'] / 1e9}
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in r:
            d['mfma_busy_frac'] = r['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * 256 * gui)
        if 'SQ_INSTS_VALU_MFMA_MOPS_F64' in r:
            d['mfma_f64_tflops_executed'] = r['SQ_INSTS_VALU_MFMA_MOPS_F64'] * 512 / r['t'] / 1e12
        groups[r['grid']].append(d)
    res = {'kernel': kname, 'by_grid': {}}
    for g, ds in sorted(groups.items()):
        ds = [d for d in ds if d['time_ms'] > 1.0] or ds   # drop warm-up stubs
        mean = {k: sum(d[k] for d in ds) / len(ds) for k in ds[0] if k != 'grid'}
        res['by_grid'][str(g)] = dict(dispatches=len(ds), **{k: round(v, 4)
                                                             for k, v in mean.items()})
    # the long dispatches together (time-weighted): the batch-64 SYRK launches of the
    # dense step, or the microbenchmark's timed ones
    longd = [r for r in disp.values() if r['t'] > 5e-3 and 'GRBM_GUI_ACTIVE' in r]
    if longd:
        gui = sum(r['GRBM_GUI_ACTIVE'] for r in longd) / 8.0
        t = sum(r['t'] for r in longd)
        res['dispatches_over_5ms'] = {
            'dispatches': len(longd), 'time_ms': round(t * 1e3, 3),
            'effective_clock_ghz': round(gui / t / 1e9, 4),
            'mfma_busy_frac': round(sum(r.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0)
                                        for r in longd) / (4 * 256 * gui), 4),
            'mfma_f64_tflops_executed': round(sum(r.get('SQ_INSTS_VALU_MFMA_MOPS_F64', 0.0)
                                                  for r in longd) * 512 / t / 1e12, 3)}
    with open(out, 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()

"""Print rocprofv3 kernel_stats.csv compactly: name (args stripped), calls, total ms,
average us. usage: python tools/kstats.py <run_kernel_stats.csv> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:top]:
    name = r['Name'].split('(')[0].replace('gpmi::', '').replace('void ', '')
    print('%-40s %6s %10.3f ms %9.2f us' % (name[:40], r['Calls'], float(r['TotalDurationNs']) / 1e6,
                                          float(r['AverageNs']) / 1e3))

"""Per-kernel statistics (calls, total / average ns) from a rocprofv3 rocpd
SQLite database (the default output when no --output-format is given), and
the GPU-idle gaps between consecutive dispatches."""
import glob
import sqlite3
import sys
from collections import defaultdict


def load(db):
    con = sqlite3.connect(db)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith('rocpd_kernel_dispatch')][0]
    ks = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
    cols = [r[1] for r in cur.execute('pragma table_info(%s)' % ks)]
    namecol = 'display_name' if 'display_name' in cols else 'kernel_name'
    q = ('select k.start, k.end, s.%s from %s k join %s s on k.kernel_id = s.id order by k.start'
         % (namecol, kd, ks))
    return cur.execute(q).fetchall()


def main():
    db = sys.argv[1] if len(sys.argv) > 1 else glob.glob('gpurun_out/**/*.db', recursive=True)[0]
    rows = load(db)
    agg = defaultdict(lambda: [0, 0])
    for s, e, name in rows:
        short = name.split('(')[0]
        agg[short][0] += 1
        agg[short][1] += e - s
    tot = sum(v[1] for v in agg.values())
    for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print('%-45s calls=%6d total_ms=%9.3f avg_us=%9.2f  %5.1f%%' % (name[:45], c, t / 1e6,
                                                                    t / c / 1e3, 100.0 * t / tot))
    span = rows[-1][1] - rows[0][0]
    busy = 0
    last_end = rows[0][0]
    for s, e, _ in rows:
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    print('kernels %d, span %.3f ms, busy %.3f ms (%.1f%%)' % (len(rows), span / 1e6, busy / 1e6,
                                                          100.0 * busy / span))


if __name__ == '__main__':
    main()

"""The profile summaries the bench lines are checked against (tools/pmc_summary.py,
tools/trace_summary.py): the timed-window selection on synthetic rocprofv3 CSVs. CPU
only; the tools are test-side, like the committed summaries under profiles/."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
WING = 'void gpmi::csr_spmm_wing_kernel<12, 8, 4>(long const*, int const*)'
MARK = 'gpmi::timing_mark_kernel(int)'


def _write(path, fields, rows):
    with open(path, 'w', newline='') as fh:
        w = csv.DictWriter(fh, fieldnames=fields)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _run(args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([sys.executable] + args, cwd=REPO, env=e, check=True,
                          capture_output=True, text=True).stdout


def test_pmc_summary_timed_window(tmp_path):
    # dispatches: a wing launch before the marks (the reference check), two between the
    # first pair of marks (the timed step), one after them (an isolated launch)
    seq = [(1, WING, 100.0), (2, MARK, 0.0), (3, WING, 10.0), (4, WING, 20.0), (5, MARK, 0.0),
           (6, WING, 1000.0)]
    fields = ['Dispatch_Id', 'Kernel_Name', 'Counter_Name', 'Counter_Value']
    for c in ('FETCH_SIZE', 'WRITE_SIZE'):
        d = tmp_path / c
        d.mkdir()
        _write(d / 'run_counter_collection.csv', fields,
               [{'Dispatch_Id': i, 'Kernel_Name': k, 'Counter_Name': c,
                 'Counter_Value': v * (2 if c == 'WRITE_SIZE' else 1)} for i, k, v in seq])
    out = tmp_path / 'summ.json'
    _run(['tools/pmc_summary.py', str(out), 'note', str(tmp_path / 'FETCH_SIZE'),
          str(tmp_path / 'WRITE_SIZE')], {'PMC_MARKS': '1'})
    k = json.load(open(out))['kernels']['void gpmi::csr_spmm_wing_kernel<12, 8, 4>']
    assert k['timed_dispatches'] == 2
    assert k['per_dispatch_timed'] == {'FETCH_SIZE': 15.0, 'WRITE_SIZE': 30.0}
    assert k['dispatches'] == 4


def test_trace_summary_timed_spmm(tmp_path):
    # kernel trace: marks at t = 100 and 1000 ns; wing<12> launches inside (200-300,
    # 400-520) and outside (50-60, 2000-2500); a wing<20> launch inside is ignored
    fields = ['Kernel_Name', 'Start_Timestamp', 'End_Timestamp']
    rows = [(MARK, 100, 101), (WING, 200, 300), (WING, 400, 520), (MARK, 1000, 1001),
            (WING, 50, 60), (WING, 2000, 2500),
            ('void gpmi::csr_spmm_wing_kernel<20, 8, 4>(long const*)', 600, 900)]
    d = tmp_path / 'prof'
    d.mkdir()
    _write(d / 'run_kernel_trace.csv', fields,
           [{'Kernel_Name': k, 'Start_Timestamp': s, 'End_Timestamp': e} for k, s, e in rows])
    line = {'roofline': {'kernel': 'csr_spmm_wing_kernel (s=12 columns)', 'avg_launch_ms': 1.1e-4,
                         'in_step_by_width': {'12': {'launches': 2}},
                         'algorithmic_bytes_per_launch': 1.0e6, 'peak': 8000.0, 'frac': 0.1}}
    bj = tmp_path / 'bench.json'
    bj.write_text(json.dumps(line) + '\n')
    out = json.loads(_run(['tools/trace_summary.py', '--timed-spmm', str(d), str(bj)]))
    assert out['timed_launches_trace'] == 2
    assert abs(out['trace_avg_launch_ms'] - 1.1e-4) < 1e-12   # (100 + 120) / 2 ns
    assert abs(out['rel_diff_vs_bench']) < 1e-9

"""Print the headline numbers of a bench.py JSON line (dense default line or a
--config sparseN line): python tools/bench_summary.py <file.json>."""

import json
import sys


def main(path):
    with open(path) as fh:
        d = json.loads([l for l in fh if l.startswith('{')][-1])
    devs = d.get('devices') or []
    print('metric %s | value %.2f %s | n_gpus %s | ms/step %.2f | devices %s'
          % (d['metric'], d['value'], d['unit'], d['n_gpus'], d['ms_per_step'],
             [(x['rank'], x['device']) for x in devs]))
    r = d.get('roofline') or {}
    if r:
        print('roofline %s frac %s avg_launch_ms %s traffic %s'
              % (r.get('kernel'), r.get('frac'), r.get('avg_launch_ms'), r.get('traffic')))
    for k in ('logdet_rel_err_vs_reference', 'lp_rel_err_vs_reference', 'lp_sample'):
        if k in d:
            print(k, d[k])
    bm = d.get('band_mode')
    if bm:
        print('band %.1f evals/s reduce %s ms (frac %s) loglik %s ms'
              % (bm['value'], bm['reduce_ms'], bm['reduction_mfma_frac'], bm['loglik_ms']))
        if 'nu25_check' in bm:
            print('band nu25', bm['nu25_check'])
        if 'der1_sweep' in bm:
            print('der1', {k: bm['der1_sweep'].get(k) for k in ('wall_ms', 'device_ms', 'selected_inversion_ms')})
    ds = d.get('dense_slq_mode')
    if ds:
        print('dense slq', {k: ds[k] for k in ds if k != 'dense_mm'})
    for k, v in (d.get('sparse_modes') or {}).items():
        cb = v.get('cpu_baseline') or {}
        print('%s %.1f evals/s (n_gpus %s) ms %.2f spmm frac %s step frac %s cpu %s ref %s'
              % (k, v['value'], v.get('n_gpus'), v['ms_per_step'], v['roofline']['frac'],
                 v['step_roofline']['frac'], cb.get('value'), v.get('reference_check')))
    if 'step_roofline' in d:
        print('step frac', d['step_roofline']['frac'], 'ref', d.get('reference_check'))
    cb = d.get('cpu_baseline')
    if cb:
        print('cpu baseline %.4g %s on %s cores (%s)' % (cb['value'], cb['unit'], cb['cores'],
                                                         cb['kind']))


if __name__ == '__main__':
    main(sys.argv[1])

#!/usr/bin/env python
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
(ameli/gaussian-process-param-estimation v0.0.1) in the development container.

Recipe:
  1. copy /root/reference/gaussian_proc to a scratch dir under /tmp (never into
     the repo), cythonize its three .pyx modules there with the directives of the
     reference setup.py:993-999 (+ legacy_implicit_noexcept for speed only; the
     results are identical) and -O3 -fopenmp, language c++;
  2. install ``oracle.imate_exact`` (the restated exact imate methods; imate is
     unpinned in requirements.txt:5 and absent here) as module ``imate``;
  3. stub ``mpl_toolkits.axes_grid1.inset_locator.InsetPosition`` (removed in
     matplotlib 3.10, only used by plotting code);
  4. import the reference and its examples/_utilities/data_utilities.py, and
     record inputs/outputs as JSON / npz (allow_pickle=False) fixtures.

Outputs are data only (inputs and expected outputs). The reference never
travels with the repo. Run:  python tests/golden/make_golden.py [--big]
                             python tests/golden/make_golden.py --only <fixture>
"""

import argparse
import json
import os
import shutil
import subprocess
import sys
import textwrap

import numpy

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
SCRATCH = '/tmp/gp_ref_build'


def build_reference():
    pkg_dst = os.path.join(SCRATCH, 'pkg')
    gc_dir = os.path.join(pkg_dst, 'gaussian_proc', 'generate_correlation')
    if os.path.isdir(gc_dir) and any(f.endswith('.so') for f in os.listdir(gc_dir)):
        return pkg_dst
    if os.path.isdir(SCRATCH):
        shutil.rmtree(SCRATCH)
    os.makedirs(pkg_dst)
    shutil.copytree(os.path.join(REF, 'gaussian_proc'),
                    os.path.join(pkg_dst, 'gaussian_proc'))
    # The shipped sparse generator raises TypeError before doing any work
    # (SURVEY §0.4). Apply the two argument fixes to the SCRATCH copy only:
    #   :390  _ball_volume(geometric_mean_radius) -> (..., dimension)
    #   :542  _estimate_max_nnz(matrix_size, dimension, density)
    #         -> (matrix_size, correlation_scale, dimension, density)
    sp = os.path.join(pkg_dst, 'gaussian_proc', 'generate_correlation',
                      '_generate_sparse_correlation.pyx')
    src = open(sp).read()
    a = '_ball_volume(geometric_mean_radius)'
    assert src.count(a) == 1
    src = src.replace(a, '_ball_volume(geometric_mean_radius, dimension)')
    import re
    m = re.search(r'max_nnz = _estimate_max_nnz\(\s*matrix_size,\s*dimension,\s*density\)', src)
    assert m, 'estimate_max_nnz call site not found'
    src = src[:m.start()] + ('max_nnz = _estimate_max_nnz(matrix_size, correlation_scale, '
                             'dimension, density)') + src[m.end():]
    open(sp, 'w').write(src)
    setup_py = textwrap.dedent('''
        from setuptools import setup, Extension
        from Cython.Build import cythonize
        import numpy
        names = ['_kernels', '_generate_dense_correlation',
                 '_generate_sparse_correlation']
        exts = [Extension('gaussian_proc.generate_correlation.' + n,
                          ['gaussian_proc/generate_correlation/' + n + '.pyx'],
                          language='c++', include_dirs=[numpy.get_include()],
                          extra_compile_args=['-O3', '-fopenmp'],
                          extra_link_args=['-fopenmp'])
                for n in names]
        setup(ext_modules=cythonize(exts, language_level=3, compiler_directives={
            'boundscheck': False, 'wraparound': False, 'cdivision': True,
            'nonecheck': False, 'legacy_implicit_noexcept': True}))
    ''')
    with open(os.path.join(pkg_dst, 'setup.py'), 'w') as f:
        f.write(setup_py)
    subprocess.check_call([sys.executable, 'setup.py', 'build_ext', '--inplace'],
                          cwd=pkg_dst, stdout=subprocess.DEVNULL)
    return pkg_dst


def import_reference():
    pkg = build_reference()
    sys.path.insert(0, REPO)
    import oracle.imate_exact
    sys.modules['imate'] = oracle.imate_exact
    import matplotlib
    matplotlib.use('Agg')
    import mpl_toolkits.axes_grid1.inset_locator as il
    if not hasattr(il, 'InsetPosition'):
        il.InsetPosition = object
    sys.path.insert(0, pkg)
    sys.path.insert(0, os.path.join(REF, 'examples'))
    import gaussian_proc
    from gaussian_proc._mixed_correlation import MixedCorrelation
    from gaussian_proc._likelihood._direct_likelihood import DirectLikelihood
    from gaussian_proc._likelihood._profile_likelihood import ProfileLikelihood
    from gaussian_proc._likelihood import Likelihood
    from _utilities import data_utilities as du
    return dict(gp=gaussian_proc, MC=MixedCorrelation, DL=DirectLikelihood,
                PL=ProfileLikelihood, Likelihood=Likelihood, du=du)


def f(x):
    return float(x)


ETAS = [1e-3, 1e-1, 1.0, 10.0]
HYPERS = [[0.1, 0.2], [1.0, 0.1], [0.5, 0.05], [1.0, 1.0], [1e-9, 0.3]]
LOG_ETAS = [-1.0, 0.0, 1.0]


def sample_idx(n, k=64, seed=7):
    rng = numpy.random.RandomState(seed)
    return numpy.sort(rng.choice(n, size=min(k, n), replace=False))


def config_case(R, name, num_points, dim, nu, scale=0.1, full_arrays=False,
                optimize=False):
    du = R['du']
    pts = du.generate_points(num_points, dim, True)
    z = du.generate_data(pts, 0.2)
    X = du.generate_basis_functions(pts, 2)
    K = R['gp'].generate_correlation(pts, scale, nu, True)
    n, m = X.shape
    ii = sample_idx(n)
    jj = sample_idx(n, seed=11)
    out = dict(name=name, num_points=num_points, dimension=dim, nu=nu,
               correlation_scale=scale, n=n, m=m,
               K_sum=f(K.sum()), K_diag_sum=f(numpy.trace(K)),
               K_samples=dict(i=ii.tolist(), j=jj.tolist(),
                              v=K[ii, jj].tolist()),
               K_row_sums_sample=K.sum(axis=1)[ii].tolist(),
               z_sum=f(z.sum()), z_samples=z[ii].tolist(),
               X_col_sums=X.sum(axis=0).tolist(), sample_rows=ii.tolist())
    arrays = {}
    mcs = {'eigenvalue': R['MC'](K, imate_method='eigenvalue'),
           'cholesky': R['MC'](K, imate_method='cholesky')}
    ops = {}
    for meth, op in mcs.items():
        d = {}
        d['logdet'] = [f(op.logdet(e)) for e in ETAS]
        d['logdet_exp2'] = [f(op.logdet(e, exponent=2)) for e in ETAS[:2]]
        d['traceinv'] = [f(op.traceinv(e)) for e in ETAS]
        d['traceinv_exp2'] = [f(op.traceinv(e, exponent=2)) for e in ETAS]
        d['trace'] = {str(p): [f(op.trace(e, exponent=p)) for e in [0.0] + ETAS]
                      for p in (0, 1, 2)}
        ops[meth] = d
    out['etas'] = ETAS
    out['operator'] = ops
    op = mcs['eigenvalue']
    DL, PL = R['DL'], R['PL']
    out['hypers'] = HYPERS
    out['direct_lp'] = [f(DL.log_likelihood(z, X, op, False, h)) for h in HYPERS]
    out['direct_lp_chol'] = [f(DL.log_likelihood(z, X, mcs['cholesky'], False, h))
                             for h in HYPERS]
    out['direct_jac'] = [DL.log_likelihood_jacobian(z, X, op, False, h).tolist()
                         for h in HYPERS]
    out['direct_hess'] = [DL.log_likelihood_hessian(z, X, op, False, h).tolist()
                          for h in HYPERS]
    out['profile_hypers'] = [[0.1, 1.0], [1.0, 0.01], [0.3, 10.0]]
    out['profile_lp'] = [f(PL.log_likelihood(z, X, op, False, h))
                         for h in out['profile_hypers']]
    out['log_etas'] = LOG_ETAS
    out['profile_der1_eta'] = [f(PL.log_likelihood_der1_eta(z, X, op, le))
                               for le in LOG_ETAS]
    out['profile_der2_eta_etas'] = [0.1, 1.0]
    out['profile_der2_eta'] = [f(PL.log_likelihood_der2_eta(z, X, op, e))
                               for e in out['profile_der2_eta_etas']]
    # operator solve / dot samples
    w = op.solve(1.0, z)
    Y = op.solve(0.1, X)
    out['solve_eta1_z_samples'] = w[ii].tolist()
    out['solve_eta1_z_sum'] = f(w.sum())
    out['solve_eta01_X_colsums'] = Y.sum(axis=0).tolist()
    d2 = op.dot(0.5, z, exponent=2)
    out['dot_eta05_exp2_z_samples'] = d2[ii].tolist()
    out['dot_eta05_exp2_z_sum'] = f(d2.sum())
    if full_arrays:
        arrays['K'] = K
        arrays['solve_eta1_z'] = w
        arrays['solve_eta01_X'] = Y
        arrays['points'] = pts
        arrays['z'] = z
        arrays['X'] = X
    if optimize:
        import io
        import contextlib
        buf = io.StringIO()
        calls = []
        der1 = PL.log_likelihood_der1_eta

        def traced(z_, X_, K_, log_eta):
            v = der1(z_, X_, K_, log_eta)
            calls.append([f(log_eta), f(v)])
            return v
        with contextlib.redirect_stdout(buf):
            if optimize != 'profiled':
                rd = R['Likelihood'](X, K, 'direct').maximize_log_likelihood(z)
                out['maximize_direct'] = {k: f(v) for k, v in rd.items()}
            PL.log_likelihood_der1_eta = staticmethod(traced)
            try:
                rp = R['Likelihood'](X, K, 'profiled').maximize_log_likelihood(z)
            finally:
                PL.log_likelihood_der1_eta = staticmethod(der1)
        out['maximize_profiled'] = {k: (f(v) if not isinstance(v, bool) else v)
                                    for k, v in rp.items()}
        # the (log10 eta, der1) sequence the reference driver evaluated:
        # bracket search, then Chandrupatla (_profile_likelihood.py:244-350)
        out['maximize_profiled_der1_calls'] = calls
        out['maximize_profiled_bracket_found'] = 'Iter' in buf.getvalue()
    return out, arrays


def matern_cases(R):
    gp = R['gp']
    rng = numpy.random.RandomState(2024)
    cases = [(1, 0.1, 0.5), (2, 0.1, 1.5), (2, 0.25, 2.5), (3, 0.3, 1.5),
             (2, [0.1, 0.3], 1.5), (3, [0.2, 0.1, 0.4], 2.5), (2, 0.2, 3.2),
             (2, 0.2, 0.8), (2, 0.2, 150.0), (1, 0.05, 1.5)]
    arrays = {}
    meta = []
    for c, (d, scale, nu) in enumerate(cases):
        pts = rng.rand(48, d)
        if c == 0:
            pts[5] = pts[3]                     # duplicate point -> distance 0
        sc = numpy.array(scale, dtype=float) if isinstance(scale, list) else scale
        K = gp.generate_correlation(pts, sc, nu, grid=False)
        arrays['points_%d' % c] = pts
        arrays['K_%d' % c] = K
        meta.append(dict(case=c, dimension=d, correlation_scale=scale, nu=nu))
    return meta, arrays


def sparse_cases(R, big=False):
    """Tapered (sparse) Matérn from the reference generator + 2 arg fixes."""
    gp = R['gp']
    du = R['du']
    cases = [('sp2d_n1024', 32, 2, 0.05, 1.5, 0.02), ('sp3d_n1000', 10, 3, 0.1, 1.5, 0.03),
             ('sp2d_n4096_nu05', 64, 2, 0.02, 0.5, 0.005)]
    if big:
        cases.append(('sp2d_n65536_cfg4', 256, 2, 0.005, 1.5, 1e-3))
    meta, arrays = [], {}
    import io
    import contextlib
    for name, npts, d, rho, nu, dens in cases:
        pts = du.generate_points(npts, d, True)
        with contextlib.redirect_stdout(io.StringIO()):
            K = gp.generate_correlation(pts, rho, nu, True, sparse=True, density=dens)
        K = K.tocsr()
        K.sort_indices()
        meta.append(dict(name=name, num_points=npts, dimension=d, correlation_scale=rho,
                         nu=nu, density=dens, n=K.shape[0], nnz=int(K.nnz),
                         data_sum=float(K.data.sum()), min_kept=float(K.data.min()),
                         note='reference + 2 arg fixes (SURVEY 0.4)'))
        if K.shape[0] <= 4096:
            arrays[name + '_indptr'] = K.indptr.astype(numpy.int64)
            arrays[name + '_indices'] = K.indices.astype(numpy.int64)
            arrays[name + '_data'] = K.data
    return meta, arrays


class _SpluOperator(object):
    """Exact sparse K + eta I for the reference's likelihood code: logdet from
    scipy's SuperLU factor (sum log|U_ii|; K + eta I is SPD for the eta used),
    solve by the same factor. Stands in for imate's sparse Cholesky (CHOLMOD,
    absent here)."""

    def __init__(self, K):
        import scipy.sparse
        self.K = K.tocsc()
        self.n = K.shape[0]
        self.I = scipy.sparse.eye(self.n, format='csc')
        self._lu = {}

    def _factor(self, eta):
        import scipy.sparse.linalg
        if eta not in self._lu:
            self._lu = {eta: scipy.sparse.linalg.splu(self.K + eta * self.I,
                                                      permc_spec='COLAMD')}
        return self._lu[eta]

    def get_matrix_size(self):
        return self.n

    def logdet(self, eta, exponent=1):
        lu = self._factor(eta)
        d = lu.U.diagonal()
        assert numpy.all(d > 0) and numpy.all(lu.L.diagonal() == 1.0)
        return exponent * float(numpy.sum(numpy.log(d)))

    def solve(self, eta, Y):
        return self._factor(eta).solve(numpy.asarray(Y, dtype=float))


def sparse_big_case(R, name, npts, d, rho, nu, dens, etas_above, hypers=True):
    """A BASELINE sparse config at full size: the reference generator (+ the 2
    argument fixes) builds K; lambda_min by ARPACK; for eta above |lambda_min|
    the exact logdet and Gram [X z]^T (K + eta I)^-1 [X z] by SuperLU, and the
    reference DirectLikelihood.log_likelihood on that exact operator."""
    import io
    import contextlib
    import time
    import scipy.sparse.linalg
    du = R['du']
    pts = du.generate_points(npts, d, True)
    z = du.generate_data(pts, 0.2)
    X = du.generate_basis_functions(pts, 2)
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        K = R['gp'].generate_correlation(pts, rho, nu, True, sparse=True, density=dens)
    K = K.tocsr()
    K.sort_indices()
    t_asm = time.time() - t0
    n = K.shape[0]
    out = dict(name=name, num_points=npts, dimension=d, correlation_scale=rho, nu=nu,
               density=dens, n=n, m=X.shape[1], nnz=int(K.nnz),
               data_sum=float(K.data.sum()), min_kept=float(K.data.min()),
               diag_sum=float(K.diagonal().sum()), frob2=float(numpy.sum(K.data ** 2)),
               reference_assembly_s=t_asm, note='reference + 2 arg fixes (SURVEY 0.4)')
    ii = sample_idx(n)
    out['sample_rows'] = ii.tolist()
    out['row_sums_sample'] = numpy.asarray(K.sum(axis=1)).ravel()[ii].tolist()
    out['row_nnz_sample'] = numpy.diff(K.indptr)[ii].tolist()
    lam = scipy.sparse.linalg.eigsh(K, k=1, which='SA', tol=1e-8, return_eigenvectors=False)
    out['lambda_min'] = float(lam[0])
    if etas_above:
        shift = abs(min(0.0, float(lam[0])))
        etas = [shift + e for e in etas_above]
        op = _SpluOperator(K)
        Rm = numpy.column_stack([X, z])
        out['etas'] = etas
        out['logdet'] = []
        out['gram'] = []
        out['direct_lp'] = []
        for e in etas:
            out['logdet'].append(op.logdet(e))
            out['gram'].append((Rm.T @ op.solve(e, Rm)).tolist())
            # reference formula (_direct_likelihood.py:31-83) at sigma=1, sigma0=sqrt(eta)
            out['direct_lp'].append(f(R['DL'].log_likelihood(z, X, op, False,
                                                             [1.0, numpy.sqrt(e)])))
    return out


def big_case(R, nu=1.5):
    """N=16384 (2D 128x128 grid; nu=1.5 the metric's kernel, nu=2.5 BASELINE
    cfg3's): 'cholesky' imate method (3 dense factorizations per lp) — the
    eigenvalue method needs a 227 s eigh."""
    du = R['du']
    pts = du.generate_points(128, 2, True)
    z = du.generate_data(pts, 0.2)
    X = du.generate_basis_functions(pts, 2)
    K = R['gp'].generate_correlation(pts, 0.1, nu, True)
    op = R['MC'](K, imate_method='cholesky')
    etas = [0.01, 1.0, 4.0]
    out = dict(name='cfg3_n16384_nu%g' % nu, n=16384, m=X.shape[1], nu=nu,
               correlation_scale=0.1, K_sum=f(K.sum()),
               etas=etas, logdet=[f(op.logdet(e)) for e in etas],
               hypers=[[0.1, 0.2], [1.0, 0.1]])
    out['direct_lp'] = [f(R['DL'].log_likelihood(z, X, op, False, h))
                        for h in out['hypers']]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--big', action='store_true', help='also the N=16384 case (~5 min)')
    ap.add_argument('--sparse-only', action='store_true')
    ap.add_argument('--sparse-big', action='store_true', help='also config 4 (~5 min)')
    ap.add_argument('--only', default=None,
                    help='write only one fixture: cfg3_nu25 (~3 min), sparse_cfg4 (~10 min), '
                         'sparse_cfg5 (~90 min), sparse_3d32, n1024 or cfg2_profiled')
    args = ap.parse_args()
    if args.only:
        R = import_reference()
        if args.only == 'cfg3_nu25':
            out = big_case(R, 2.5)
        elif args.only == 'sparse_cfg4':
            out = sparse_big_case(R, 'cfg4_n65536_2d', 256, 2, 0.005, 1.5, 1e-3,
                                  [0.05, 0.5, 5.0])
        elif args.only == 'sparse_cfg5':
            out = sparse_big_case(R, 'cfg5_n262144_3d', 64, 3, 0.02, 1.5, 6e-4, [])
        elif args.only == 'sparse_3d32':
            # cfg5's 3-D stencil on a 32^3 grid (half the points per axis: rho and
            # density scaled so that a row keeps the same neighbours, nnz/row ~ 32),
            # small enough for SuperLU's exact logdet and Gram
            out = sparse_big_case(R, 'sparse3d_n32768', 32, 3, 0.04, 1.5, 4.8e-3,
                                  [0.05, 0.5, 5.0])
        elif args.only == 'n1024':
            out, _ = config_case(R, 'n1024_2d_nu2.5', 32, 2, 2.5, optimize=True)
            args.only = 'n1024_nu25'
        elif args.only == 'cfg2_profiled':
            out, _ = config_case(R, 'cfg2_n4096_2d', 64, 2, 1.5, optimize='profiled')
        else:
            raise SystemExit('unknown fixture %r' % args.only)
        with open(os.path.join(HERE, args.only + '.json'), 'w') as fh:
            json.dump(out, fh, indent=1)
        print('golden fixture written:', args.only)
        return
    R = import_reference()
    smeta, sarr = sparse_cases(R, args.sparse_big)
    numpy.savez_compressed(os.path.join(HERE, 'sparse_small.npz'), **sarr)
    with open(os.path.join(HERE, 'sparse.json'), 'w') as fh:
        json.dump(smeta, fh, indent=1)
    if args.sparse_only:
        return
    meta, arr = matern_cases(R)
    numpy.savez_compressed(os.path.join(HERE, 'matern_small.npz'), **arr)
    with open(os.path.join(HERE, 'matern_small.json'), 'w') as fh:
        json.dump(meta, fh, indent=1)
    c1, a1 = config_case(R, 'cfg1_n256_1d', 256, 1, 1.5, full_arrays=True,
                         optimize=True)
    numpy.savez_compressed(os.path.join(HERE, 'cfg1_arrays.npz'), **a1)
    with open(os.path.join(HERE, 'cfg1.json'), 'w') as fh:
        json.dump(c1, fh, indent=1)
    c2, _ = config_case(R, 'cfg2_n4096_2d', 64, 2, 1.5)
    with open(os.path.join(HERE, 'cfg2.json'), 'w') as fh:
        json.dump(c2, fh, indent=1)
    c25, _ = config_case(R, 'n1024_2d_nu2.5', 32, 2, 2.5, optimize=True)
    with open(os.path.join(HERE, 'n1024_nu25.json'), 'w') as fh:
        json.dump(c25, fh, indent=1)
    if args.big:
        with open(os.path.join(HERE, 'cfg3_big.json'), 'w') as fh:
            json.dump(big_case(R), fh, indent=1)
        with open(os.path.join(HERE, 'cfg3_nu25.json'), 'w') as fh:
            json.dump(big_case(R, 2.5), fh, indent=1)
    print('golden fixtures written to', HERE)


if __name__ == '__main__':
    main()

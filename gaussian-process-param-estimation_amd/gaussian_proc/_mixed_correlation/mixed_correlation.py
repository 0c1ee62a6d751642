"""The mixed-correlation operator K + eta I, device-resident.

Drop-in for ``MixedCorrelation`` of the reference
(gaussian_proc/_mixed_correlation/mixed_correlation.py:25-335). K lives in HBM
once per operator.

* imate_method='eigenvalue' (the reference's one-time eigh in __init__,
  :76-79, then cheap per-eta logdet, :239-248): the device reduces K once to
  band form K = Q B Q^T (bandwidth 128, csrc/gpmi_band.hip, on first use);
  logdet(eta) and the likelihood terms are then one banded Cholesky of
  B + eta I per eta. traceinv of exponent 1 and 2 comes from selected inversion
  of that factor (and its eta-tangent, gpmi_bcr.hip); trace / traceinv of other
  exponents are sums over the eigenvalues of B (= those of K; device bulge chase
  + bisection, computed once on first use, csrc/gpmi_chase.hip), as imate's
  'eigenvalue' method (:172-181), which also serves exponents 1 and 2 once the
  eigenvalues exist.
  solve(eta, Y) uses the dense Cholesky below.
* 'cholesky' (and 'hutchinson' for logdet, which the reference maps to
  Cholesky at :250-261): one fp64 MFMA Cholesky of K + eta I
  (csrc/gpmi_chol.hip), cached per eta so that logdet(eta) followed by
  solve(eta, .) factorizes once; exact traceinv from its device triangular
  inverse.
* 'hutchinson' traceinv (:193-203): Rademacher probes solved with the device
  Cholesky (stochastic; parity unpinned against imate, which is absent).
* 'slq' on a dense K: the same device Lanczos quadrature as on a sparse K,
  its products K X on fp64 MFMA over the resident dense K
  (_hip.SparseOperator.from_dense, dense_mm_kernel). The reference's branch
  passes the misspelt ``self.K_afm`` to imate (:141,207,266) and raises
  AttributeError; this is the estimator that branch names (parity unpinned:
  no reference value exists; tests check it against the exact logdet within
  the probes' standard error).
* sparse K: 'slq' (logdet / traceinv by device Lanczos quadrature) and
  'hutchinson' traceinv (CG solves); solve by device CG as the reference's
  linear_solver (_linear_solver.py:57-68). The exact methods ('cholesky', and
  'hutchinson' logdet, which the reference hands to imate's sparse Cholesky
  via CHOLMOD, :250-261; 'eigenvalue', whose eigh of a sparse K raises in the
  reference, :76-79) run the dense device paths above on a copy of K scattered
  from the CSR on the device (8 n_pad^2 bytes per copy: N = 65536 takes 34 GB
  of the 288 GB HBM).

``interpolate=True`` answers traceinv from an interpolant in eta built on the
exact values at ``interpolant_points`` (_interpolate.py; the reference's
imate.InterpolateTraceInv, :52-66,167-170; parity unpinned, imate is absent).

Error conventions follow the reference: ``ValueError`` for an unknown method
(:146,212,271) or a bad ``dot`` exponent (:323-326), ``TypeError`` for
``interpolate`` without points (:53-55), and ``numpy.linalg.LinAlgError`` when
K + eta I is not positive definite (scipy's posv behaviour).
"""

import numpy
import scipy.sparse

from .. import _hip
from .. import _slq
from ..generate_correlation.generate_correlation import DeviceCorrelation, \
    DeviceSparseCorrelation

__all__ = ['MixedCorrelation']

_METHODS = ('eigenvalue', 'cholesky', 'hutchinson', 'slq')

# The imate keyword options the reference forwards as **imate_options
# (mixed_correlation.py:133-143,183-209,241-268) to imate's trace / traceinv /
# logdet functions of each method; those functions take no other keywords, so
# any other key is a TypeError there (and here, at construction). The keys the
# reference passes itself (exponent, symmetric, eigenvalues, assume_matrix,
# parameters) are duplicates, a TypeError as well.
_IMATE_OPTIONS = {
    'eigenvalue': {'non_zero_ratio', 'tol'},
    'cholesky': {'cholmod', 'invert_cholesky'},
    'hutchinson': {'min_num_samples', 'max_num_samples', 'error_atol', 'error_rtol',
                   'confidence_level', 'outlier_significance_level', 'solver_tol',
                   'orthogonalize', 'num_threads', 'verbose', 'plot', 'seed'},
    'slq': {'min_num_samples', 'max_num_samples', 'error_atol', 'error_rtol',
            'confidence_level', 'outlier_significance_level', 'lanczos_degree', 'lanczos_tol',
            'orthogonalize', 'num_threads', 'num_gpu_devices', 'gpu', 'verbose', 'plot', 'seed'},
}
# this build's extensions ("imate options"): a fixed probe count,
# the CG tolerance of the sparse solves, and the bounds of the lanczos_tol control
_EXTENSIONS = {
    'hutchinson': {'num_samples', 'cg_rtol'},
    'slq': {'num_samples', 'cg_rtol', 'max_lanczos_degree', 'spectrum_lower_bound'},
}


def _next_degree(seen, tol):
    """The next Lanczos degree of the lanczos_tol search from the (degree, gap)
    pairs so far: twice the last degree, or, with two decreasing gaps, the degree
    where the line through their logarithms reaches tol (+10 %; the quadrature
    error decays at least geometrically in the degree, faster once the extreme
    Ritz values settle, so the line overshoots), at least 8 more steps."""
    m2, g2 = seen[-1]
    nxt = 2 * m2
    if len(seen) >= 2:
        m1, g1 = seen[-2]
        if 0.0 < g2 < g1 and m2 > m1:
            rate = (numpy.log(g1) - numpy.log(g2)) / float(m2 - m1)
            want = m2 + (numpy.log(g2) - numpy.log(tol)) / rate
            nxt = int(min(1e6, numpy.ceil(1.1 * want / 8.0) * 8))
    return max(m2 + 8, nxt)


def _check_options(method, options):
    """TypeError for a key imate's functions of ``method`` would not accept."""
    if method not in _IMATE_OPTIONS:
        return
    allowed = _IMATE_OPTIONS[method] | _EXTENSIONS.get(method, set())
    bad = sorted(k for k in (options or {}) if k not in allowed)
    if bad:
        raise TypeError("imate_options for imate_method='%s': unexpected keyword argument%s %s"
                        % (method, 's' if len(bad) > 1 else '', ', '.join(map(repr, bad))))


class MixedCorrelation(object):
    """K + eta I without forming sigma^2 K + sigma0^2 I."""

    def __init__(self, K, interpolate=False, interpolant_points=None,
                 imate_method='cholesky', imate_options={}, device=None, max_batch=None):
        self.interpolate = interpolate
        self.interpolant_points = interpolant_points
        self.imate_method = imate_method
        self.imate_options = imate_options
        _check_options(imate_method, imate_options)
        if self.interpolate:
            if self.interpolant_points is None:
                raise TypeError('When "interpolate" is set to "True", the '
                                '"interpolant_points" cannot be None.')
        self.interpolate_traceinv = None
        self.sparse = False
        if isinstance(K, DeviceSparseCorrelation) or scipy.sparse.issparse(K):
            self._init_sparse(K, device, max_batch)
            return
        self.sop = None
        if isinstance(K, DeviceCorrelation):
            if max_batch is not None and max_batch > K.op.max_batch:
                raise ValueError('DeviceCorrelation was created with max_batch=%d'
                                 % K.op.max_batch)
            self.K = K
            self.op = K.op
        else:
            if hasattr(K, 'toarray') and not isinstance(K, numpy.ndarray):
                raise NotImplementedError('sparse K is not implemented on the device yet')
            K = numpy.ascontiguousarray(K, dtype=float)
            if K.ndim != 2 or K.shape[0] != K.shape[1]:
                raise ValueError('K must be a square matrix')
            self.K = K
            self.op = _hip.Operator(K.shape[0], device=device, max_batch=max_batch or 1)
            self.op.load_matrix(K)
        self.n = self.op.n
        self._trace_cache = None
        self._rhs_cache = None
        self._band = None
        self._band_rhs = None
        self._eig = None
        self._slq_options()
        if self.imate_method == 'slq':
            # Krylov primitives over the resident dense K (dense_mm_kernel)
            self.sop = _hip.SparseOperator.from_dense(self.op)
        if self.interpolate:
            self._build_interpolant()

    def _slq_options(self):
        """The stochastic estimators' options ('slq', 'hutchinson'; INTEGRATION.md
        lists where the defaults differ from imate's)."""
        opts = dict(self.imate_options or {})
        self.num_samples = int(opts.get('num_samples', opts.get('max_num_samples', 20)))
        self.lanczos_degree = int(opts.get('lanczos_degree', 20))   # imate's default
        self.seed = int(opts.get('seed', 0) or 0)
        self.cg_rtol = float(opts.get('cg_rtol', opts.get('solver_tol', 1e-6)))
        # imate's Lanczos option, with imate's default 0 (the plain three-term
        # recurrence; -1 full reorthogonalisation, DCGS2 on the device; k > 0 the last
        # k vectors). The quadrature converges without reorthogonalisation (lost
        # orthogonality only duplicates converged Ritz values; cfg 4 / 5 logdet curves
        # equal to the reorthogonalised ones within 0.001 probe standard errors)
        self.orthogonalize = int(opts.get('orthogonalize', 0))
        if self.imate_method == 'hutchinson':
            # imate's Hutchinson option: orthogonalised probes (its default True)
            self.orthogonalize = bool(opts.get('orthogonalize', True))
        # imate's lanczos_tol: the Lanczos runs until the quadrature has converged
        # to this relative tolerance at the eta asked (the gap of the Gauss and
        # Gauss-Radau rules, _slq.bracket), its degree growing from lanczos_degree
        # (_next_degree) up to max_lanczos_degree (extension; 256, the device's
        # limit). None: the fixed lanczos_degree, as imate.
        tol = opts.get('lanczos_tol')
        self.lanczos_tol = None if tol is None else float(tol)
        self.max_lanczos_degree = max(self.lanczos_degree,
                                      min(256, int(opts.get('max_lanczos_degree', 256))))
        # the Gauss-Radau node: a lower bound of the spectrum of K (a dense
        # correlation matrix is positive semi-definite: 0; a sparse tapered K is
        # indefinite: its Gershgorin bound unless given)
        lb = opts.get('spectrum_lower_bound')
        self.spectrum_lower_bound = None if lb is None else float(lb)
        # imate's adaptive sample count (opt-in: any of its error options without
        # 'num_samples'): probes are added until the confidence-interval half width
        # z sigma / sqrt(k) of the estimate meets max(error_atol, error_rtol |mean|),
        # between min_num_samples and max_num_samples (imate's defaults 10, 50, 1e-2,
        # 0.95). Counter-based probes: the adaptive set is a prefix of the fixed one.
        # The probes it adds are kept apart from the fixed set (num_samples and
        # slq_nodes() do not change with earlier adaptive calls).
        self._adaptive = 'num_samples' not in opts and any(
            k in opts for k in ('min_num_samples', 'error_rtol', 'error_atol',
                                'confidence_level'))
        if self._adaptive:
            self.min_num_samples = int(opts.get('min_num_samples', 10))
            self.max_num_samples = max(self.min_num_samples,
                                       int(opts.get('max_num_samples', 50)))
            self.error_rtol = float(opts.get('error_rtol', 1e-2) or 0.0)
            self.error_atol = float(opts.get('error_atol', 0.0) or 0.0)
            self.confidence_level = float(opts.get('confidence_level', 0.95))
            self.num_samples = self.min_num_samples
        self._nodes = None
        self._lz = None            # (generation, degree, alpha, beta) of the fixed set
        self._extra = []           # adaptive probes beyond the fixed set: (alpha, beta)
        self.lanczos_degree_used = self.lanczos_degree

    def _build_interpolant(self):
        """imate.InterpolateTraceInv of the reference (mixed_correlation.py:52-66),
        restated in _interpolate.py (parity unpinned: imate is absent); its
        nodes are the operator's exact traceinv at the interpolant points."""
        from ._interpolate import InterpolateTraceInv
        interp, self.interpolate = self.interpolate, False   # exact values for the nodes
        try:
            self.interpolate_traceinv = InterpolateTraceInv(
                lambda t: self.traceinv(t, 1), self.n, self.trace(0.0, 1),
                self.interpolant_points)
        finally:
            self.interpolate = interp

    # ---- 'eigenvalue': one-time band reduction -----------------------------

    def eigenvalues(self):
        """Eigenvalues of K (ascending), the reference's K_eigenvalues
        (mixed_correlation.py:76-79): band form on the device, then bulge
        chasing to tridiagonal and bisection (computed once, on first use)."""
        if self._eig is None:
            self._eig = self.band().eigenvalues()
        return self._eig

    def band(self):
        """The one-time spectral setup of imate_method='eigenvalue' (the
        reference's eigh(K) in __init__, mixed_correlation.py:76-79), on the
        device: K = Q B Q^T with B banded (bandwidth 128), computed on first use.
        Afterwards logdet(eta) and the likelihood terms cost one banded Cholesky
        of B + eta I per eta (csrc/gpmi_band.hip)."""
        if self._band is None:
            self._band = _hip.Band(self._dense())
        return self._band

    def refresh_band(self, X=None, z=None):
        """Redo the one-time band reduction of K (same K: the timing form of the
        setup); with X, z the Q^T [X z] the likelihood terms need is applied
        during the reduction instead of after it."""
        b = self.band()
        self._der_cache = None
        if X is None:
            b.refresh()
            self._band_rhs = None
            return
        X = numpy.asarray(X, dtype=float)
        z = numpy.asarray(z, dtype=float)
        if X.shape[1] + 1 > _hip.MAX_RHS:
            raise ValueError('at most %d basis functions' % (_hip.MAX_RHS - 1))
        b.refresh(numpy.column_stack([X, z]))
        self._band_rhs = (X.copy(), z.copy())

    def _band_rhs_set(self, X, z):
        b = self.band()
        if X is not None:
            X = numpy.asarray(X, dtype=float)
            z = numpy.asarray(z, dtype=float)
            c = self._band_rhs
            if c is None or c[0].shape != X.shape or not numpy.array_equal(c[0], X) or \
                    not numpy.array_equal(c[1], z):
                if X.shape[1] + 1 > _hip.MAX_RHS:
                    raise ValueError('at most %d basis functions' % (_hip.MAX_RHS - 1))
                b.set_rhs(numpy.column_stack([X, z]))
                self._band_rhs = (X.copy(), z.copy())
        return b

    @staticmethod
    def _check_info(etas, info):
        if numpy.any(info):
            bad = int(numpy.flatnonzero(info)[0])
            raise numpy.linalg.LinAlgError(
                'K + eta I is not positive definite for eta = %r (pivot %d)'
                % (numpy.atleast_1d(etas)[bad], info[bad]))

    def _band_terms(self, etas, X=None, z=None):
        ld, g, info = self._band_rhs_set(X, z).loglik(etas)
        self._check_info(etas, info)
        return ld, g

    def der_terms(self, etas, X, z, traceinv=False):
        """The eigenvalue operator's eta-derivative terms: for each eta,
        logdet(K + eta I) and Gp = [X z]^T (K + eta I)^-p [X z] for p = 1, 2, 3,
        from one banded factorization and two more banded sweeps per eta
        (csrc/gpmi_band.hip, gpmi_bcr.hip). They replace the 2-5 dense solves
        per eta of ProfileLikelihood.log_likelihood_der1_eta / der2_eta
        (_profile_likelihood.py:91-192). Returns (logdet, G1, G2, G3); with
        ``traceinv`` (True or 1) also tr1 = trace((K + eta I)^-1) per eta,
        appended, and with ``traceinv=2`` tr1 and tr2 = trace((K + eta I)^-2):
        from the eigenvalues when they are already computed
        (mixed_correlation.py:172-181), else from the same cyclic-reduction factor
        on the device (gpmi_band_der_terms_ex2: selected inversion, and for tr2
        its eta-tangent), without the one-time eigenvalue chase."""
        if self.imate_method != 'eigenvalue':
            raise NotImplementedError('der_terms needs the eigenvalue operator')
        etas = numpy.atleast_1d(numpy.asarray(etas, dtype=float))
        want = 0 if not traceinv else (2 if traceinv == 2 else 1)
        b = self._band_rhs_set(X, z)
        c = getattr(self, '_der_cache', None)
        # the Jacobian and Hessian of one point ask for the same eta: reuse
        if c is not None and c[0] is self._band_rhs and c[1] is b and \
                numpy.array_equal(c[2], etas) and (c[5] >= want or self._eig is not None):
            res, trs = c[3], c[4]
        elif want and self._eig is None:
            out = b.der_terms(etas, traceinv=want)
            info = out[-1]
            self._check_info(etas, info)
            res, trs = out[:4], out[4:-1]
            self._der_cache = (self._band_rhs, b, etas.copy(), res, trs, want)
        else:
            ld, g1, g2, g3, info = b.der_terms(etas)
            self._check_info(etas, info)
            res, trs = (ld, g1, g2, g3), ()
            self._der_cache = (self._band_rhs, b, etas.copy(), res, trs, 0)
        if not want:
            return res
        if len(trs) < want:
            lam = self._eig
            trs = tuple(numpy.array([float(numpy.sum((lam + e) ** -float(p))) for e in etas])
                        for p in range(1, want + 1))
        return res + tuple(trs[:want])

    def _eig_traceinv(self, eta, exponent):
        """traceinv(eta, 1 or 2) on the 'eigenvalue' operator: the sums over the
        eigenvalues when they are already computed (imate 'eigenvalue',
        :172-181), else selected inversion of the cyclic-reduction factor of
        B + eta I (exponent 2: its eta-tangent) on the device, without the one-time
        eigenvalue chase. The choice depends only on whether eigenvalues() has run.
        A shift that leaves K + eta I indefinite takes the eigenvalue sums, as the
        reference's eigenvalue traceinv does (it never raises)."""
        if self._eig is None:
            tr, info = self.band().traceinv([eta], exponent)
            if not numpy.any(info):
                return float(tr[0])
        return float(numpy.sum((self.eigenvalues() + eta) ** (-float(exponent))))

    # ---- sparse K (tapered Matérn, CSR on the device) -------------------------

    def _init_sparse(self, K, device, max_batch):
        """Sparse K: logdet / traceinv by stochastic Lanczos quadrature
        ('slq'; one device Lanczos run per probe, cached, serves every eta) or
        Hutchinson ('hutchinson' traceinv, CG solves); solve by blocked CG with
        the reference's tolerance (_linear_solver.py:24,57-68: rtol 1e-6)."""
        self.sparse = True
        if isinstance(K, DeviceSparseCorrelation):
            self.K = K
            self.sop = K.op
        else:
            self.K = K.tocsr()
            self.sop = _hip.SparseOperator.from_csr(self.K, device=device)
        self.n = self.sop.n
        self.op = None            # dense copy of K for the exact methods (_dense)
        self._max_batch = max_batch
        self._trace_cache = None
        self._rhs_cache = None
        self._band = None
        self._band_rhs = None
        self._eig = None
        self._slq_options()
        if self.interpolate:
            self._build_interpolant()

    def _generation(self):
        return getattr(self.op, 'generation', 0) if not self.sparse else 0

    def _lower_bound(self):
        if self.spectrum_lower_bound is not None:
            return self.spectrum_lower_bound
        if not self.sparse:
            return 0.0
        Kc = self.sop.csr()
        off = numpy.asarray(abs(Kc).sum(axis=1)).ravel() - numpy.abs(Kc.diagonal())
        return float(numpy.min(Kc.diagonal() - off))

    def _lanczos(self, nprobe, degree, offset=0):
        return self.sop.lanczos(nprobe, degree, self.seed, probe_offset=offset,
                                orthogonalize=self.orthogonalize)

    def _fixed_lanczos(self, degree):
        """alpha / beta of the fixed probe set at ``degree`` (cached per K)."""
        c = self._lz
        if c is None or c[0] != self._generation() or c[1] != degree:
            a, b = self._lanczos(self.num_samples, degree)
            self._lz = (self._generation(), degree, a, b)
            self._nodes = None
            self._extra = []
        return self._lz[2], self._lz[3]

    def slq_nodes(self, etas=None, funcs=('logdet',)):
        """Ritz nodes of every probe of the fixed set (eta-independent; cached
        until K changes). With ``lanczos_tol`` set and ``etas`` given, the
        Lanczos degree is first raised (_next_degree, up to max_lanczos_degree) until
        the Gauss / Gauss-Radau gap of the probe-mean quadrature of each of
        ``funcs`` at min(etas) is within lanczos_tol (slq_converge)."""
        if etas is not None and self.lanczos_tol is not None:
            self.slq_converge(etas, funcs)
        a, b = self._fixed_lanczos(self.lanczos_degree_used)
        if self._nodes is None:
            self._nodes = _slq.nodes(a, b)
        return self._nodes

    def slq_converge(self, etas, funcs=('logdet',)):
        """imate's lanczos_tol on this operator: the Lanczos degree of the fixed
        probe set at which the quadrature of ``funcs`` (names of _slq.FUNCS or
        callables) has converged at min(etas) to lanczos_tol, relative (or the
        max_lanczos_degree cap). Returns dict(degree, bracket, converged)."""
        etas = numpy.atleast_1d(numpy.asarray(etas, dtype=float))
        e = [float(etas.min())]
        fns = [_slq.FUNCS[f] if isinstance(f, str) else f for f in funcs]
        lo = self._lower_bound()
        deg = self.lanczos_degree_used
        seen = []
        while True:
            a, b = self._fixed_lanczos(deg)
            g = _slq.nodes(a, b)
            _slq.check_shifts(_slq.min_ritz(g), e)
            node, rigorous = _slq.radau_node(lo, g, e)
            r = _slq.radau_nodes(a, b, node)
            gap = float(numpy.max([_slq.bracket(g, r, e, f)[0] for f in fns]))
            ok = gap <= self.lanczos_tol
            if ok or deg >= self.max_lanczos_degree:
                break
            seen.append((deg, gap))
            deg = min(self.max_lanczos_degree, _next_degree(seen, self.lanczos_tol))
        self.lanczos_degree_used = deg
        self._nodes = g
        self.last_slq_convergence = {'degree': deg, 'bracket': gap, 'converged': ok,
                                     'eta': e[0], 'radau_node': node,
                                     'rigorous_bound': rigorous}
        return self.last_slq_convergence

    def _slq(self, eta, what):
        fn = _slq.FUNCS[what] if isinstance(what, str) else what
        nodes = self.slq_nodes([eta], (fn,))
        q = self.n * _slq.quadrature(nodes, [eta], fn)[:, 0]
        if self._adaptive:
            import scipy.stats
            zc = float(scipy.stats.norm.ppf(0.5 * (1.0 + self.confidence_level)))
            deg = self.lanczos_degree_used
            extra = [x for x in self._extra if x[0] == deg]
            for _, a, b in extra:
                q = numpy.concatenate([q, self.n * _slq.quadrature(_slq.nodes(a, b), [eta],
                                                                   fn)[:, 0]])
            while True:
                k = q.size
                err = zc * q.std(ddof=1) / numpy.sqrt(k) if k > 1 else numpy.inf
                if err <= max(self.error_atol, self.error_rtol * abs(q.mean())) or \
                        k >= self.max_num_samples:
                    break
                more = min(self.max_num_samples - k, max(1, self.min_num_samples))
                a, b = self._lanczos(more, deg, offset=k)
                self._extra.append((deg, a, b))
                q = numpy.concatenate([q, self.n * _slq.quadrature(_slq.nodes(a, b), [eta],
                                                                   fn)[:, 0]])
        self.last_num_samples = int(q.size)
        return float(q.mean())

    def _probes(self, k, offset=0):
        """Hutchinson probes [n, k]: the counter-based Rademacher set, with imate's
        ``orthogonalize`` (default True) orthonormalised and scaled by sqrt(n)
        (Householder QR: the first columns do not depend on later ones, so a
        larger set extends a smaller one). The block depends only on (n, seed,
        column count), so it is built once and kept (traceinv is called once per
        eta): only a request for more columns than the cached block rebuilds it."""
        m = offset + k
        c = getattr(self, '_probe_cache', None)
        if c is None or c[0] != self.seed or c[1] != bool(self.orthogonalize) or \
                c[2].shape[1] < m:
            V = _slq.rademacher(self.n, m, self.seed)
            if self.orthogonalize and m <= self.n:
                Q, _ = numpy.linalg.qr(V)
                V = Q * numpy.sqrt(self.n)
            V.setflags(write=False)
            c = (self.seed, bool(self.orthogonalize), V)
            self._probe_cache = c
        return c[2][:, offset:m]

    def _hutchinson_traceinv(self, eta, exponent):
        """imate 'hutchinson' traceinv (:193-203): tr (K + eta I)^-p ~ mean_v
        v^T (K + eta I)^-p v, with u = (K + eta I)^-q v, q = floor(p / 2):
        |u|^2 for even p, u^T (K + eta I)^-1 u for odd p, so ceil(p / 2) solves
        per probe (device Cholesky solves with the factor cached per eta, or CG on
        a sparse K); a negative p takes products instead."""
        if float(exponent) != int(exponent):
            raise ValueError('"exponent" should be an integer.')
        p = int(exponent)
        if p == 0:
            return float(self.n)

        def solve(W):
            return self.sop.cg(eta, W, rtol=self.cg_rtol) if self.sparse else \
                self.op.solve(eta, W)

        def apply(W):
            KW = self.sop.spmm(0.0, W) if self.sparse else self.op.matvec(W)
            return KW + eta * W

        def estimates(V):
            step = solve if p > 0 else apply
            U = V
            for _ in range(abs(p) // 2):
                U = step(U)
            W = step(U) if abs(p) % 2 else U
            return numpy.sum(U * W, axis=0)

        if not self._adaptive:
            self.last_num_samples = self.num_samples
            return float(numpy.mean(estimates(self._probes(self.num_samples))))
        import scipy.stats
        zc = float(scipy.stats.norm.ppf(0.5 * (1.0 + self.confidence_level)))
        q = estimates(self._probes(self.min_num_samples))
        while q.size < self.max_num_samples:
            err = zc * q.std(ddof=1) / numpy.sqrt(q.size) if q.size > 1 else numpy.inf
            if err <= max(self.error_atol, self.error_rtol * abs(q.mean())):
                break
            more = min(self.max_num_samples - q.size, max(1, self.min_num_samples))
            q = numpy.concatenate([q, estimates(self._probes(more, q.size))])
        self.last_num_samples = int(q.size)
        return float(q.mean())

    def _sparse_traces(self):
        if self._trace_cache is None:
            Kc = self.sop.csr()
            self._trace_cache = (float(Kc.diagonal().sum()), float(numpy.sum(Kc.data ** 2)))
        return self._trace_cache

    def _dense(self):
        """The dense device operator the exact methods run on: K itself, or
        for a sparse K a dense copy scattered from its CSR on the device (created
        on first use). imate factorizes a sparse K with CHOLMOD (absent here);
        the dense fp64 MFMA Cholesky gives the same exact values."""
        if self.op is None:
            op = _hip.Operator(self.n, device=self.sop.device,
                               max_batch=self._max_batch or 1)
            op.load_sparse(self.sop)
            self.op = op
        return self.op

    # ---- reference duck type -------------------------------------------------

    def get_matrix_size(self):                                     # :85-90
        return self.n

    def _traces(self):
        if self.sparse:
            return self._sparse_traces()
        if self._trace_cache is None:
            self._trace_cache = self.op.trace()
        return self._trace_cache

    def trace(self, eta, exponent=1):                              # :96-149
        if exponent == 0:
            return float(self.n)
        if exponent == 1:
            t = self._traces()[0]
            if eta != 0:
                t += eta * self.n
            return t
        if exponent == 2:
            tk, tk2 = self._traces()
            if eta == 0:
                return tk2
            return tk2 + 2.0 * eta * tk + eta ** 2 * self.n
        if self.imate_method == 'eigenvalue':
            # sum over the eigenvalues (imate 'eigenvalue', :127-133)
            return float(numpy.sum((self.eigenvalues() + eta) ** float(exponent)))
        if self.imate_method == 'slq':
            # tr (K + eta I)^p ~ n E[e1^T f(T) e1], f(x) = x^p (imate.trace, 'slq')
            p = float(exponent)
            return self._slq(eta, lambda x: x ** p)
        raise ValueError('Existing methods are "exact", "eigenvalue", and "slq".')

    def traceinv(self, eta, exponent=1):                           # :155-215
        if self.interpolate:
            # :167-170: the interpolant of tr((K + eta I)^-1), whatever the exponent
            return self.interpolate_traceinv.interpolate(eta)
        if self.imate_method == 'slq' and self.sop is not None:
            if exponent == 0:
                return float(self.n)
            if exponent in (1, 2):
                return self._slq(eta, 'traceinv' if exponent == 1 else 'traceinv2')
            p = float(exponent)
            return self._slq(eta, lambda x: x ** -p)
        if self.imate_method == 'hutchinson':
            # Hutchinson estimator (imate 'hutchinson', assume_matrix='sym_pos')
            return self._hutchinson_traceinv(eta, exponent)
        if self.imate_method not in ('eigenvalue', 'cholesky'):
            raise ValueError('Existing methods are "eigenvalue", "cholesky,"'
                             '"hutchinson", and "slq".')
        if exponent == 0:
            return float(self.n)
        if self.imate_method == 'eigenvalue':
            # sum over the eigenvalues (imate 'eigenvalue', :172-181); exponents 1
            # and 2 by selected inversion unless the eigenvalues exist (_eig_traceinv)
            if exponent in (1, 2):
                return self._eig_traceinv(eta, exponent)
            return float(numpy.sum((self.eigenvalues() + eta) ** (-float(exponent))))
        if exponent in (1, 2):
            # exact, from the device triangular inverse of the cached factor
            return self._dense().traceinv(eta, exponent)
        # higher powers (not used by the likelihoods): columns of A^-1 solved on the device
        Ainv = self._dense().solve(eta, numpy.eye(self.n))
        return float(numpy.trace(numpy.linalg.matrix_power(Ainv, exponent)))

    def logdet(self, eta, exponent=1):                             # :221-274
        if self.imate_method == 'slq' and self.sop is not None:
            return exponent * self._slq(eta, 'logdet')
        if self.imate_method not in ('eigenvalue', 'cholesky', 'hutchinson'):
            raise ValueError('Existing methods are "eigenvalue", "cholesky",'
                             ' and "slq".')
        if self.imate_method == 'eigenvalue':
            return exponent * float(self._band_terms([eta])[0][0])
        return exponent * self._dense().logdet(eta)

    def solve(self, eta, Y):                                       # :280-299
        if self.sparse:
            return self.sop.cg(eta, Y, rtol=self.cg_rtol)
        return self.op.solve(eta, Y)

    def dot(self, eta, x, exponent=1):                             # :305-335
        if not isinstance(exponent, int):
            raise ValueError('"exponent" should be an integer.')
        elif exponent < 0:
            raise ValueError('"exponent" should be a non-negative integer.')
        y = numpy.zeros_like(x, dtype=float)
        if exponent == 0:
            return y
        Kx = self.sop.spmm(0.0, x) if self.sparse else self.op.matvec(x)
        for _ in range(exponent):
            y += Kx
            if eta != 0:
                y += eta * x
        return y

    # ---- fused hot path (extension) -----------------------------------------

    def set_rhs(self, X, z):
        """Make [X | z] the resident RHS block (skipped if unchanged)."""
        X = numpy.asarray(X, dtype=float)
        z = numpy.asarray(z, dtype=float)
        c = self._rhs_cache
        if c is not None and c[0].shape == X.shape and numpy.array_equal(c[0], X) and \
                numpy.array_equal(c[1], z):
            return
        if X.shape[1] + 1 > _hip.MAX_RHS:
            raise ValueError('at most %d basis functions' % (_hip.MAX_RHS - 1))
        self.op.set_rhs(numpy.column_stack([X, z]))
        self._rhs_cache = (X.copy(), z.copy())

    def loglik_terms(self, etas, X, z):
        """For each eta: logdet(K + eta I) and G = [X z]^T (K + eta I)^-1 [X z]
        from ONE Cholesky per eta, batched over up to ``max_batch`` etas per
        device call. Returns (logdet[neta], G[neta, m+1, m+1])."""
        etas = numpy.atleast_1d(numpy.asarray(etas, dtype=float))
        if self.sparse and self.imate_method == 'slq':
            # SLQ logdet per eta (cached Ritz nodes) and all Gram blocks from one
            # multi-shift CG on K + min(eta) I (tolerance as _linear_solver.py:24)
            R = numpy.column_stack([numpy.asarray(X, dtype=float), numpy.asarray(z, dtype=float)])
            lds = numpy.array([self.logdet(e) for e in etas])
            return lds, self.sop.msgram(etas, R, rtol=self.cg_rtol)
        if self.imate_method == 'eigenvalue':
            return self._band_terms(etas, X, z)
        self._dense()
        self.set_rhs(X, z)
        if self.imate_method == 'slq':
            # dense K: SLQ logdet (imate 'slq') and the exact Gram blocks of the
            # dense solve the reference pairs it with (_linear_solver.py:71)
            lds = numpy.array([self.logdet(e) for e in etas])
            return lds, self._exact_terms(etas)[1]
        return self._exact_terms(etas)

    def _exact_terms(self, etas):
        lds, gs = [], []
        mb = self.op.max_batch
        for i in range(0, etas.size, mb):
            ld, g, info = self.op.loglik_batch(etas[i:i + mb])
            if numpy.any(info):
                bad = int(numpy.flatnonzero(info)[0])
                raise numpy.linalg.LinAlgError(
                    'K + eta I is not positive definite for eta = %r (pivot %d)'
                    % (etas[i + bad], info[bad]))
            lds.append(ld)
            gs.append(g)
        return numpy.concatenate(lds), numpy.concatenate(gs)

"""Scalar bracketing and Chandrupatla root finding (host-side drivers).

Restates the reference's gaussian_proc/_likelihood/_root_finding.py:
  find_interval_with_sign_change  :21-148  (midpoint probe, then one outward step)
  chandrupatla_method             :155-309 (IQI / bisection hybrid)
The decision rules and return values match the reference for scalar f; the
per-iteration diagnostic prints of the bracket search are kept.

``BatchedFunction`` + ``find_interval_with_sign_change_batched`` evaluate the
same bracket search with every point it may need next requested in ONE batched
call (the device evaluates many eta per call at almost the cost of one): per
trial the midpoint and the one outward probe the current |f0|, |f1| select, and
up front also the first Chandrupatla point of the initial bracket. Function
values do not depend on the batch they are computed in (one device workgroup
per eta), so the decisions, the returned bracket and the root are identical to
the sequential reference driver.
"""

import numpy

__all__ = ['find_interval_with_sign_change', 'chandrupatla_method', 'BatchedFunction',
           'find_interval_with_sign_change_batched']


class BatchedFunction(object):
    """Scalar view f(x) of a batched function fb(xs) -> values, memoised by the
    exact float x. ``request(xs, speculative)`` evaluates the missing points of
    xs, plus the missing speculative points, in one call of fb (speculative
    points only up to ``spec_budget`` points per call, required ones included:
    the band operator's default 64 keeps every call on its cyclic-reduction
    path, gpmi_band_der_terms' limit; 0 turns speculation off); ``f(x)``
    returns a cached value or evaluates x alone. ``calls`` counts the batched
    calls, ``points`` the evaluated points.

    Speculative points are ones the sequential reference may never evaluate
    (an outward bracket probe, a candidate of the next Chandrupatla step). A
    speculative point must not change what the caller sees: when the combined
    call raises (``LinAlgError``: K + eta I not positive definite at one of the
    speculative eta) the required points are evaluated again on their own, and
    a non-finite speculative value is not memoised (a later request evaluates
    it as a required point, so any error it causes surfaces where the
    reference's would)."""

    def __init__(self, fb, spec_budget=64):
        self.fb = fb
        self.spec_budget = spec_budget
        self.memo = {}
        self.calls = 0
        self.points = 0
        self.max_points = 0
        self.spec_failures = 0

    def _missing(self, xs, skip=()):
        miss = []
        for x in xs:
            x = float(x)
            if x not in self.memo and x not in miss and x not in skip:
                miss.append(x)
        return miss

    def _eval(self, miss):
        vals = self.fb(numpy.array(miss))
        self.calls += 1
        self.points += len(miss)
        self.max_points = max(self.max_points, len(miss))
        return [float(v) for v in vals]

    def request(self, xs, speculative=()):
        miss = self._missing(xs)
        spec = self._missing(speculative, skip=miss)[:max(0, self.spec_budget - len(miss))]
        if not miss:
            # nothing is needed yet: prefetching alone would be a call the
            # reference does not make
            return
        if spec:
            try:
                vals = self._eval(miss + spec)
            except numpy.linalg.LinAlgError:
                self.spec_failures += 1
                vals = None
            if vals is not None:
                for x, v in zip(miss, vals[:len(miss)]):
                    self.memo[x] = v
                for x, v in zip(spec, vals[len(miss):]):
                    if numpy.isfinite(v):
                        self.memo[x] = v
                return
        for x, v in zip(miss, self._eval(miss)):
            self.memo[x] = v

    def __call__(self, x, *args):
        x = float(x)
        if x not in self.memo:
            self.request([x])
        return self.memo[x]


def _mid(x0, x1):
    return x0 * (1.0 - 0.5) + x1 * 0.5


def _outward(x0, x1, f0, f1):
    t = 1.5 if numpy.abs(f0) > numpy.abs(f1) else -0.5
    return x0 * (1.0 - t) + x1 * t


def find_interval_with_sign_change_batched(fb, bracket, num_bracket_trials, tol=None):
    """find_interval_with_sign_change (:21-148) with batched evaluations.
    ``fb`` is a BatchedFunction. Call 1: x0, x1, and speculatively the first
    trial's midpoint, both of its possible outward probes and the first
    Chandrupatla point (:155-309, t = 0.5 from a = x1) of [x0, x1] (with
    ``tol``, the Chandrupatla eps_m = eps_a, also the candidate tree that
    follows it, _chandrupatla_candidates); each later
    trial: its midpoint, and its outward probe speculatively."""
    x0, x1 = float(bracket[0]), float(bracket[1])
    xm = _mid(x0, x1)
    spec = [xm, x0 * (1.0 - 1.5) + x1 * 1.5, x0 * (1.0 + 0.5) + x1 * -0.5]
    xt = x1 + 0.5 * (x0 - x1)
    spec.append(xt)
    if tol is not None:
        spec += _chandrupatla_candidates(x1, x0, x1, xt, tol, tol,
                                         max(0, fb.spec_budget - len(spec) - 2))
    fb.request([x0, x1], speculative=spec)

    def f(x):
        return fb(x)
    f0, f1 = f(x0), f(x1)
    for it in range(1, num_bracket_trials + 1):
        if numpy.sign(f0) != numpy.sign(f1):
            return True, [x0, x1], [f0, f1]
        xm = _mid(x0, x1)
        fb.request([xm], speculative=[_outward(x0, x1, f0, f1)])
        print('bracket was not found. Search for bracket. Iteration: %d' % it)
        print('x0: %0.2f, f0: %0.16f' % (x0, f0))
        print('x1: %0.2f, f1: %0.16f' % (x1, f1))
        fm = f(xm)
        print('x_new: %0.2f, f_new: %0.16f' % (xm, fm))
        left_smaller = numpy.abs(f0) < numpy.abs(f1)
        if numpy.sign(f0) != numpy.sign(fm):
            if left_smaller:
                return True, [x0, xm], [f0, fm]
            return True, [xm, x1], [fm, f1]
        if numpy.abs(fm) < min(numpy.abs(f0), numpy.abs(f1)):
            if left_smaller:
                x1, f1 = xm, fm
            else:
                x0, f0 = xm, fm
            continue
        right = numpy.abs(f0) > numpy.abs(f1)
        xo = _outward(x0, x1, f0, f1)
        fo = f(xo)
        if numpy.sign(f0) != numpy.sign(fo):
            if right:
                return True, [xo, x0], [fo, f0]
            return True, [x1, xo], [f1, fo]
        if right:
            x0, f0, x1, f1 = x1, f1, xo, fo
        else:
            x1, f1, x0, f0 = x0, f0, xo, fo
    return False, [x0, x1], [f0, f1]


def find_interval_with_sign_change(f, bracket, num_bracket_trials, args=()):
    x0, x1 = bracket[0], bracket[1]
    f0, f1 = f(x0, *args), f(x1, *args)
    for it in range(1, num_bracket_trials + 1):
        if numpy.sign(f0) != numpy.sign(f1):
            return True, [x0, x1], [f0, f1]
        print('bracket was not found. Search for bracket. Iteration: %d' % it)
        print('x0: %0.2f, f0: %0.16f' % (x0, f0))
        print('x1: %0.2f, f1: %0.16f' % (x1, f1))
        xm = _mid(x0, x1)
        fm = f(xm, *args)
        print('x_new: %0.2f, f_new: %0.16f' % (xm, fm))
        left_smaller = numpy.abs(f0) < numpy.abs(f1)
        if numpy.sign(f0) != numpy.sign(fm):
            if left_smaller:
                return True, [x0, xm], [f0, fm]
            return True, [xm, x1], [fm, f1]
        if numpy.abs(fm) < min(numpy.abs(f0), numpy.abs(f1)):
            # shrink toward the side with the smaller |f|
            if left_smaller:
                x1, f1 = xm, fm
            else:
                x0, f0 = xm, fm
            continue
        # probe one half-width outside, on the side of the smaller |f|
        right = numpy.abs(f0) > numpy.abs(f1)
        t = 1.5 if right else -0.5
        xo = x0 * (1.0 - t) + x1 * t
        fo = f(xo, *args)
        if numpy.sign(f0) != numpy.sign(fo):
            if right:
                return True, [xo, x0], [fo, f0]
            return True, [x1, xo], [f1, fo]
        if right:
            x0, f0, x1, f1 = x1, f1, xo, fo
        else:
            x1, f1, x0, f0 = x0, f0, xo, fo
    return False, [x0, x1], [f0, f1]


def _chandrupatla_candidates(a, b, c, xt, eps_m, eps_a, budget):
    """Points later iterations of chandrupatla_method can evaluate whatever
    f(xt) turns out to be, except interior inverse-quadratic ones, breadth
    first (at most ``budget``). For either sign of f(xt) (which fixes the new
    b, c) and either of the new a = xt, b as the smaller-|f| end xm (which
    fixes tlim): the bisection point t = 0.5 and the two clamped steps
    t = tlim, 1 - tlim, each formed by the same float expression as the
    iteration itself (a + t (b - a)); then the same from each of those points.
    The bracketing chain of the first iterations is bisections, and near the
    root every step is clamped, so these cover most non-IQI iterations."""
    out, seen = [], set()
    level = [(a, b, c, xt)]
    while level and len(out) < budget:
        nxt = []
        for a0, b0, c0, x0 in level:
            for same in (True, False):
                bn, cn = (b0, a0) if same else (a0, b0)
                for xm in (x0, bn):
                    tol = 2 * eps_m * numpy.abs(xm) + eps_a
                    tlim = tol / numpy.abs(bn - cn)
                    if not tlim <= 0.5:
                        continue
                    for t in (0.5, tlim, 1 - tlim):
                        t = min(1 - tlim, max(tlim, t))
                        xn = x0 + t * (bn - x0)
                        if float(xn) in seen:
                            continue
                        seen.add(float(xn))
                        out.append(xn)
                        nxt.append((x0, bn, cn, xn))
        level = nxt
    return out[:budget]


def chandrupatla_method(f, bracket, bracket_values, verbose=False, eps_m=None, eps_a=None,
                        maxiter=50, args=()):
    b, a = float(bracket[0]), float(bracket[1])
    if bracket_values is None:
        fa, fb = f(a, *args), f(b, *args)
    else:
        fa, fb = bracket_values[1], bracket_values[0]
    assert numpy.sign(fa) * numpy.sign(fb) <= 0
    c, fc = a, fa
    eps = numpy.finfo(float).eps
    eps_m = eps if eps_m is None else eps_m
    eps_a = 2 * eps if eps_a is None else eps_a
    t = 0.5
    iterations = 0
    xm = b
    # speculative candidates beside the one required point xt per call
    budget = getattr(f, 'spec_budget', 0) - 1 if isinstance(f, BatchedFunction) and not args \
        else 0
    while maxiter > 0:
        maxiter -= 1
        xt = a + t * (b - a)
        if budget > 0 and float(xt) not in f.memo:
            f.request([xt], speculative=_chandrupatla_candidates(a, b, c, xt, eps_m, eps_a,
                                                                 budget))
        ft = f(xt, *args)
        if numpy.sign(ft) == numpy.sign(fa):
            c, fc = a, fa
        else:
            c, fc = b, fb
            b, fb = a, fa
        a, fa = xt, ft
        if numpy.abs(fa) < numpy.abs(fb):
            xm, fm = a, fa
        else:
            xm, fm = b, fb
        tol = 2 * eps_m * numpy.abs(xm) + eps_a
        tlim = tol / numpy.abs(b - c)
        if verbose:
            print('xt=%r ft=%r fm=%r tlim=%r' % (xt, ft, fm, tlim))
        if fm == 0 or tlim > 0.5:
            break
        iterations += 1
        xi = (a - b) / (c - b)
        phi = (fa - fb) / (fc - fb)
        if phi ** 2 < xi and (1 - phi) ** 2 < 1 - xi:
            t = fa / (fb - fa) * fc / (fb - fc) + (c - a) / (b - a) * fa / (fc - fa) * fb / (fc - fb)
        else:
            t = 0.5
        t = min(1 - tlim, max(tlim, t))
    return {'root': xm, 'iterations': iterations}

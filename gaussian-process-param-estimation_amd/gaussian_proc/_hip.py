"""ctypes binding of libgpmi.so (the C ABI declared in include/gpmi.h).

There is no CPU fallback: if the library (built for gfx950 by
``__graft_entry__.build()``) is missing, or no HIP device is visible when a
device call is made, the call raises. The CPU restatement lives in
``oracle/`` and is test infrastructure only.
"""

import ctypes
import os

import numpy

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), '_lib')
# GPMI_LIB_VARIANT=<name> loads _lib/libgpmi_<name>.so instead (kernel experiments)
LIB_PATH = os.path.join(_LIB_DIR, 'libgpmi%s.so' % (
    '_' + os.environ['GPMI_LIB_VARIANT'] if os.environ.get('GPMI_LIB_VARIANT') else ''))
MAX_RHS = 16

_lib = None

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int_p = ctypes.POINTER(ctypes.c_int)
c_i64 = ctypes.c_int64
c_op_p = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/gpmi.h
SIGNATURES = {
    'gpmi_version': (ctypes.c_int, []),
    'gpmi_last_error': (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    'gpmi_device_count': (ctypes.c_int, [c_int_p]),
    'gpmi_matern_dense': (ctypes.c_int, [ctypes.c_int, c_double_p, c_i64, ctypes.c_int,
                                         c_double_p, ctypes.c_double, c_double_p, c_i64]),
    'gpmi_op_create': (ctypes.c_int, [ctypes.c_int, c_i64, ctypes.c_int,
                                      ctypes.POINTER(c_op_p)]),
    'gpmi_op_destroy': (ctypes.c_int, [c_op_p]),
    'gpmi_op_size': (ctypes.c_int, [c_op_p, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    'gpmi_op_load_matrix': (ctypes.c_int, [c_op_p, c_double_p, c_i64]),
    'gpmi_op_load_sparse': (ctypes.c_int, [c_op_p, c_op_p]),
    'gpmi_op_assemble_matern': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p,
                                               ctypes.c_double]),
    'gpmi_op_get_matrix': (ctypes.c_int, [c_op_p, c_double_p, c_i64]),
    'gpmi_op_set_rhs': (ctypes.c_int, [c_op_p, c_double_p, c_i64, ctypes.c_int]),
    'gpmi_op_loglik_batch': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p,
                                            c_double_p, c_int_p]),
    'gpmi_op_logdet': (ctypes.c_int, [c_op_p, ctypes.c_double, c_double_p]),
    'gpmi_op_solve': (ctypes.c_int, [c_op_p, ctypes.c_double, c_double_p, c_i64, ctypes.c_int,
                                     c_double_p, c_i64]),
    'gpmi_op_matvec': (ctypes.c_int, [c_op_p, c_double_p, c_i64, ctypes.c_int, c_double_p,
                                      c_i64]),
    'gpmi_op_trace': (ctypes.c_int, [c_op_p, c_double_p, c_double_p]),
    'gpmi_op_traceinv': (ctypes.c_int, [c_op_p, ctypes.c_double, ctypes.c_int, c_double_p]),
    'gpmi_op_set_timing': (ctypes.c_int, [c_op_p, ctypes.c_int]),
    'gpmi_op_last_timing': (ctypes.c_int, [c_op_p, c_double_p, c_int_p, c_double_p,
                                           c_double_p, c_double_p]),
    'gpmi_op_set_outer': (ctypes.c_int, [c_op_p, ctypes.c_int]),
    'gpmi_last_assembly_ms': (ctypes.c_int, [c_double_p]),
    'gpmi_matern_values': (ctypes.c_int, [ctypes.c_int, c_double_p, c_i64, ctypes.c_double,
                                          c_double_p]),
    'gpmi_sp_create_matern': (ctypes.c_int, [ctypes.c_int, c_double_p, c_i64, ctypes.c_int,
                                             c_double_p, ctypes.c_double, ctypes.c_double,
                                             ctypes.POINTER(c_op_p)]),
    'gpmi_sp_create_csr': (ctypes.c_int, [ctypes.c_int, c_i64, ctypes.POINTER(c_i64),
                                          c_int_p, c_double_p, ctypes.POINTER(c_op_p)]),
    'gpmi_sp_create_dense': (ctypes.c_int, [c_op_p, ctypes.POINTER(c_op_p)]),
    'gpmi_sp_destroy': (ctypes.c_int, [c_op_p]),
    'gpmi_sp_info': (ctypes.c_int, [c_op_p, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    'gpmi_sp_get_csr': (ctypes.c_int, [c_op_p, ctypes.POINTER(c_i64), c_int_p, c_double_p]),
    'gpmi_sp_spmm': (ctypes.c_int, [c_op_p, ctypes.c_double, c_double_p, c_i64, ctypes.c_int,
                                    c_double_p, c_i64]),
    'gpmi_sp_lanczos': (ctypes.c_int, [c_op_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                       ctypes.c_int, c_double_p, c_double_p]),
    'gpmi_sp_lanczos_ex': (ctypes.c_int, [c_op_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                          ctypes.c_int, ctypes.c_int, c_double_p, c_double_p]),
    'gpmi_sp_bench_spmm': (ctypes.c_int, [c_op_p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                          c_double_p]),
    'gpmi_sp_set_timing': (ctypes.c_int, [c_op_p, ctypes.c_int]),
    'gpmi_sp_spmm_timing': (ctypes.c_int, [c_op_p, ctypes.c_int, c_int_p, c_int_p, c_int_p,
                                           c_double_p]),
    'gpmi_sp_cg': (ctypes.c_int, [c_op_p, ctypes.c_double, c_double_p, c_i64, ctypes.c_int,
                                  ctypes.c_double, ctypes.c_int, c_double_p, c_i64, c_int_p]),
    'gpmi_sp_msgram': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p, c_i64,
                                      ctypes.c_int, ctypes.c_double, ctypes.c_int, c_double_p,
                                      c_int_p]),
    'gpmi_sp_msgram_cols': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p, c_i64,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_double, ctypes.c_int, c_double_p, c_int_p]),
    'gpmi_sp_set_rhs': (ctypes.c_int, [c_op_p, c_double_p, c_i64, ctypes.c_int]),
    'gpmi_band_create': (ctypes.c_int, [c_op_p, ctypes.POINTER(c_op_p)]),
    'gpmi_band_destroy': (ctypes.c_int, [c_op_p]),
    'gpmi_band_refresh': (ctypes.c_int, [c_op_p, c_op_p]),
    'gpmi_band_refresh_rhs': (ctypes.c_int, [c_op_p, c_op_p, c_double_p, c_i64, ctypes.c_int]),
    'gpmi_band_set_rhs': (ctypes.c_int, [c_op_p, c_double_p, c_i64, ctypes.c_int]),
    'gpmi_band_loglik': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p,
                                        c_double_p, c_int_p]),
    'gpmi_band_get': (ctypes.c_int, [c_op_p, c_double_p, c_i64]),
    'gpmi_band_eigenvalues': (ctypes.c_int, [c_op_p, c_double_p]),
    'gpmi_band_der_terms': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p,
                                           c_double_p, c_double_p, c_double_p, c_int_p]),
    'gpmi_band_der_ms': (ctypes.c_int, [c_op_p, c_double_p]),
    'gpmi_band_der_terms_ex': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p,
                                              c_double_p, c_double_p, c_double_p, c_double_p,
                                              c_int_p]),
    'gpmi_band_traceinv': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p,
                                          c_int_p]),
    'gpmi_band_der_terms_ex2': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p,
                                               c_double_p, c_double_p, c_double_p, c_double_p,
                                               c_double_p, c_int_p]),
    'gpmi_band_traceinv2': (ctypes.c_int, [c_op_p, c_double_p, ctypes.c_int, c_double_p,
                                           c_double_p, c_int_p]),
    'gpmi_band_sinv_ms': (ctypes.c_int, [c_op_p, c_double_p]),
    'gpmi_band_stats': (ctypes.c_int, [c_op_p, c_int_p, c_int_p]),
    'gpmi_band_cq_stats': (ctypes.c_int, [c_op_p, c_int_p, c_int_p, c_int_p]),
    'gpmi_band_chase_info': (ctypes.c_int, [c_op_p, c_int_p, c_int_p, c_int_p]),
    'gpmi_sp_last_status': (ctypes.c_int, [c_op_p, c_int_p]),
    'gpmi_sp_msgram_compactions': (ctypes.c_int, [c_op_p, c_int_p]),
    'gpmi_sp_msgram_segments': (ctypes.c_int, [c_op_p, ctypes.c_int, c_int_p, c_int_p,
                                               c_int_p]),
    'gpmi_sp_spmm_info': (ctypes.c_int, [c_op_p, c_int_p, c_double_p, c_int_p]),
    'gpmi_sp_spmm_kernel': (ctypes.c_int, [c_op_p, ctypes.c_int, c_int_p]),
    'gpmi_band_last_timing': (ctypes.c_int, [c_op_p, c_double_p, c_double_p, c_double_p]),
}


def rhs_block(R, n):
    """R as a C-contiguous n x k block (k <= MAX_RHS) for the resident RHS."""
    R = as_c(R)
    if R.ndim == 1:
        R = R[:, None]
    if R.shape[0] != n or R.shape[1] > MAX_RHS:
        raise ValueError('RHS must be %d x k with k <= %d' % (n, MAX_RHS))
    return R


class GPMIError(RuntimeError):
    """Error reported by libgpmi (HIP error or invalid argument)."""


def load():
    """Load libgpmi.so (once). Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise ImportError(
            'libgpmi.so not found at %s: build the HIP library first '
            '(python -c "import __graft_entry__ as g; g.build()")' % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error():
    buf = ctypes.create_string_buffer(512)
    load().gpmi_last_error(buf, 512)
    return buf.value.decode(errors='replace')


def check(rc, what):
    """Map a C status to Python: <0 -> GPMIError; >0 -> LinAlgError (not SPD)."""
    if rc == 0:
        return
    if rc > 0:
        raise numpy.linalg.LinAlgError(
            '%s: matrix K + eta I is not positive definite (pivot %d)' % (what, rc))
    raise GPMIError('%s failed (%d): %s' % (what, rc, last_error()))


def device_count():
    n = ctypes.c_int(0)
    check(load().gpmi_device_count(ctypes.byref(n)), 'gpmi_device_count')
    return n.value


def require_device(device):
    cnt = device_count()
    if cnt < 1:
        raise GPMIError('no HIP device visible: gaussian_proc runs only on MI355X (gfx950)')
    if not 0 <= device < cnt:
        raise GPMIError('device %d outside [0, %d)' % (device, cnt))


def default_device():
    return int(os.environ.get('LOCAL_RANK', '0'))


def dptr(a):
    return a.ctypes.data_as(c_double_p)


def as_c(a):
    return numpy.ascontiguousarray(a, dtype=numpy.float64)


class Operator(object):
    """Owning wrapper of a ``gpmi_op`` handle (device-resident K + workspace)."""

    def __init__(self, n, device=None, max_batch=1):
        self.lib = load()
        self.device = default_device() if device is None else int(device)
        require_device(self.device)
        self.n = int(n)
        self.max_batch = int(max_batch)
        h = c_op_p()
        check(self.lib.gpmi_op_create(self.device, self.n, self.max_batch, ctypes.byref(h)),
              'gpmi_op_create')
        self.h = h
        npad = c_i64()
        check(self.lib.gpmi_op_size(self.h, None, ctypes.byref(npad)), 'gpmi_op_size')
        self.n_pad = npad.value
        self.nrhs = 0
        # bumped whenever K changes: caches over K (e.g. SLQ Ritz nodes) compare it
        self.generation = 0

    def close(self):
        if getattr(self, 'h', None) is not None and self.h.value:
            self.lib.gpmi_op_destroy(self.h)
            self.h = c_op_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_matrix(self, K):
        K = as_c(K)
        if K.shape != (self.n, self.n):
            raise ValueError('K must be %d x %d' % (self.n, self.n))
        check(self.lib.gpmi_op_load_matrix(self.h, dptr(K), self.n), 'gpmi_op_load_matrix')
        self.generation += 1

    def load_sparse(self, sop):
        """K from a SparseOperator on the same device (device-side scatter of its
        CSR): the exact methods on a sparse K."""
        if sop.n != self.n:
            raise ValueError('sparse operator has n = %d, expected %d' % (sop.n, self.n))
        check(self.lib.gpmi_op_load_sparse(self.h, sop.h), 'gpmi_op_load_sparse')
        self.generation += 1

    def assemble_matern(self, points, scale, nu):
        points = as_c(points)
        scale = as_c(scale)
        check(self.lib.gpmi_op_assemble_matern(self.h, dptr(points), points.shape[1],
                                               dptr(scale), float(nu)),
              'gpmi_op_assemble_matern')
        self.generation += 1

    def get_matrix(self):
        K = numpy.empty((self.n, self.n))
        check(self.lib.gpmi_op_get_matrix(self.h, dptr(K), self.n), 'gpmi_op_get_matrix')
        return K

    def set_rhs(self, R):
        R = rhs_block(R, self.n)
        check(self.lib.gpmi_op_set_rhs(self.h, dptr(R), R.shape[1], R.shape[1]),
              'gpmi_op_set_rhs')
        self.nrhs = R.shape[1]

    def loglik_batch(self, etas):
        """-> (logdet[neta], gram[neta, nrhs, nrhs], info[neta])"""
        etas = as_c(numpy.atleast_1d(etas))
        ne = etas.shape[0]
        ld = numpy.empty(ne)
        g = numpy.empty((ne, self.nrhs, self.nrhs))
        info = numpy.zeros(ne, dtype=numpy.int32)
        check(self.lib.gpmi_op_loglik_batch(self.h, dptr(etas), ne, dptr(ld), dptr(g),
                                            info.ctypes.data_as(c_int_p)),
              'gpmi_op_loglik_batch')
        return ld, g, info

    def logdet(self, eta):
        out = ctypes.c_double()
        check(self.lib.gpmi_op_logdet(self.h, float(eta), ctypes.byref(out)), 'gpmi_op_logdet')
        return out.value

    def solve(self, eta, Y):
        Y = as_c(Y)
        Y2 = Y[:, None] if Y.ndim == 1 else Y
        sol = numpy.empty_like(Y2)
        check(self.lib.gpmi_op_solve(self.h, float(eta), dptr(Y2), Y2.shape[1], Y2.shape[1],
                                     dptr(sol), sol.shape[1]), 'gpmi_op_solve')
        return sol[:, 0] if Y.ndim == 1 else sol

    def matvec(self, x):
        x = as_c(x)
        x2 = x[:, None] if x.ndim == 1 else x
        y = numpy.empty_like(x2)
        check(self.lib.gpmi_op_matvec(self.h, dptr(x2), x2.shape[1], x2.shape[1], dptr(y),
                                      y.shape[1]), 'gpmi_op_matvec')
        return y[:, 0] if x.ndim == 1 else y

    def trace(self):
        a = ctypes.c_double()
        b = ctypes.c_double()
        check(self.lib.gpmi_op_trace(self.h, ctypes.byref(a), ctypes.byref(b)), 'gpmi_op_trace')
        return a.value, b.value

    def traceinv(self, eta, exponent=1):
        """Exact tr((K + eta I)^-exponent), exponent 1 or 2 (device triangular
        inverse of the cached Cholesky factor)."""
        v = ctypes.c_double()
        check(self.lib.gpmi_op_traceinv(self.h, float(eta), int(exponent), ctypes.byref(v)),
              'gpmi_op_traceinv')
        return v.value

    def set_timing(self, on):
        check(self.lib.gpmi_op_set_timing(self.h, int(bool(on))), 'gpmi_op_set_timing')

    def last_timing(self):
        ms = ctypes.c_double()
        nl = ctypes.c_int()
        fl = ctypes.c_double()
        tot = ctypes.c_double()
        busy = ctypes.c_double()
        check(self.lib.gpmi_op_last_timing(self.h, ctypes.byref(ms), ctypes.byref(nl),
                                           ctypes.byref(fl), ctypes.byref(tot),
                                           ctypes.byref(busy)),
              'gpmi_op_last_timing')
        return dict(syrk_ms=ms.value, syrk_launches=nl.value, syrk_flops=fl.value,
                    total_ms=tot.value, syrk_busy_ms=busy.value)

    def set_outer(self, s):
        check(self.lib.gpmi_op_set_outer(self.h, int(s)), 'gpmi_op_set_outer')


class Band(object):
    """Owning wrapper of a ``gpmi_band`` handle: the operator's K reduced once on
    the device to band form K = Q B Q^T (bandwidth 128); afterwards logdet and
    the Gram block R^T (K + eta I)^-1 R for any number of eta cost one banded
    Cholesky each (all eta concurrently, one workgroup per eta)."""

    CHUNK = 4096   # eta values per device call

    def __init__(self, op):
        self.lib = load()
        self.op = op   # keeps the operator (and its device) alive
        self.n = op.n
        self.device = op.device
        h = c_op_p()
        check(self.lib.gpmi_band_create(op.h, ctypes.byref(h)), 'gpmi_band_create')
        self.h = h
        self.nrhs = 0

    def close(self):
        if getattr(self, 'h', None) is not None and self.h.value:
            self.lib.gpmi_band_destroy(self.h)
            self.h = c_op_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def refresh(self, R=None):
        """Reduce the operator's current K again (buffers reused). Without R the
        resident RHS is reset; with R, Q^T R is applied during the reduction."""
        if R is None:
            check(self.lib.gpmi_band_refresh(self.h, self.op.h), 'gpmi_band_refresh')
            self.nrhs = 0
            return
        R = self._check_rhs(R)
        check(self.lib.gpmi_band_refresh_rhs(self.h, self.op.h, dptr(R), R.shape[1], R.shape[1]),
              'gpmi_band_refresh_rhs')
        self.nrhs = R.shape[1]

    def _check_rhs(self, R):
        return rhs_block(R, self.n)

    def set_rhs(self, R):
        R = as_c(R)
        if R.ndim == 1:
            R = R[:, None]
        if R.shape[0] != self.n or R.shape[1] > MAX_RHS:
            raise ValueError('RHS must be %d x k with k <= %d' % (self.n, MAX_RHS))
        check(self.lib.gpmi_band_set_rhs(self.h, dptr(R), R.shape[1], R.shape[1]),
              'gpmi_band_set_rhs')
        self.nrhs = R.shape[1]

    def loglik(self, etas):
        """-> (logdet[neta], gram[neta, nrhs, nrhs], info[neta])"""
        etas = as_c(numpy.atleast_1d(etas))
        ne = etas.shape[0]
        ld = numpy.empty(ne)
        g = numpy.empty((ne, self.nrhs, self.nrhs))
        info = numpy.zeros(ne, dtype=numpy.int32)
        for i in range(0, ne, self.CHUNK):
            e = as_c(etas[i:i + self.CHUNK])
            k = e.shape[0]
            ldk = numpy.empty(k)
            gk = numpy.empty((k, self.nrhs, self.nrhs))
            ik = numpy.zeros(k, dtype=numpy.int32)
            check(self.lib.gpmi_band_loglik(self.h, dptr(e), k, dptr(ldk), dptr(gk),
                                            ik.ctypes.data_as(c_int_p)), 'gpmi_band_loglik')
            ld[i:i + k], g[i:i + k], info[i:i + k] = ldk, gk, ik
        return ld, g, info

    DER_CHUNK = 256   # GPMI_BAND_DER_MAX

    TR_CHUNK = 64   # etas per selected-inversion call (its workspace: ~170 MB per eta
    #                 at n = 16384, the cyclic-reduction factor and the inverse's blocks)

    def der_terms(self, etas, traceinv=False):
        """-> (logdet[neta], g1, g2, g3 [neta, nrhs, nrhs], info[neta]) with
        gp = R^T (K + eta I)^-p R for the resident RHS R; with ``traceinv`` also
        tr1[neta] = trace((K + eta I)^-1) (selected inversion, no eigenvalues),
        appended as the last-but-one item; with ``traceinv=2`` also
        tr2[neta] = trace((K + eta I)^-2) (its eta-tangent), after tr1."""
        etas = as_c(numpy.atleast_1d(etas))
        ne, m = etas.shape[0], self.nrhs
        ld = numpy.empty(ne)
        g = [numpy.empty((ne, m, m)) for _ in range(3)]
        tr = numpy.empty(ne)
        tr2 = numpy.empty(ne)
        info = numpy.zeros(ne, dtype=numpy.int32)
        chunk = self.TR_CHUNK if traceinv else self.DER_CHUNK
        for i in range(0, ne, chunk):
            e = as_c(etas[i:i + chunk])
            k = e.shape[0]
            ldk = numpy.empty(k)
            gk = [numpy.empty((k, m, m)) for _ in range(3)]
            ik = numpy.zeros(k, dtype=numpy.int32)
            if traceinv:
                tk = numpy.empty(k)
                t2k = numpy.empty(k)
                check(self.lib.gpmi_band_der_terms_ex2(self.h, dptr(e), k, dptr(ldk),
                                                       dptr(gk[0]), dptr(gk[1]), dptr(gk[2]),
                                                       dptr(tk),
                                                       dptr(t2k) if traceinv == 2 else None,
                                                       ik.ctypes.data_as(c_int_p)),
                      'gpmi_band_der_terms_ex2')
                tr[i:i + k] = tk
                tr2[i:i + k] = t2k
            else:
                check(self.lib.gpmi_band_der_terms(self.h, dptr(e), k, dptr(ldk), dptr(gk[0]),
                                                   dptr(gk[1]), dptr(gk[2]),
                                                   ik.ctypes.data_as(c_int_p)),
                      'gpmi_band_der_terms')
            ld[i:i + k], info[i:i + k] = ldk, ik
            for q in range(3):
                g[q][i:i + k] = gk[q]
        if traceinv == 2:
            return ld, g[0], g[1], g[2], tr, tr2, info
        if traceinv:
            return ld, g[0], g[1], g[2], tr, info
        return ld, g[0], g[1], g[2], info

    def traceinv(self, etas, exponent=1):
        """-> (tr[neta], info[neta]): trace((K + eta I)^-exponent), exponent 1 or 2,
        by selected inversion of the cyclic-reduction factor of B + eta I (exponent
        2: its eta-tangent, trace((B + eta I)^-2) = -d/deta trace((B + eta I)^-1);
        gpmi_band_traceinv2)."""
        if exponent not in (1, 2):
            raise ValueError('selected inversion gives exponent 1 or 2')
        etas = as_c(numpy.atleast_1d(etas))
        ne = etas.shape[0]
        tr = numpy.empty(ne)
        info = numpy.zeros(ne, dtype=numpy.int32)
        for i in range(0, ne, self.TR_CHUNK):
            e = as_c(etas[i:i + self.TR_CHUNK])
            k = e.shape[0]
            tk = numpy.empty(k)
            t2k = numpy.empty(k)
            ik = numpy.zeros(k, dtype=numpy.int32)
            check(self.lib.gpmi_band_traceinv2(self.h, dptr(e), k, dptr(tk),
                                               dptr(t2k) if exponent == 2 else None,
                                               ik.ctypes.data_as(c_int_p)),
                  'gpmi_band_traceinv2')
            tr[i:i + k] = tk if exponent == 1 else t2k
            info[i:i + k] = ik
        return tr, info

    def sinv_ms(self):
        v = ctypes.c_double()
        check(self.lib.gpmi_band_sinv_ms(self.h, ctypes.byref(v)), 'gpmi_band_sinv_ms')
        return v.value

    def stats(self):
        """-> dict(panel_fallbacks, panel_maxg, panel, cholqr_fallbacks,
        cholqr_panel_fallbacks) (see gpmi_band_stats, gpmi_band_cq_stats)."""
        fb, mg = ctypes.c_int(), ctypes.c_int()
        check(self.lib.gpmi_band_stats(self.h, ctypes.byref(fb), ctypes.byref(mg)),
              'gpmi_band_stats')
        pm, cf, cp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self.lib.gpmi_band_cq_stats(self.h, ctypes.byref(pm), ctypes.byref(cf),
                                          ctypes.byref(cp)), 'gpmi_band_cq_stats')
        return dict(panel_fallbacks=fb.value, panel_maxg=mg.value,
                    panel='cholqr' if pm.value == 0 else 'householder',
                    cholqr_fallbacks=cf.value, cholqr_panel_fallbacks=cp.value)

    def chase_info(self):
        """-> dict(systolic (2 split, 1 one-per-position, 0 launches), fallbacks,
        maxg) of the last eigenvalues() (see gpmi_band_chase_info)."""
        sy, fb, mg = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self.lib.gpmi_band_chase_info(self.h, ctypes.byref(sy), ctypes.byref(fb),
                                            ctypes.byref(mg)), 'gpmi_band_chase_info')
        return dict(systolic=sy.value, fallbacks=fb.value, maxg=mg.value)

    def der_ms(self):
        v = ctypes.c_double()
        check(self.lib.gpmi_band_der_ms(self.h, ctypes.byref(v)), 'gpmi_band_der_ms')
        return v.value

    # gpmi_band_eigenvalues calls made by this process (bench: the optimizer's count)
    eigenvalue_calls = 0

    def eigenvalues(self):
        """The n eigenvalues of K, ascending (device bulge chase + bisection)."""
        Band.eigenvalue_calls += 1
        lam = numpy.empty(self.n)
        check(self.lib.gpmi_band_eigenvalues(self.h, dptr(lam)), 'gpmi_band_eigenvalues')
        return lam

    def band(self):
        """B as a dense symmetric n x n host matrix (tests)."""
        B = numpy.empty((self.n, self.n))
        check(self.lib.gpmi_band_get(self.h, dptr(B), self.n), 'gpmi_band_get')
        return B

    def last_timing(self):
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(self.lib.gpmi_band_last_timing(self.h, ctypes.byref(a), ctypes.byref(b),
                                             ctypes.byref(c)), 'gpmi_band_last_timing')
        return dict(reduce_ms=a.value, rhs_ms=b.value, loglik_ms=c.value)


def matern_dense(points, scale, nu, device=None):
    """Dense Matérn K on the device, returned as a host ndarray."""
    lib = load()
    device = default_device() if device is None else int(device)
    require_device(device)
    points = as_c(points)
    scale = as_c(scale)
    n, d = points.shape
    K = numpy.empty((n, n))
    check(lib.gpmi_matern_dense(device, dptr(points), n, d, dptr(scale), float(nu), dptr(K),
                                n), 'gpmi_matern_dense')
    return K


def last_assembly_ms():
    """Device ms of this thread's last dense Matérn assembly kernel."""
    v = ctypes.c_double()
    check(load().gpmi_last_assembly_ms(ctypes.byref(v)), 'gpmi_last_assembly_ms')
    return v.value


def matern_values(x, nu, device=None):
    """matern(x) evaluated by the device kernel (used for the taper threshold)."""
    lib = load()
    device = default_device() if device is None else int(device)
    require_device(device)
    x = as_c(numpy.atleast_1d(x))
    out = numpy.empty_like(x)
    check(lib.gpmi_matern_values(device, dptr(x), x.size, float(nu), dptr(out)),
          'gpmi_matern_values')
    return out


class SparseOperator(object):
    """Owning wrapper of a ``gpmi_sp`` handle (device CSR + Krylov workspace)."""

    def __init__(self, handle, device):
        self.lib = load()
        self.h = handle
        self.device = device
        n = c_i64()
        nnz = c_i64()
        check(self.lib.gpmi_sp_info(self.h, ctypes.byref(n), ctypes.byref(nnz)), 'gpmi_sp_info')
        self.n, self.nnz = n.value, nnz.value

    @classmethod
    def from_points(cls, points, scale, nu, tau, device=None):
        lib = load()
        device = default_device() if device is None else int(device)
        require_device(device)
        points = as_c(points)
        scale = as_c(scale)
        h = c_op_p()
        check(lib.gpmi_sp_create_matern(device, dptr(points), points.shape[0], points.shape[1],
                                        dptr(scale), float(nu), float(tau), ctypes.byref(h)),
              'gpmi_sp_create_matern')
        return cls(h, device)

    @classmethod
    def from_csr(cls, K, device=None):
        lib = load()
        device = default_device() if device is None else int(device)
        require_device(device)
        K = K.tocsr()
        K.sort_indices()
        ip = numpy.ascontiguousarray(K.indptr, dtype=numpy.int64)
        ix = numpy.ascontiguousarray(K.indices, dtype=numpy.int32)
        dv = as_c(K.data)
        h = c_op_p()
        check(lib.gpmi_sp_create_csr(device, K.shape[0], ip.ctypes.data_as(ctypes.POINTER(c_i64)),
                                     ix.ctypes.data_as(c_int_p), dptr(dv), ctypes.byref(h)),
              'gpmi_sp_create_csr')
        return cls(h, device)

    @classmethod
    def from_dense(cls, op):
        """The Krylov primitives (spmm, lanczos, cg, msgram) on a dense
        ``Operator``'s device K (fp64 MFMA products, dense_mm_kernel): imate's
        'slq' on a dense K. Borrows op's matrix; keeps op alive."""
        h = c_op_p()
        check(op.lib.gpmi_sp_create_dense(op.h, ctypes.byref(h)), 'gpmi_sp_create_dense')
        out = cls(h, op.device)
        out.dense_op = op
        return out

    def close(self):
        if getattr(self, 'h', None) is not None and self.h.value:
            self.lib.gpmi_sp_destroy(self.h)
            self.h = c_op_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def csr(self):
        import scipy.sparse
        ip = numpy.empty(self.n + 1, dtype=numpy.int64)
        ix = numpy.empty(self.nnz, dtype=numpy.int32)
        dv = numpy.empty(self.nnz)
        check(self.lib.gpmi_sp_get_csr(self.h, ip.ctypes.data_as(ctypes.POINTER(c_i64)),
                                       ix.ctypes.data_as(c_int_p), dptr(dv)), 'gpmi_sp_get_csr')
        return scipy.sparse.csr_matrix((dv, ix, ip), shape=(self.n, self.n))

    def spmm(self, eta, X):
        X = as_c(X)
        X2 = X[:, None] if X.ndim == 1 else X
        Y = numpy.empty_like(X2)
        check(self.lib.gpmi_sp_spmm(self.h, float(eta), dptr(X2), X2.shape[1], X2.shape[1],
                                    dptr(Y), Y.shape[1]), 'gpmi_sp_spmm')
        return Y[:, 0] if X.ndim == 1 else Y

    def spmm_info(self):
        """-> dict(windowed, mean_window, max_window) (see gpmi_sp_spmm_info)."""
        w, mw, xw = ctypes.c_int(), ctypes.c_double(), ctypes.c_int()
        check(self.lib.gpmi_sp_spmm_info(self.h, ctypes.byref(w), ctypes.byref(mw),
                                         ctypes.byref(xw)), 'gpmi_sp_spmm_info')
        return dict(windowed=bool(w.value), mean_window=mw.value, max_window=xw.value)

    def spmm_kernel(self, s):
        """-> the SpMM kernel an s-column block runs: 'csr_spmm_kernel' (gather),
        'csr_spmm_win_kernel' (window, 8-column chunks), 'csr_spmm_pair_kernel'
        (gather by column pairs), 'dense_mm_kernel' (a dense K) or
        'csr_spmm_wing_kernel' (window with latency-hidden staging) (see
        gpmi_sp_spmm_kernel). It names the kernel for a 16-byte aligned block,
        which every block the library forms is (host inputs are copied into
        hipMalloc'd workspaces whose segments are even numbers of doubles); an
        unaligned device block handed in directly runs csr_spmm_kernel."""
        k = ctypes.c_int()
        check(self.lib.gpmi_sp_spmm_kernel(self.h, int(s), ctypes.byref(k)),
              'gpmi_sp_spmm_kernel')
        # index 2 was the round-2 one-pass window (superseded by the wing kernel)
        return ('csr_spmm_kernel', 'csr_spmm_win_kernel', 'csr_spmm_winf_kernel',
                'csr_spmm_pair_kernel', 'dense_mm_kernel', 'csr_spmm_wing_kernel')[k.value]

    def lanczos(self, nprobe, steps, seed=0, probe_offset=0, orthogonalize=-1):
        """-> alpha[nprobe, steps], beta[nprobe, steps] (beta = 0 ends a tridiagonal).
        orthogonalize: imate's option: -1 full reorthogonalisation (DCGS2), 0 the
        plain three-term recurrence, k > 0 against the last k vectors."""
        a = numpy.zeros((nprobe, steps))
        b = numpy.zeros((nprobe, steps))
        check(self.lib.gpmi_sp_lanczos_ex(self.h, int(nprobe), int(steps), int(seed),
                                          int(probe_offset), int(orthogonalize), dptr(a),
                                          dptr(b)), 'gpmi_sp_lanczos_ex')
        return a, b

    def set_timing(self, on):
        """In-step SpMM timing while on: every window SpMM launch of this operator
        stamps its span on the device wall clock (other SpMM kinds: a HIP event pair
        around it). set_timing(True) starts a new window (the log is cleared),
        set_timing(False) ends it and keeps its log for spmm_timing()."""
        check(self.lib.gpmi_sp_set_timing(self.h, int(bool(on))), 'gpmi_sp_set_timing')

    def spmm_timing(self):
        """{width s: (launches, total_ms)} of the SpMM launches logged since
        set_timing(True)."""
        nw = ctypes.c_int(0)
        w = (ctypes.c_int * 64)()
        c = (ctypes.c_int * 64)()
        t = (ctypes.c_double * 64)()
        check(self.lib.gpmi_sp_spmm_timing(self.h, 64, ctypes.byref(nw), w, c, t),
              'gpmi_sp_spmm_timing')
        return {int(w[k]): (int(c[k]), float(t[k])) for k in range(min(64, nw.value))}

    def bench_spmm(self, s, reps, eta=0.0):
        ms = ctypes.c_double()
        check(self.lib.gpmi_sp_bench_spmm(self.h, int(s), int(reps), float(eta),
                                          ctypes.byref(ms)), 'gpmi_sp_bench_spmm')
        return ms.value

    def cg(self, eta, B, rtol=1e-6, maxiter=None):
        B = as_c(B)
        B2 = B[:, None] if B.ndim == 1 else B
        X = numpy.empty_like(B2)
        it = ctypes.c_int(0)
        maxiter = 10 * self.n if maxiter is None else int(maxiter)
        check(self.lib.gpmi_sp_cg(self.h, float(eta), dptr(B2), B2.shape[1], B2.shape[1],
                                  float(rtol), maxiter, dptr(X), X.shape[1], ctypes.byref(it)),
              'gpmi_sp_cg')
        self.last_cg_iterations = it.value
        self._warn_unconverged('cg', maxiter)
        return X[:, 0] if B.ndim == 1 else X

    MS_MAXS = 16

    def set_rhs(self, B):
        """Keep the [n, s] block B resident in HBM (gpmi_sp_set_rhs): msgram(etas,
        None) then reads it there instead of uploading B per call."""
        B = as_c(B)
        B2 = B[:, None] if B.ndim == 1 else B
        if B2.shape[0] != self.n:
            raise ValueError('set_rhs: %d rows, the operator has %d' % (B2.shape[0], self.n))
        check(self.lib.gpmi_sp_set_rhs(self.h, dptr(B2), B2.shape[1], B2.shape[1]),
              'gpmi_sp_set_rhs')
        self.rhs_cols = B2.shape[1]

    rhs_cols = 0

    def msgram(self, etas, B, rtol=1e-6, maxiter=None, cols=None):
        """G[j] = B^T (K + etas[j] I)^-1 B for all etas from one multi-shift CG
        (B: [n, s], s <= 16; None: the block of set_rhs, resident in HBM). Returns
        G [neta, s, s]; with cols = (c_lo, c_hi) only those right-hand sides are
        solved (dotted with all of B): G [neta, s, c_hi - c_lo], the columns of the
        full G (gpmi_sp_msgram_cols)."""
        if B is None:
            if not self.rhs_cols:
                raise ValueError('msgram: no resident right-hand sides (set_rhs)')
            B2, s, ld = None, self.rhs_cols, self.rhs_cols
        else:
            B = as_c(B)
            B2 = B[:, None] if B.ndim == 1 else B
            s = ld = B2.shape[1]
        etas = as_c(numpy.atleast_1d(etas))
        c_lo, c_hi = (0, s) if cols is None else (int(cols[0]), int(cols[1]))
        w = c_hi - c_lo
        G = numpy.empty((etas.size, s, w))
        it = ctypes.c_int(0)
        maxiter = 10 * self.n if maxiter is None else int(maxiter)
        step = max(1, 1024 // max(1, w))
        for j0 in range(0, etas.size, step):
            e = as_c(etas[j0:j0 + step])
            Gj = numpy.empty((e.size, s, w))
            if cols is None:
                check(self.lib.gpmi_sp_msgram(self.h, dptr(e), e.size,
                                              None if B2 is None else dptr(B2), ld, s,
                                              float(rtol), maxiter, dptr(Gj), ctypes.byref(it)),
                      'gpmi_sp_msgram')
            else:
                check(self.lib.gpmi_sp_msgram_cols(self.h, dptr(e), e.size,
                                                   None if B2 is None else dptr(B2), ld, s,
                                                   c_lo, c_hi, float(rtol), maxiter, dptr(Gj),
                                                   ctypes.byref(it)),
                      'gpmi_sp_msgram_cols')
            G[j0:j0 + e.size] = Gj
            self._warn_unconverged('msgram', maxiter)
        self.last_cg_iterations = it.value
        return G

    def msgram_compactions(self):
        """Active-column compactions of the last msgram call (diagnostic)."""
        v = ctypes.c_int(0)
        check(self.lib.gpmi_sp_msgram_compactions(self.h, ctypes.byref(v)),
              'gpmi_sp_msgram_compactions')
        return v.value

    def msgram_segments(self):
        """The last msgram call's launch segments [(block width, iterations), ...]:
        the full block, then each compacted block (diagnostic)."""
        cap = 64
        w = (ctypes.c_int * cap)()
        k = (ctypes.c_int * cap)()
        m = ctypes.c_int(0)
        check(self.lib.gpmi_sp_msgram_segments(self.h, cap, w, k, ctypes.byref(m)),
              'gpmi_sp_msgram_segments')
        return [(w[q], k[q]) for q in range(m.value)]

    def _warn_unconverged(self, what, maxiter):
        """scipy's cg (the reference's sparse solve, _linear_solver.py:64,68)
        returns an unconverged iterate silently; here it is a RuntimeWarning."""
        ok = ctypes.c_int(1)
        check(self.lib.gpmi_sp_last_status(self.h, ctypes.byref(ok)), 'gpmi_sp_last_status')
        if not ok.value:
            import warnings
            warnings.warn('%s: CG stopped at maxiter=%d before reaching rtol' % (what, maxiter),
                          RuntimeWarning, stacklevel=3)

"""ctypes binding of libmamg.so (include/mamg.h).

The product path: this module is the thin ctypes C-ABI the north star asks
for (Python host code -> libmamg.so -> HIP).  It fails loudly if the built
library is missing; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('MAMG_LIB', os.path.join(_HERE, 'libmamg.so'))

MAMG_ABI_VERSION = 4
OK, ERR_ARG, ERR_HIP, ERR_SETUP, ERR_UNSUPPORTED, ERR_NOMEM, ERR_BREAKDOWN = 0, -1, -2, -3, -4, -5, -6


class MamgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__('mamg error %d: %s' % (code, msg))
        self.code = code


class mamg_params(C.Structure):
    _fields_ = [
        ('abi_version', C.c_int32), ('AMG_type', C.c_int32), ('cycle_type', C.c_int32),
        ('max_levels', C.c_int32), ('maxit', C.c_int32), ('smoother', C.c_int32),
        ('relaxation', C.c_double), ('presmooth_iter', C.c_int32),
        ('postsmooth_iter', C.c_int32), ('coarse_dof', C.c_int32),
        ('coarse_solver', C.c_int32), ('coarse_scaling', C.c_int32),
        ('aggregation_type', C.c_int32), ('strong_coupled', C.c_double),
        ('max_aggregation', C.c_int32), ('amli_degree', C.c_int32),
        ('Schwarz_levels', C.c_int32), ('Schwarz_mmsize', C.c_int32),
        ('Schwarz_maxlvl', C.c_int32), ('Schwarz_type', C.c_int32),
        ('Schwarz_blksolver', C.c_int32), ('print_level', C.c_int32),
        ('sa_omega', C.c_double), ('rho_iters', C.c_int32),
        ('max_coarse_dense', C.c_int32), ('device', C.c_int32), ('spmv_lanes', C.c_int32),
        ('num_functions', C.c_int32), ('node_block_smoother', C.c_int32),
        ('sa_block_diag', C.c_int32), ('post_fusion', C.c_int32),
        ('poly_degree', C.c_int32), ('poly_ratio', C.c_double),
        ('strength_measure', C.c_int32),
    ]


class mamg_csr(C.Structure):
    _fields_ = [('nrows', C.c_int64), ('ncols', C.c_int64), ('nnz', C.c_int64),
                ('rowptr', C.POINTER(C.c_int64)), ('colind', C.POINTER(C.c_int32)),
                ('values', C.POINTER(C.c_double))]


P_I64 = C.POINTER(C.c_int64)
P_I32 = C.POINTER(C.c_int32)
P_F64 = C.POINTER(C.c_double)
VP = C.c_void_p

# mamg_exchange (host-staged transport of a multi-GPU handle)
SENDRECV_FN = C.CFUNCTYPE(C.c_int, VP, C.c_int, C.POINTER(P_F64), P_I64, C.POINTER(P_F64), P_I64)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, VP, P_F64, C.c_int64)


class mamg_exchange(C.Structure):
    _fields_ = [('ctx', VP), ('sendrecv', SENDRECV_FN), ('allreduce', ALLREDUCE_FN)]

# every symbol include/mamg.h and include/mamg_test.h declare: name -> (restype, argtypes)
SIGNATURES = {
    'mamg_abi_version': (C.c_int, []),
    'mamg_release_setup_cache': (C.c_int, []),
    'mamg_set_setup_cache_limit': (C.c_int, [C.c_int64]),
    'mamg_setup_cache_bytes': (C.c_int, [C.c_int, P_I64, P_I64]),
    'mamg_set_option': (C.c_int, [C.c_char_p, C.c_char_p]),
    'mamg_option_names': (C.c_char_p, []),
    'mamg_last_error': (C.c_char_p, []),
    'mamg_params_default': (None, [C.POINTER(mamg_params)]),
    'mamg_gen_bidomain_size': (C.c_int, [C.c_int, C.c_int64, P_I64, P_I64]),
    'mamg_gen_bidomain': (C.c_int, [C.c_int, C.c_int64, C.c_double, C.c_double, C.c_double,
                                    P_I64, P_I32, P_F64]),
    'mamg_gen_bidomain_device': (C.c_int, [C.c_int, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_int64,
                                           VP, VP, VP]),
    'mamg_gen_bidomain_mms': (C.c_int, [C.c_int, C.c_int64, C.c_double, C.c_double, C.c_double, P_F64]),
    'mamg_bidomain_mms_error': (C.c_int, [C.c_int, C.c_int64, C.c_double, C.c_double, C.c_double,
                                          P_F64, P_F64]),
    'mamg_host_setup': (C.c_int, [C.POINTER(mamg_csr), P_I32, C.c_int64,
                                  C.POINTER(mamg_params), C.POINTER(VP)]),
    'mamg_hier_free': (None, [VP]),
    'mamg_hier_num_levels': (C.c_int, [VP]),
    'mamg_hier_params': (C.c_int, [VP, C.POINTER(mamg_params)]),
    'mamg_hier_level_sizes': (C.c_int, [VP, C.c_int, P_I64]),
    'mamg_hier_level_export': (C.c_int, [VP, C.c_int] + [P_I64, P_I32, P_F64] * 4
                               + [P_F64, P_I64, P_F64]),
    'mamg_hier_dist_plan': (C.c_int, [VP, C.c_int, C.c_int, C.c_int64, C.POINTER(VP)]),
    'mamg_plan_free': (None, [VP]),
    'mamg_plan_num_levels': (C.c_int, [VP]),
    'mamg_plan_level_sizes': (C.c_int, [VP, C.c_int, P_I64]),
    'mamg_plan_level_export': (C.c_int, [VP, C.c_int, P_I64, P_I64, P_I64, P_I64]
                               + [P_I64, P_I32, P_F64] * 3 + [P_F64]),
    'mamg_comm_id_bytes': (C.c_int, []),
    'mamg_comm_unique_id': (C.c_int, [C.c_char_p]),
    'mamg_setup_dist': (C.c_int, [C.POINTER(mamg_csr), P_I32, C.c_int64, C.POINTER(mamg_params),
                                  C.c_int, C.c_int, C.c_char_p, C.c_int64, C.POINTER(VP)]),
    'mamg_setup_dist_device': (C.c_int, [C.POINTER(mamg_csr), P_I32, C.c_int64, C.POINTER(mamg_params),
                                         C.c_int, C.c_int, C.c_char_p, C.c_int64, C.POINTER(VP)]),
    'mamg_dist_range': (C.c_int, [VP, P_I64, P_I64, P_I64]),
    'mamg_dist_apply_bytes': (C.c_int, [VP, P_F64]),
    'mamg_dist_apply_launches': (C.c_int, [VP, C.POINTER(C.c_int64)]),
    'mamg_dist_apply_device': (C.c_int, [VP, VP, VP, VP]),
    'mamg_dist_apply_graph': (C.c_int, [VP, VP, VP, VP]),
    'mamg_dist_graph_prepare': (C.c_int, [VP, VP, VP]),
    'mamg_dist_virtual_apply_graph': (C.c_int, [C.POINTER(VP), C.c_int, C.POINTER(VP), C.POINTER(VP), VP]),
    'mamg_dist_time_apply': (C.c_int, [VP, VP, VP, C.c_int, C.c_int, P_F64, P_F64, P_F64, VP]),
    'mamg_dist_virtual_apply': (C.c_int, [C.POINTER(VP), C.c_int, C.POINTER(VP), C.POINTER(VP), VP]),
    'mamg_dist_spmv_device': (C.c_int, [VP, VP, VP, VP]),
    'mamg_dist_virtual_spmv': (C.c_int, [C.POINTER(VP), C.c_int, C.POINTER(VP), C.POINTER(VP), VP]),
    'mamg_dist_destroy': (None, [VP]),
    'mamg_dist_set_exchange': (C.c_int, [VP, C.POINTER(mamg_exchange)]),
    'mamg_setup': (C.c_int, [C.POINTER(mamg_csr), P_I32, C.c_int64, C.POINTER(mamg_params),
                             C.POINTER(VP)]),
    'mamg_setup_gpu': (C.c_int, [C.POINTER(mamg_csr), P_I32, C.c_int64, C.POINTER(mamg_params),
                                 C.POINTER(VP)]),
    'mamg_setup_gpu_device': (C.c_int, [C.POINTER(mamg_csr), P_I32, C.c_int64, C.POINTER(mamg_params),
                                        C.POINTER(VP)]),
    'mamg_gpu_host_setup': (C.c_int, [C.POINTER(mamg_csr), P_I32, C.c_int64, C.POINTER(mamg_params),
                                      C.POINTER(VP)]),
    'mamg_sharded_galerkin_check': (C.c_int, [C.POINTER(mamg_csr), C.POINTER(mamg_csr), C.POINTER(mamg_csr),
                                              C.c_int, C.c_int, P_I64]),
    'mamg_setup_timings': (C.c_int, [VP, P_F64]),
    'mamg_layout_timings': (C.c_int, [VP, P_F64]),
    'mamg_upload': (C.c_int, [VP, C.POINTER(mamg_csr), C.POINTER(mamg_params), C.POINTER(VP)]),
    'mamg_destroy': (None, [VP]),
    'mamg_nrows': (C.c_int64, [VP]),
    'mamg_num_levels': (C.c_int, [VP]),
    'mamg_device_layout': (C.c_int, [VP]),
    'mamg_level_format': (C.c_int, [VP, C.c_int]),
    'mamg_handle_params': (C.c_int, [VP, C.POINTER(mamg_params)]),
    'mamg_kregion_info': (C.c_int, [VP, P_F64, C.c_int, P_I32, P_I32]),
    'mamg_apply_bytes': (C.c_int, [VP, P_F64]),
    'mamg_apply': (C.c_int, [VP, P_F64, P_F64]),
    'mamg_apply_device': (C.c_int, [VP, VP, VP, VP]),
    'mamg_spmv_device': (C.c_int, [VP, VP, VP, VP]),
    'mamg_pcg_device': (C.c_int, [VP, VP, VP, C.c_double, C.c_int, C.c_int, P_F64, P_F64,
                                  P_F64, P_I32, VP]),
    'mamg_time_apply': (C.c_int, [VP, VP, VP, C.c_int, C.c_int, P_F64, P_F64, P_F64, VP]),
}

_lib = None


def lib():
    """Load libmamg.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError('libmamg.so not built (%s); run __graft_entry__.build() '
                              'or make -C metric-amg-examples_amd/csrc' % LIB_PATH)
        # One HIP runtime per process: torch's wheel ships its own
        # libamdhip64 (soname libamdhip64.so.7, NEEDED as "libamdhip64.so").
        # Loaded first, it also satisfies libmamg's libamdhip64.so.7; loaded
        # after libmamg, torch would bring up a second runtime that finds no
        # device.  So torch (when installed) is imported before the library.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.mamg_abi_version() != MAMG_ABI_VERSION:
            raise ImportError('libmamg ABI mismatch')
        _lib = L
    return _lib


def set_option(name, value):
    """mamg_set_option (include/mamg_test.h): set (value not None) or reset
    one of the library's internal layout switches for the process."""
    v = None if value is None else str(value).encode()
    check(lib().mamg_set_option(name.encode(), v))


def option_names():
    return lib().mamg_option_names().decode().split(',')


def check(rc):
    if rc != 0:
        raise MamgError(rc, lib().mamg_last_error().decode(errors='replace'))
    return rc


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def as_csr_struct(indptr: np.ndarray, indices: np.ndarray, data: np.ndarray, ncols: int):
    """Build a mamg_csr view (arrays must stay alive while it is used)."""
    n = len(indptr) - 1
    s = mamg_csr()
    s.nrows, s.ncols, s.nnz = n, ncols, int(indptr[-1])
    s.rowptr = ptr(indptr, C.c_int64)
    s.colind = ptr(indices, C.c_int32)
    s.values = ptr(data, C.c_double)
    return s

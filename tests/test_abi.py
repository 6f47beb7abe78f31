"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/mamg.h declares, validates parameters with explicit errors (no
silent fallback), and the generator sizes match the survey's formulas."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = ''.join(open(os.path.join(ROOT, 'include', f)).read() for f in sorted(os.listdir(os.path.join(ROOT, 'include')))
                  if f.endswith('.h'))
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(mamg_[a-z_0-9]+)\s*\(', txt)))


def test_exports_every_declared_symbol(lib_built):
    import metric_amg_examples_amd as M
    L = M._lib.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
        assert s in M._lib.SIGNATURES, 'ctypes prototype missing for %s' % s


DIAG_SWITCHES = ('MAMG_DEBUG_SUMS', 'MAMG_K_VARIANT', 'MAMG_TAIL_PROFILE', 'MAMG_OP_PROFILE', 'MAMG_FREE_MODE',
                 'MAMG_ALLOC_LOG', 'MAMG_DIAG_CONTIG', 'MAMG_DEBUG_PTRS')


def test_diagnosis_switches_only_in_the_diag_build(lib_built):
    """the product library reads none of the diagnosis
    switches (their names are not even in the binary); the diagnosis build
    (make diag, -DMAMG_DIAG=1) has them all."""
    prod = open(lib_built, 'rb').read()
    for k in DIAG_SWITCHES:
        assert k.encode() not in prod, k
    from conftest import DIAG_LIB
    diag = open(DIAG_LIB, 'rb').read()
    for k in DIAG_SWITCHES:
        assert k.encode() in diag, k


def test_params_struct_layout(lib_built):
    import metric_amg_examples_amd as M
    p = M.parameters.make_params()
    assert p.abi_version == 4 and p.strength_measure == 1 and p.post_fusion == 1 and p.AMG_type == 2 and p.cycle_type == 1
    assert p.poly_degree == 2 and p.poly_ratio == 16.0     # last fields: struct tail matches mamg.h
    assert abs(p.relaxation - 4.0 / 3.0) < 1e-15 and p.coarse_dof == 100
    assert p.num_functions == 1 and p.node_block_smoother == 1
    assert M.parameters.make_params(M.parameters.parameters_metric_mi355x).num_functions == 2
    d = M.parameters.params_to_dict(p)
    assert set(M.parameters.KEYS) - {'prectype'} <= set(d)


@pytest.mark.parametrize('bad,code', [
    (dict(smoother=11), -4),                 # SGS is a node-block smoother: num_functions 2
    (dict(aggregation_type=3), -4),          # MWM rejected (MIS, HEM and VMB run)
    (dict(coarse_scaling=2), -1),
    (dict(Schwarz_type=3), -4),              # overlapping multiplicative Schwarz: nodal systems only
    (dict(num_functions=2, Schwarz_type=3, Schwarz_maxlvl=0), -4),   # seed nodes: SYMMETRIC needs SGS
    (dict(num_functions=2, smoother=11, Schwarz_type=9), -1),        # unknown Schwarz_type
    (dict(num_functions=2, smoother=11, Schwarz_type=4), -4),
    (dict(Schwarz_maxlvl=2), -4),            # overlapping seed + ring blocks need SCHWARZ_ADDITIVE
    (dict(Schwarz_maxlvl=0), -4),            # seed-node blocks need num_functions >= 2
    (dict(num_functions=2, smoother=11, Schwarz_type=5), -4),   # ADDITIVE is for Jacobi-family smoothers
    (dict(cycle_type=3), -4),
    (dict(max_levels=0), -1),
    (dict(spmv_lanes=3), -1),
    (dict(num_functions=0), -1),
])
def test_rejects_unsupported(lib_built, bad, code):
    import metric_amg_examples_amd as M
    from mamg_oracle import laplace1d
    with pytest.raises(M._lib.MamgError) as ei:
        M.HostHierarchy(laplace1d(30), **bad)
    assert ei.value.code == code
    assert len(str(ei.value)) > 20


def test_reference_presets_map_and_report(lib_built):
    import metric_amg_examples_amd as M
    P = M.parameters
    # the reference's names carry the reference's values; every component of
    # parameters_metric_schwarz now exists (UA, parallel HEM, W, SGS as
    # multicolour node-block SGS, coarse scaling, symmetric seed blocks), so it
    # runs as given on a nodal system, and is rejected loudly where a
    # component is missing (SGS on a scalar system)
    assert P.parameters_metric_schwarz['aggregation_type'] == P.HEM
    assert P.parameters_metric_schwarz['smoother'] == P.SMOOTHER_SGS
    from mamg_oracle import laplace1d
    with pytest.raises(M._lib.MamgError) as ei:
        M.HostHierarchy(laplace1d(30), parameters=P.parameters_metric_schwarz)
    assert ei.value.code == -4 and len(str(ei.value)) > 20
    s = M.problems.bidomain(2, 16, 1e4)
    H = M.HostHierarchy(s, idofs=s.idofs, parameters=P.parameters_metric_schwarz, num_functions=2)
    assert H.num_levels >= 2
    # the reference's SCHWARZ_SYMMETRIC on the seeds' 1-rings runs as the
    # overlapping node patches (not the non-overlapping seed blocks)
    assert H.effective_params['Schwarz_type'] == P.SCHWARZ_PATCHES
    H.close()
    # its old meaning has its own name; GS/SGS on the seed blocks
    H = M.HostHierarchy(s, idofs=s.idofs, parameters=P.parameters_metric_mi355x_sgs)
    assert H.effective_params['Schwarz_type'] == P.SCHWARZ_SEED_BLOCKS
    H.close()
    # sparse seeds (not one on every node), or rings of 2: the reference's
    # overlapping multiplicative form runs as the seed rings (SCHWARZ_RINGS)
    H = M.HostHierarchy(s, idofs=s.idofs[::2], parameters=P.parameters_metric_schwarz, num_functions=2)
    assert H.effective_params['Schwarz_type'] == P.SCHWARZ_RINGS
    H.close()
    H = M.HostHierarchy(s, idofs=s.idofs, parameters=dict(P.parameters_metric_schwarz, Schwarz_maxlvl=2),
                        num_functions=2)
    assert H.effective_params['Schwarz_type'] == P.SCHWARZ_RINGS
    H.close()
    # ... the reference's default dict too (src/utils.py:60-82); without seeds
    # no Schwarz level (the level smoother everywhere, src/utils.py:88)
    H = M.HostHierarchy(s, idofs=s.idofs[::3], parameters=P.parameters_metric_default, num_functions=2)
    assert H.effective_params['Schwarz_type'] == P.SCHWARZ_RINGS
    H.close()
    H = M.HostHierarchy(s, parameters=P.parameters_metric_default, num_functions=2)
    assert H.effective_params['Schwarz_levels'] == 0
    H.close()
    # forward-only multiplicative Schwarz on overlapping blocks is not built
    with pytest.raises(M._lib.MamgError) as ei:
        M.HostHierarchy(s, idofs=s.idofs, parameters=dict(P.parameters_metric_schwarz, Schwarz_maxlvl=2,
                                                           Schwarz_type=P.SCHWARZ_FORWARD), num_functions=2)
    assert ei.value.code == -4 and 'SCHWARZ_ADDITIVE' in str(ei.value)
    # explicit mapping keeps what is implemented and reports what it changes
    mapped, notes = P.to_gpu_profile(P.parameters_standard)
    assert mapped['aggregation_type'] == P.VMB and not any('aggregation' in n for n in notes)
    mapped_mwm, notes = P.to_gpu_profile(dict(P.parameters_standard, aggregation_type=P.MWM))
    assert mapped_mwm['aggregation_type'] == P.MIS and any('aggregation_type' in n for n in notes)
    mapped, notes = P.to_gpu_profile(P.parameters_metric_schwarz)
    assert mapped['smoother'] == P.SMOOTHER_SGS and mapped['aggregation_type'] == P.HEM
    assert mapped['Schwarz_type'] == P.SCHWARZ_PATCHES and mapped['coarse_scaling'] == P.ON
    assert any('SCHWARZ_PATCHES' in n for n in notes)
    assert mapped['num_functions'] == 2
    assert P.parameters_metric_schwarz_gpu_mapped == mapped
    H = M.HostHierarchy(laplace1d(300), parameters=P.parameters_standard_gpu_mapped,
                        num_functions=1, smoother=P.SMOOTHER_JACOBI_RHO)
    assert H.num_levels >= 2
    with pytest.raises(KeyError):
        P.make_params({'no_such_key': 1})


def test_generator_sizes(lib_built):
    import metric_amg_examples_amd as M
    L = M._lib.lib()
    N, nnz = C.c_int64(), C.c_int64()
    # bidomain_3d nrefs=6 -> n=256, N = 2*257^3
    assert L.mamg_gen_bidomain_size(3, 256, C.byref(N), C.byref(nnz)) == 0
    assert N.value == 33949186 and 9.9e8 < nnz.value < 1.02e9
    assert L.mamg_gen_bidomain_size(2, 1024, C.byref(N), C.byref(nnz)) == 0
    assert N.value == 2101250
    assert L.mamg_gen_bidomain_size(4, 8, C.byref(N), C.byref(nnz)) == -1
    assert M.problems.finest_n(3, 6) == 256 and M.problems.finest_n(2, 6) == 1024


def test_bad_csr_rejected(lib_built):
    import metric_amg_examples_amd as M
    ip = np.array([0, 1, 5], np.int64)        # rowptr[n] != nnz
    ix = np.array([0, 1], np.int32)
    dv = np.ones(2)
    with pytest.raises(ValueError):
        M.HostHierarchy((ip, ix, dv))
    # column out of range / non-monotone rowptr: rejected by the C side
    ip = np.array([0, 1, 2], np.int64)
    ix = np.array([0, 7], np.int32)
    with pytest.raises(M._lib.MamgError) as ei:
        M.HostHierarchy((ip, ix, dv))
    assert ei.value.code == -1


def test_no_cpu_fallback_without_gpu(lib_built):
    import torch
    import metric_amg_examples_amd as M
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from mamg_oracle import laplace1d
    with pytest.raises(M._lib.MamgError) as ei:
        M.MetricAMG(laplace1d(30))
    assert ei.value.code == -2                # HIP error, never a CPU fallback


def _dist_rc(M, s, prm):
    L = M._lib.lib()
    csr = M._lib.as_csr_struct(s.indptr, s.indices, s.data, s.N)
    cid, out = (C.c_char * 128)(), C.c_void_p()
    rc = L.mamg_setup_dist(C.byref(csr), None, 0, C.byref(prm), 0, 2, cid, 0, C.byref(out))
    return rc, L.mamg_last_error().decode()


def test_setup_dist_parameter_checks_before_gpu(lib_built):
    """mamg_setup_dist (include/mamg.h, multi-GPU section) takes V and W cycles:
    a W-cycle profile passes every parameter check and reaches the device
    (no device here: MAMG_ERR_HIP), as do the node-patch and the seed-ring
    Schwarz, while an invalid cycle and maxit > 1 are refused before the
    rank touches its GPU."""
    import torch
    import metric_amg_examples_amd as M
    if torch.cuda.is_available():
        pytest.skip('GPU present: tests/test_gpu_dist.py runs the W cycle on two ranks')
    P = M.parameters
    s = M.problems.bidomain(2, 16, 1e4)
    for cyc in (P.V_CYCLE, P.W_CYCLE):
        rc, msg = _dist_rc(M, s, P.make_params(P.parameters_metric_mi355x, cycle_type=cyc))
        assert rc == -2 and 'hip' in msg.lower(), (cyc, rc, msg)
    rc, msg = _dist_rc(M, s, P.make_params(P.parameters_metric_mi355x, cycle_type=3))
    assert rc == -4, msg
    rc, msg = _dist_rc(M, s, P.make_params(P.parameters_metric_mi355x, maxit=2))
    assert rc == -4 and 'maxit' in msg
    # the node patches run on N GPUs (round 5): they pass to the device
    rc, msg = _dist_rc(M, s, P.make_params(P.parameters_metric_schwarz_gpu_mapped))
    assert rc == -2 and 'hip' in msg.lower(), msg
    # the seed rings run on N GPUs too (round 6): they pass to the device
    rc, msg = _dist_rc(M, s, P.make_params(P.parameters_metric_mi355x_patch, Schwarz_type=P.SCHWARZ_RINGS,
                                           Schwarz_maxlvl=2))
    assert rc == -2 and 'hip' in msg.lower(), msg


def test_num_functions_inference_is_reported_and_overridable(lib_built):
    """MetricAMG / DistMetricAMG infer num_functions from a W of equal blocks
    (amg.py _with_functions); the inference is a note, a UserWarning when a
    reference dict without num_functions is passed, and a caller's
    num_functions (keyword or dict) always wins."""
    import warnings
    import metric_amg_examples_amd as M
    from metric_amg_examples_amd.amg import _with_functions
    P = M.parameters
    W = [100, 100]
    ov, notes = _with_functions(W, None, {})
    assert ov == {'num_functions': 2} and len(notes) == 1 and 'num_functions=1' in notes[0]
    with pytest.warns(UserWarning, match='inferred from W'):
        ov, notes = _with_functions(W, P.parameters_standard, {})
    assert ov['num_functions'] == 2
    with warnings.catch_warnings():
        warnings.simplefilter('error')
        ov, notes = _with_functions(W, P.parameters_standard, {'num_functions': 1})
        assert ov == {'num_functions': 1} and notes == []
        ov, notes = _with_functions(W, dict(P.parameters_standard, num_functions=1), {})
        assert ov == {} and notes == []
        assert _with_functions([100, 50], P.parameters_standard, {}) == ({}, [])
        assert _with_functions(None, P.parameters_standard, {}) == ({}, [])
    assert P.make_params(P.parameters_standard, **_with_functions(W, P.parameters_standard,
                                                                   {'num_functions': 1})[0]).num_functions == 1


def test_no_stream_ordered_pool_or_contiguous_allocations(lib_built):
    """the runtime's stream-ordered pool hands out
    live blocks that share physical memory (bench/contig_alias.hip), and the
    contiguous re-homed arrays broke the next setup; the library imports
    neither allocator (its setup temporaries come from dmem.h's own cache)."""
    import subprocess
    so = os.path.join(ROOT, 'metric-amg-examples_amd', 'libmamg.so')
    out = subprocess.run(['nm', '-D', '--undefined-only', so], capture_output=True, text=True,
                         check=True).stdout
    imported = set(re.findall(r'\b(hip\w+)@', out))
    assert 'hipMalloc' in imported
    for bad in ('hipMallocAsync', 'hipFreeAsync', 'hipMallocFromPoolAsync', 'hipExtMallocWithFlags'):
        assert bad not in imported, bad


def test_release_setup_cache_without_gpu(lib_built):
    """mamg_release_setup_cache (include/mamg.h): with nothing cached it makes
    no device call, so it returns 0 on a host without a GPU too."""
    import metric_amg_examples_amd as M
    M.release_setup_cache()


PRODUCT_OPTIONS = ('MAMG_POST_K', 'MAMG_SELL_MIN_ROWS', 'MAMG_MSELL_MIN_ROWS', 'MAMG_TAIL_NODES', 'MAMG_TAIL_VL',
                   'MAMG_TAIL_LDS', 'MAMG_TAIL_PROG_LDS', 'MAMG_TAIL_RES', 'MAMG_HALF', 'MAMG_HALF_BANDS', 'MAMG_R_BANDS', 'MAMG_K_SORT', 'MAMG_K_COL16',
                   'MAMG_FUSE_RBD',
                   'MAMG_CSR2BSR_FILL', 'MAMG_KREGION_TRIES', 'MAMG_KREGION_BUDGET_MS', 'MAMG_REHOME',
                   'MAMG_PRERESERVE_B_PER_NNZ', 'MAMG_POISON', 'MAMG_OVERLAP', 'MAMG_DIST_TEST', 'MAMG_SPGEMM_PAIR',
                   'MAMG_SPGEMM_STAGE_GB', 'MAMG_SPGEMM_STAGE_STRIDE', 'MAMG_MIS_STAGED', 'MAMG_UPLOAD_THREADS',
                   'MAMG_PATCH_INV')


def _diag_regions(src):
    """line numbers inside #if MAMG_DIAG ... (#else | #endif) blocks"""
    inside, stack, out = False, [], set()
    for i, line in enumerate(src.split('\n'), 1):
        t = line.strip()
        if t.startswith('#if'):
            stack.append(t.startswith('#if MAMG_DIAG'))
        elif t.startswith('#else') and stack:
            stack[-1] = False if stack[-1] else stack[-1]
        elif t.startswith('#endif') and stack:
            stack.pop()
        inside = any(stack)
        if inside:
            out.add(i)
    return out


def test_product_reads_no_environment(lib_built):
    """the product library's switches are set only
    through mamg_set_option (include/mamg_test.h), a fixed list; every getenv
    in the library's sources sits in a diagnosis-build block (#if MAMG_DIAG)."""
    import metric_amg_examples_amd as M
    assert M._lib.option_names() == list(PRODUCT_OPTIONS)
    with pytest.raises(M._lib.MamgError) as ei:
        M._lib.set_option('MAMG_TMP_KEEP', '1')        # gone: the cache limit replaces it
    assert ei.value.code == -1 and 'MAMG_HALF' in str(ei.value)
    M._lib.set_option('MAMG_HALF', '0')
    M._lib.set_option('MAMG_HALF', None)
    csrc = os.path.join(ROOT, 'metric-amg-examples_amd', 'csrc')
    for f in sorted(os.listdir(csrc)):
        if not f.endswith(('.hip', '.cpp', '.h')):
            continue
        src = open(os.path.join(csrc, f)).read()
        diag = _diag_regions(src)
        for i, line in enumerate(src.split('\n'), 1):
            code = line.split('//')[0]
            if 'getenv(' in code:
                assert i in diag, '%s:%d reads the environment outside #if MAMG_DIAG: %s' % (f, i, line.strip())
    prod = open(lib_built, 'rb').read()
    assert b'MAMG_TMP_KEEP' not in prod and b'MAMG_GRAPH_MAX_OPS' not in prod


def test_setup_cache_limit_api(lib_built):
    """mamg_set_setup_cache_limit / mamg_setup_cache_bytes (include/mamg.h):
    the bound of the idle setup cache, default (< 0) an eighth of the device's
    HBM (the GPU test checks the value and that a setup leaves at most that)."""
    import metric_amg_examples_amd as M
    L = M._lib.lib()
    idle, lim = C.c_int64(-1), C.c_int64(-1)
    M._lib.check(L.mamg_set_setup_cache_limit(5 * 10**9))
    M._lib.check(L.mamg_setup_cache_bytes(0, C.byref(idle), C.byref(lim)))
    assert lim.value == 5 * 10**9 and idle.value == 0
    M._lib.check(L.mamg_set_setup_cache_limit(-1))
    assert L.mamg_setup_cache_bytes(64, None, None) == -1

"""AMG parameter dictionaries with the reference's key names.

Keys and enum *names* follow /root/reference/src/amg_parameters.py:3-89 and
/root/reference/src/utils.py:20-38,60-82 (haznics constants).  Numeric enum
values are build-defined (HAZmath's are not available here).

* ``parameters_standard``, ``parameters_standard_schwarz``,
  ``parameters_metric``, ``parameters_metric_schwarz``: the reference's
  presets with their values verbatim.  ``MetricAMG`` runs what they select
  (parameters_standard: UA + sequential Vanek-Mandel-Brezina aggregation
  (VMB) + W-cycle + multicolour SGS + coarse scaling;
  parameters_metric_schwarz: UA + parallel HEM + W-cycle + multicolour SGS
  + coarse scaling, and on level 0 the reference's SCHWARZ_SYMMETRIC on the
  seeds' overlapping 1-ring blocks, which on a nodal system with a seed on
  every node is exactly ``SCHWARZ_PATCHES``, and ``SCHWARZ_RINGS`` for sparse
  seed sets) or raises MAMG_ERR_UNSUPPORTED naming the component it lacks
  (SGS and multiplicative Schwarz on scalar systems); there is no silent
  substitution under these names.  ``MetricAMG(A, W, ...)``
  takes ``num_functions`` from W (equal-sized blocks) when the dict does
  not set it, as the reference's metricAMG receives the block space W.
* ``parameters_metric_mi355x``: the GPU profile "mi355x_sa_v" (nodal SA,
  V-cycle, node-block Jacobi): the north star's profile, the drivers' and
  the bench's default.
* ``parameters_metric_mi355x_poly``: the same with the Chebyshev smoother --
  the shortest time to solution measured.
* ``parameters_metric_mi355x_sgs``: the reference's smoother family on the
  GPU: multicolour node-block SGS on every level (level 0: the SGS order on
  the non-overlapping seed blocks, ``SCHWARZ_SEED_BLOCKS``), coarse-grid
  correction scaling ON.
* ``parameters_metric_mi355x_patch``: the reference's level-0 smoother --
  symmetric multiplicative Schwarz on the seeds' overlapping 1-ring blocks
  (``SCHWARZ_PATCHES``), node-block Jacobi below.
  ``SCHWARZ_SYMMETRIC`` keeps the reference's meaning (overlapping
  seed + ``Schwarz_maxlvl``-ring blocks): with ``Schwarz_maxlvl`` 1 on a
  nodal system it runs as ``SCHWARZ_PATCHES``; ``SCHWARZ_SEED_BLOCKS``
  names the non-overlapping seed blocks under the level smoother.
* ``parameters_metric_3d1d``: additive overlapping Schwarz on the 1-D seeds'
  rings.
* ``parameters_metric_default`` / ``parameters_amg_default``: the dicts the
  reference's factories use when called without parameters
  (src/utils.py:60-82 / :20-38); ``precond`` falls back to them, so
  ``get_hazmath_metric_precond(A, W, bcs, interface_dofs=...)`` (the EMI
  drivers) runs the reference's SCHWARZ_SYMMETRIC on the interface seeds'
  2-rings as ``SCHWARZ_RINGS``.
* ``to_gpu_profile(d)``: explicit opt-in mapping of a HAZmath dict onto
  implemented components; returns the mapped dict and every substitution.
  ``*_gpu_mapped`` are the reference presets passed through it.
"""
from __future__ import annotations

import ctypes as C

from . import _lib

# ---- enums (names as haznics exposes them) --------------------------------
UA_AMG, SA_AMG = 1, 2
V_CYCLE, W_CYCLE = 1, 2
SMOOTHER_JACOBI, SMOOTHER_L1DIAG, SMOOTHER_JACOBI_RHO = 1, 2, 3
SMOOTHER_GS, SMOOTHER_SGS = 10, 11
SMOOTHER_POLY = 12            # Chebyshev polynomial in W A (HAZmath/FASP SMOOTHER_POLY)
VMB, MIS, MWM, HEC, HEM = 1, 2, 3, 4, 5
SCHWARZ_FORWARD, SCHWARZ_BACKWARD, SCHWARZ_SYMMETRIC, SCHWARZ_BLOCK_JACOBI = 1, 2, 3, 4
SCHWARZ_ADDITIVE = 5          # overlapping seed + Schwarz_maxlvl-ring blocks, additive (sparse seed sets)
SCHWARZ_PATCHES = 6           # the reference's overlapping seed + 1-ring blocks, symmetric multiplicative
                              # (one patch per node, distance-3 multicolour order; level 0, nodal)
SCHWARZ_SEED_BLOCKS = 7       # the level smoother on non-overlapping seed blocks (seed + joined non-seeds)
SCHWARZ_RINGS = 8             # the reference's overlapping seed + Schwarz_maxlvl-ring blocks, symmetric
                              # multiplicative (one block per seed, greedy conflict colours) + node-block GS
                              # on the dofs in no block (level 0, nodal; sparse seed sets such as EMI's)
OFF, ON = 0, 1
STRENGTH_DIAG, STRENGTH_ROWMAX = 0, 1   # strength_measure: classical theta sqrt(|a_ii a_jj|) | row maximum (default)
SOLVER_UMFPACK = 32          # coarse_solver / Schwarz_blksolver: dense direct here

KEYS = ('prectype', 'AMG_type', 'cycle_type', 'max_levels', 'maxit', 'smoother',
        'relaxation', 'presmooth_iter', 'postsmooth_iter', 'coarse_dof',
        'coarse_solver', 'coarse_scaling', 'aggregation_type', 'strong_coupled',
        'max_aggregation', 'amli_degree', 'Schwarz_levels', 'Schwarz_mmsize',
        'Schwarz_maxlvl', 'Schwarz_type', 'Schwarz_blksolver', 'print_level',
        # build-defined extensions
        'sa_omega', 'rho_iters', 'max_coarse_dense', 'device', 'spmv_lanes',
        'num_functions', 'node_block_smoother', 'sa_block_diag', 'post_fusion',
        'poly_degree', 'poly_ratio', 'strength_measure')

# ---- the GPU profile "mi355x_sa_v"  -------------------
parameters_metric_mi355x = {
    "AMG_type": SA_AMG,
    "cycle_type": V_CYCLE,
    "max_levels": 20,
    "maxit": 1,
    "smoother": SMOOTHER_JACOBI_RHO,
    "relaxation": 4.0 / 3.0,
    "presmooth_iter": 1,
    "postsmooth_iter": 1,
    "coarse_dof": 100,
    "coarse_solver": SOLVER_UMFPACK,
    "coarse_scaling": OFF,
    "aggregation_type": MIS,
    "strong_coupled": 0.0,        # nodal strength: theta = 0 (0.08 stalls coarsening)
    "max_aggregation": 100,
    "amli_degree": 3,
    "Schwarz_levels": 1,
    "Schwarz_mmsize": 100,
    "Schwarz_maxlvl": 1,          # non-overlapping partition of the seeds' 1-rings
    "Schwarz_type": SCHWARZ_BLOCK_JACOBI,
    "Schwarz_blksolver": SOLVER_UMFPACK,
    "print_level": 0,
    "num_functions": 2,
}

# the same hierarchy with the Chebyshev smoother (SMOOTHER_POLY, degree 2 on
# [relaxation / 16, relaxation] of W A): half the PCG iterations of node-block
# Jacobi for two extra level-0 SpMVs per cycle
parameters_metric_mi355x_poly = dict(
    parameters_metric_mi355x, smoother=SMOOTHER_POLY, poly_degree=2, poly_ratio=16.0)

# 3D-1D (sparse 1-D seeds, scalar hierarchy, CSR layout): the seeds' 2-ring
# blocks (src/input_metric.dat:96-100) overlapping, smoothed additively --
# the parallel counterpart of HAZmath's multiplicative Schwarz there, which
# is what makes the averaged coupling gamma-robust
parameters_metric_3d1d = dict(
    parameters_metric_mi355x, num_functions=1, Schwarz_type=SCHWARZ_ADDITIVE, Schwarz_maxlvl=2,
    Schwarz_mmsize=200, coarse_dof=300, max_levels=30)

# the reference's smoothers on the GPU: multicolour
# node-block SGS (level 0: the same SGS order on the non-overlapping seed
# blocks) and coarse-grid correction scaling, on the nodal SA V-cycle
parameters_metric_mi355x_sgs = dict(
    parameters_metric_mi355x, smoother=SMOOTHER_SGS, coarse_scaling=ON,
    Schwarz_type=SCHWARZ_SEED_BLOCKS)

# the reference's level-0 smoother on the GPU:
# symmetric multiplicative Schwarz on the seeds' overlapping 1-ring blocks
# (src/amg_parameters.py:83-87, src/utils.py:84) = one patch per node, exact
# local solves; node-block Jacobi on the coarser levels of the SA V-cycle.
# PCG iterations within 1.2x of the reference algorithm's (oracle, 3-D)
parameters_metric_mi355x_patch = dict(parameters_metric_mi355x, Schwarz_type=SCHWARZ_PATCHES)

# ---- the reference's presets, verbatim values (src/amg_parameters.py) ------
parameters_standard = {
    "prectype": 2, "AMG_type": UA_AMG, "cycle_type": W_CYCLE, "max_levels": 20, "maxit": 1,
    "smoother": SMOOTHER_SGS, "relaxation": 1.2, "presmooth_iter": 1, "postsmooth_iter": 1,
    "coarse_dof": 100, "coarse_solver": 32, "coarse_scaling": ON, "aggregation_type": VMB,
    "strong_coupled": 0.1, "max_aggregation": 100, "Schwarz_levels": 0, "print_level": 10,
}
parameters_standard_schwarz = dict(
    parameters_standard, Schwarz_levels=1, Schwarz_mmsize=100, Schwarz_maxlvl=1,
    Schwarz_type=SCHWARZ_SYMMETRIC, Schwarz_blksolver=32, print_level=5)
parameters_metric = {
    "AMG_type": UA_AMG, "cycle_type": W_CYCLE, "max_levels": 20, "maxit": 1,
    "smoother": SMOOTHER_SGS, "relaxation": 1.2, "presmooth_iter": 1, "postsmooth_iter": 1,
    "coarse_dof": 100, "coarse_solver": 32, "coarse_scaling": ON, "aggregation_type": HEM,
    "strong_coupled": 0.1, "max_aggregation": 100, "amli_degree": 3, "Schwarz_levels": 0,
    "print_level": 5,
}
parameters_metric_schwarz = dict(
    parameters_metric, Schwarz_levels=1, Schwarz_mmsize=100, Schwarz_maxlvl=1,
    Schwarz_type=SCHWARZ_SYMMETRIC, Schwarz_blksolver=32)
# the defaults the reference's factories fall back to when called without
# parameters: get_hazmath_metric_precond(_mono) (src/utils.py:60-82; the EMI
# drivers' call, src/emi_3d.py:139, src/emi_2d.py:207) and
# get_hazmath_amg_precond (src/utils.py:20-38).  On a nodal system with
# sparse seeds the first runs SCHWARZ_SYMMETRIC on the seeds' 2-rings as
# SCHWARZ_RINGS; with a seed on every node its 2-rings are too (the 1-ring
# node patches need Schwarz_maxlvl 1)
parameters_metric_default = {
    "AMG_type": UA_AMG, "cycle_type": W_CYCLE, "max_levels": 20, "maxit": 1,
    "smoother": SMOOTHER_SGS, "relaxation": 1.2, "presmooth_iter": 1, "postsmooth_iter": 1,
    "coarse_dof": 100, "coarse_solver": 32, "coarse_scaling": ON, "aggregation_type": HEM,
    "strong_coupled": 0.1, "max_aggregation": 100, "amli_degree": 3, "Schwarz_levels": 1,
    "Schwarz_mmsize": 100, "Schwarz_maxlvl": 2, "Schwarz_type": SCHWARZ_SYMMETRIC,
    "Schwarz_blksolver": 32, "print_level": 10,
}
parameters_amg_default = {
    "prectype": 2, "AMG_type": UA_AMG, "cycle_type": W_CYCLE, "max_levels": 20, "maxit": 1,
    "smoother": SMOOTHER_SGS, "relaxation": 1.2, "presmooth_iter": 1, "postsmooth_iter": 1,
    "coarse_dof": 100, "coarse_solver": 32, "coarse_scaling": ON, "aggregation_type": VMB,
    "strong_coupled": 0.1, "max_aggregation": 100, "Schwarz_levels": 0, "print_level": 10,
}
# round-1 names of the same verbatim dicts
hazmath_parameters_standard = parameters_standard
hazmath_parameters_standard_schwarz = parameters_standard_schwarz
hazmath_parameters_metric = parameters_metric
hazmath_parameters_metric_schwarz = parameters_metric_schwarz


def to_gpu_profile(params: dict) -> tuple[dict, list[str]]:
    """Map a HAZmath parameter dict onto implemented components (explicit
    opt-in).  Returns (mapped dict, list of human-readable substitutions)."""
    out = dict(params)
    notes = []
    if out.get('aggregation_type', MIS) not in (MIS, HEM, VMB):
        notes.append('aggregation_type %r -> MIS (deterministic parallel MIS-2)'
                     % out.get('aggregation_type'))
        out['aggregation_type'] = MIS
    if out.get('Schwarz_levels', 0) > 1:
        notes.append('Schwarz_levels %d -> 1' % out['Schwarz_levels'])
        out['Schwarz_levels'] = 1
    smo = out.get('smoother', SMOOTHER_JACOBI_RHO)
    gsm = smo in (SMOOTHER_GS, SMOOTHER_SGS)
    st, lvl = out.get('Schwarz_type'), out.get('Schwarz_maxlvl', 1)
    if out.get('Schwarz_levels', 0) >= 1:
        if st == SCHWARZ_SYMMETRIC and lvl == 1:
            # the library runs this as given on a nodal system; stated here too
            notes.append('Schwarz_type SCHWARZ_SYMMETRIC on the seeds\' 1-rings = SCHWARZ_PATCHES (the same '
                         'overlapping blocks, multiplicative in a distance-3 multicolour order; nodal systems '
                         'with a seed on every node) or, for sparse seed sets, SCHWARZ_RINGS')
            out['Schwarz_type'] = SCHWARZ_PATCHES
            out['num_functions'] = 2
        elif st == SCHWARZ_SYMMETRIC and lvl >= 2:
            notes.append('Schwarz_type SCHWARZ_SYMMETRIC on the seeds\' %d-rings = SCHWARZ_RINGS (the same '
                         'overlapping blocks, multiplicative in a greedy conflict-colour order, node-block GS on '
                         'the rest; nodal systems)' % lvl)
            out['Schwarz_type'] = SCHWARZ_RINGS
            out['num_functions'] = 2
        elif st in (SCHWARZ_FORWARD, SCHWARZ_BACKWARD) and lvl >= 1:
            notes.append('Schwarz_type %r on overlapping seed + %d-ring blocks -> SCHWARZ_SEED_BLOCKS (the level '
                         'smoother on the non-overlapping seed blocks, seed + joined 1-ring)' % (st, lvl))
            out['Schwarz_type'] = SCHWARZ_SEED_BLOCKS
            out['Schwarz_maxlvl'] = 1
        elif st in (SCHWARZ_BLOCK_JACOBI, SCHWARZ_ADDITIVE) and gsm:
            notes.append('Schwarz_type %r -> SCHWARZ_SEED_BLOCKS (GS/SGS on the seed blocks)' % st)
            out['Schwarz_type'] = SCHWARZ_SEED_BLOCKS
        elif st is None:
            out['Schwarz_type'] = SCHWARZ_SEED_BLOCKS if gsm else SCHWARZ_BLOCK_JACOBI
        if out.get('Schwarz_maxlvl', 1) > 1 and out['Schwarz_type'] not in (SCHWARZ_ADDITIVE, SCHWARZ_RINGS):
            notes.append('Schwarz_maxlvl %d -> 1' % out['Schwarz_maxlvl'])
            out['Schwarz_maxlvl'] = 1
    if smo in (SMOOTHER_GS, SMOOTHER_SGS) and out.get('num_functions', 1) != 2:
        notes.append('num_functions -> 2 (the multicolour GS smoothers are node-block smoothers)')
        out['num_functions'] = 2
    out.pop('prectype', None)
    return out, notes


# the reference presets through to_gpu_profile
parameters_standard_gpu_mapped = to_gpu_profile(parameters_standard)[0]
parameters_standard_schwarz_gpu_mapped = to_gpu_profile(parameters_standard_schwarz)[0]
parameters_metric_gpu_mapped = to_gpu_profile(parameters_metric)[0]
parameters_metric_schwarz_gpu_mapped = to_gpu_profile(parameters_metric_schwarz)[0]


def make_params(parameters: dict | None = None, **overrides) -> _lib.mamg_params:
    """dict with reference key names -> struct mamg_params (defaults =
    parameters_metric_mi355x).  Unknown keys raise KeyError."""
    p = _lib.mamg_params()
    _lib.lib().mamg_params_default(C.byref(p))
    merged = dict(parameters or {})
    merged.update(overrides)
    for k, v in merged.items():
        if k not in KEYS:
            raise KeyError('unknown AMG parameter %r' % k)
        if k == 'prectype':
            continue                      # HAZmath precond selector; single type here
        setattr(p, k, type(getattr(p, k))(v))
    return p


def params_to_dict(p: _lib.mamg_params) -> dict:
    return {k: getattr(p, k) for k, _ in p._fields_}

"""AMG parameter dictionaries with the reference's key names.

Keys and enum *names* follow /root/reference/src/amg_parameters.py:3-89 and
/root/reference/src/utils.py:20-38,60-82 (haznics constants).  Numeric enum
values are build-defined (HAZmath's are not available here).

The reference's presets select sequential HAZmath components (SGS smoother,
multiplicative Schwarz, VMB/HEM aggregation, coarse scaling) that cannot be
reproduced on a GPU.  ``MetricAMG`` rejects them with MAMG_ERR_UNSUPPORTED
(no silent fallback).  ``to_gpu_profile`` maps such a dict to the nearest
GPU-parallel components and reports every substitution; the presets below
with the reference's names are those mapped versions, so a driver that does
``amgparams = parameters.parameters_metric_schwarz`` runs unchanged.
"""
from __future__ import annotations

import ctypes as C

from . import _lib

# ---- enums (names as haznics exposes them) --------------------------------
UA_AMG, SA_AMG = 1, 2
V_CYCLE, W_CYCLE = 1, 2
SMOOTHER_JACOBI, SMOOTHER_L1DIAG, SMOOTHER_JACOBI_RHO = 1, 2, 3
SMOOTHER_GS, SMOOTHER_SGS = 10, 11
VMB, MIS, MWM, HEC, HEM = 1, 2, 3, 4, 5
SCHWARZ_FORWARD, SCHWARZ_BACKWARD, SCHWARZ_SYMMETRIC, SCHWARZ_BLOCK_JACOBI = 1, 2, 3, 4
OFF, ON = 0, 1
SOLVER_UMFPACK = 32          # coarse_solver / Schwarz_blksolver: dense direct here

KEYS = ('prectype', 'AMG_type', 'cycle_type', 'max_levels', 'maxit', 'smoother',
        'relaxation', 'presmooth_iter', 'postsmooth_iter', 'coarse_dof',
        'coarse_solver', 'coarse_scaling', 'aggregation_type', 'strong_coupled',
        'max_aggregation', 'amli_degree', 'Schwarz_levels', 'Schwarz_mmsize',
        'Schwarz_maxlvl', 'Schwarz_type', 'Schwarz_blksolver', 'print_level',
        # build-defined extensions
        'sa_omega', 'rho_iters', 'max_coarse_dense', 'device', 'spmv_lanes',
        'num_functions', 'node_block_smoother', 'sa_block_diag', 'post_fusion')

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
    "Schwarz_maxlvl": 1,
    "Schwarz_type": SCHWARZ_BLOCK_JACOBI,
    "Schwarz_blksolver": SOLVER_UMFPACK,
    "print_level": 0,
}

# ---- the reference's presets, verbatim values (src/amg_parameters.py) ------
hazmath_parameters_standard = {
    "prectype": 2, "AMG_type": UA_AMG, "cycle_type": W_CYCLE, "max_levels": 20, "maxit": 1,
    "smoother": SMOOTHER_SGS, "relaxation": 1.2, "presmooth_iter": 1, "postsmooth_iter": 1,
    "coarse_dof": 100, "coarse_solver": 32, "coarse_scaling": ON, "aggregation_type": VMB,
    "strong_coupled": 0.1, "max_aggregation": 100, "Schwarz_levels": 0, "print_level": 10,
}
hazmath_parameters_standard_schwarz = dict(
    hazmath_parameters_standard, Schwarz_levels=1, Schwarz_mmsize=100, Schwarz_maxlvl=1,
    Schwarz_type=SCHWARZ_SYMMETRIC, Schwarz_blksolver=32, print_level=5)
hazmath_parameters_metric = {
    "AMG_type": UA_AMG, "cycle_type": W_CYCLE, "max_levels": 20, "maxit": 1,
    "smoother": SMOOTHER_SGS, "relaxation": 1.2, "presmooth_iter": 1, "postsmooth_iter": 1,
    "coarse_dof": 100, "coarse_solver": 32, "coarse_scaling": ON, "aggregation_type": HEM,
    "strong_coupled": 0.1, "max_aggregation": 100, "amli_degree": 3, "Schwarz_levels": 0,
    "print_level": 5,
}
hazmath_parameters_metric_schwarz = dict(
    hazmath_parameters_metric, Schwarz_levels=1, Schwarz_mmsize=100, Schwarz_maxlvl=1,
    Schwarz_type=SCHWARZ_SYMMETRIC, Schwarz_blksolver=32)


def to_gpu_profile(params: dict) -> tuple[dict, list[str]]:
    """Map a HAZmath parameter dict onto GPU-parallel components.

    Returns (mapped dict, list of human-readable substitutions)."""
    out = dict(params)
    notes = []
    if out.get('smoother') in (SMOOTHER_GS, SMOOTHER_SGS):
        notes.append('smoother SGS/GS -> SMOOTHER_JACOBI_RHO (relaxation/rho(D^-1A) Jacobi)')
        out['smoother'] = SMOOTHER_JACOBI_RHO
    if out.get('aggregation_type', MIS) != MIS:
        notes.append('aggregation_type %r -> MIS (deterministic parallel MIS-2)'
                     % out.get('aggregation_type'))
        out['aggregation_type'] = MIS
    if out.get('coarse_scaling', OFF) == ON:
        notes.append('coarse_scaling ON -> OFF (keeps the cycle linear/symmetric for CG)')
        out['coarse_scaling'] = OFF
    if out.get('Schwarz_levels', 0) >= 1 and out.get('Schwarz_type') != SCHWARZ_BLOCK_JACOBI:
        notes.append('Schwarz_type %r -> SCHWARZ_BLOCK_JACOBI (additive seed blocks)'
                     % out.get('Schwarz_type'))
        out['Schwarz_type'] = SCHWARZ_BLOCK_JACOBI
    if out.get('Schwarz_levels', 0) > 1:
        notes.append('Schwarz_levels %d -> 1' % out['Schwarz_levels'])
        out['Schwarz_levels'] = 1
    out.pop('prectype', None)
    return out, notes


# reference names -> GPU-mapped presets (drop-in for src/amg_parameters.py)
parameters_standard = to_gpu_profile(hazmath_parameters_standard)[0]
parameters_standard_schwarz = to_gpu_profile(hazmath_parameters_standard_schwarz)[0]
parameters_metric = to_gpu_profile(hazmath_parameters_metric)[0]
parameters_metric_schwarz = to_gpu_profile(hazmath_parameters_metric_schwarz)[0]


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

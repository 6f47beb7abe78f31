"""metric-amg-examples_amd: MI355X-native metric-AMG preconditioner.

Drop-in for the reference's `metric_mono` hot path:
    from metric_amg_examples_amd import metricAMG, ConjGrad, parameters
    BB = metricAMG(AA_, W, idofs=interface_dofs, parameters=parameters.parameters_metric_mi355x)
    AAinv = ConjGrad(AA_, precond=BB, tolerance=1e-8, maxiter=500)
    xx = AAinv * bb_
Block form (src/utils.py:45-53): precond.get_hazmath_metric_precond -> R.T * Minv * R.
File boundary (src/utils.py:304-333, src/run_solver_3d1d.py): fileio, drivers.
"""
from . import _lib, fileio, parameters, precond, problems
from .amg import DistMetricAMG, DistPlan, GlooExchange, HostHierarchy, MetricAMG, metricAMG
from .krylov import ConjGrad, DistConjGrad, lanczos_eigenvalues


def release_setup_cache():
    """Release the device blocks the GPU setups keep cached for the process's
    next setup (include/mamg.h mamg_release_setup_cache): for a caller that
    shares the GPU with other allocators, after its setups."""
    rc = _lib.lib().mamg_release_setup_cache()
    if rc:
        raise RuntimeError('mamg_release_setup_cache failed (%d)' % rc)


__all__ = ['MetricAMG', 'metricAMG', 'HostHierarchy', 'DistPlan', 'DistMetricAMG', 'GlooExchange', 'ConjGrad', 'DistConjGrad',
           'lanczos_eigenvalues', 'release_setup_cache', 'parameters', 'problems', 'precond', 'fileio', '_lib']

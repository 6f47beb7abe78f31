import sys, time
sys.path.insert(0, '.')
import numpy as np
import metric_amg_examples_amd as M
P = M.parameters
for n in (16, 32, 64, 128):
    s = M.problems.bidomain(3, n, 1e6)
    A = s.scipy()
    b = M.problems.seeded_rhs(s.N)
    for name, prm in (('standard(VMB)', P.parameters_standard), ('metric(HEM)', P.parameters_metric),
                      ('standard+MIS', dict(P.parameters_standard, aggregation_type=P.MIS))):
        B = M.metricAMG(A, s.W, idofs=s.idofs, parameters=prm)
        cg = M.ConjGrad(A, precond=B, tolerance=1e-8, maxiter=500)
        cg * b
        print(n, name, 'levels', B.num_levels, 'its', len(cg.residuals) - 1, flush=True)
        B.close()

#!/usr/bin/env python3
"""GPU setup phases of the reference family (UA + parallel HEM + W-cycle +
multicolour SGS + coarse scaling, strong_coupled 0.1, coarse_dof 100; the
profile of bench/prof_ref_family.py) at nrefs (default 6): wall seconds and
mamg_setup_timings per setup, one JSON line each, with the MAMG_* switches
set in the environment.

    python bench/ref_setup_phases.py [nrefs] [reps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (the library loads torch's HIP runtime first)
    import metric_amg_examples_amd as M
    nrefs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    s = M.problems.bidomain(3, M.problems.finest_n(3, nrefs), 1e6)
    A = s.scipy()
    for _ in range(reps):
        t = time.time()
        B = M.MetricAMG(A, s.W, idofs=s.idofs, num_functions=2, setup='gpu', AMG_type=1, aggregation_type=5,
                        cycle_type=2, smoother=11, coarse_scaling=1, Schwarz_type=7, coarse_dof=100)
        w = time.time() - t
        print(json.dumps(dict(env={k: v for k, v in os.environ.items() if k.startswith('MAMG_')}, levels=B.num_levels,
                              wall_s=round(w, 3), phases_ms={k: round(v, 1) for k, v in B.setup_timings.items()})),
              flush=True)
        B.close()


if __name__ == '__main__':
    main()

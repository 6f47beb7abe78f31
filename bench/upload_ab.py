#!/usr/bin/env python3
"""A/B of the A_0 upload inside the GPU setup: the bench's
system (bidomain_3d nrefs=6, generated fresh on the host) set up once per
process; prints the setup phases.  Run under the diagnosis build with
MAMG_UPLOAD_PLAIN=1 for the runtime's pageable hipMemcpy, unset for the
staged copy (csrc/gsetup.hip h2d_staged)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import metric_amg_examples_amd as M
    nrefs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    n = M.problems.finest_n(3, nrefs)
    s = M.problems.bidomain(3, n, 1e6)
    torch.cuda.synchronize()
    t0 = time.time()
    B = M.MetricAMG(s, s.W, idofs=s.idofs, num_functions=2, setup='gpu')
    torch.cuda.synchronize()
    print(json.dumps({'plain': os.environ.get('MAMG_UPLOAD_PLAIN', '0'), 'wall_s': round(time.time() - t0, 3),
                      'upload_A0_ms': round(B.setup_timings['upload_A0'], 1),
                      'setup_total_ms': round(B.setup_timings['setup_total'], 1)}), flush=True)
    B.close()


if __name__ == '__main__':
    main()

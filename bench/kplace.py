#!/usr/bin/env python3
"""Placement diagnosis of the level-0 K kernel: within
ONE process, move one array of the K launch at a time into a fresh allocation
(MAMG_KMOVE: val, col, x1, r1, w, e; the same bytes) and time K after each
move, so the kernel's time can be attributed to the placement of one array.

    python bench/kplace.py [--nrefs 6] [--reps 20] [--moves val:4,col:3,x1:3,r1:3,w:3,e:2]

One JSON line per placement: the array moved (or 'start'), K ms, residual ms.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nrefs', type=int, default=6)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--moves', default='val:4,col:3,x1:3,r1:3,w:3,e:2')
    ap.add_argument('--variants', default='0', help='K kernel variants timed at every placement')
    ap.add_argument('--shuffle', type=int, default=0,
                    help='store K\'s SELL slices in a scrambled order (groups of this many slices) first')
    args = ap.parse_args()
    import torch
    import metric_amg_examples_amd as M
    n = M.problems.finest_n(3, args.nrefs)
    s = M.problems.bidomain(3, n, 1e6)
    B = M.MetricAMG(s.scipy(), s.W, idofs=s.idofs, setup='gpu', num_functions=2)
    del s
    r = torch.as_tensor(M.problems.seeded_rhs(B.shape[0])).cuda()
    z = torch.zeros_like(r)
    st = torch.cuda.current_stream()

    def timed(tag):
        for v in args.variants.split(','):   # <K variant>[s|t]: K values split globally / per slot row
            os.environ['MAMG_K_VARIANT'] = v.rstrip('st')
            os.environ['MAMG_K_LAYOUT'] = 'split' if v.endswith('s') else 'split2' if v.endswith('t') else 'block'
            B.time_apply(r, z, 3, 0, st)
            ms, kms, _ = B.time_apply(r, z, args.reps, 0, st)
            print(json.dumps({'moved': tag, 'variant': v, 'K_ms': round(kms[1], 4),
                              'resid_ms': round(kms[0], 4), 'ms_per_apply': round(ms, 4)}), flush=True)
        os.environ['MAMG_K_VARIANT'] = '0'
        os.environ['MAMG_K_LAYOUT'] = 'block'

    if args.shuffle:
        os.environ['MAMG_K_SHUFFLE'] = str(args.shuffle)
        B.time_apply(r, z, 1, 0, st)          # performs the re-layout
        del os.environ['MAMG_K_SHUFFLE']
    timed('start')
    timed('start')
    for item in args.moves.split(','):
        what, cnt = item.split(':')
        for _ in range(int(cnt)):
            os.environ['MAMG_KMOVE'] = what
            B.time_apply(r, z, 1, 0, st)          # performs the move
            del os.environ['MAMG_KMOVE']
            timed(what)
    B.close()


if __name__ == '__main__':
    main()

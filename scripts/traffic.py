#!/usr/bin/env python3
"""Measured HBM bytes per launch of the bench's two dominant kernels, from
rocprofv3 PMC counter CSVs, written to profiles/traffic.json (read by
bench.py as roofline.traffic).

    python scripts/traffic.py FETCH_CSV WRITE_CSV --N 33949186 [--layout bsr2]

Calibration (profiles/r01_pmc_calibration.txt, bench/spmv_micro.hip calib):
on this gfx950 + rocprofv3 stack FETCH_SIZE * 1024 = 0.5 x the bytes a
streaming kernel reads (4..32-byte lanes alike), WRITE_SIZE * 1024 = 1.0 x
the bytes written (full and half 128-byte lines alike).  So
    bytes = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE.
Kernel -> class (per launch, medians over the launches of the largest grid):
  L0_resid        sell2 / hsell2 / bsr2 with EPI_RESID = 2, TAG 0
  L0_smooth_spmv  the fused post kernel: msell <.., KPOST, .., TAG 0> / bsr2_post TAG 0
  L0_restrict     bsr2 with EPI_Y = 0, TAG 0 (R_0 r_1)
  L0_smoother     bd2_kernel at level 0's grid (the first pre-smoothing W r)
and per apply (sum over every launch / the number of L0_resid launches):
  coarse_levels   every TAG >= 1 SpMV / post / GS launch, bd2 below level 0's
                  grid, tail_kernel, gemv_kernel (the coarsest solve)
With --bench-json (a bench.py line with its per-class breakdown) each class
also gets ratio = measured bytes / algorithmic bytes.
"""
import argparse
import csv
import json
import re
import statistics

FETCH_SCALE = 2 * 1024
WRITE_SCALE = 1024


FAMILY = r'(hsell2_kernel|msell_kernel|sell2_kernel|bsr2_kernel|bsr2_post_kernel|gs2_kernel)<([^>]*)>'


def classify(name):
    """level-0 class of one launch, 'coarse' for a coarse-level apply kernel,
    'bd2' for the block-diagonal apply (split by grid later), else None"""
    if re.search(r'\bbd2_kernel<', name):
        return 'bd2'
    if re.search(r'\b(tail_kernel|gemv_kernel)\b', name):
        return 'coarse'
    m = re.search(FAMILY, name)
    if not m:
        return None
    kind, targs = m.group(1), [t.strip() for t in m.group(2).split(',')]
    if kind == 'msell_kernel':          # <LPR, U, EPI, XFM, SYM, SPL, TAG, PROBE>
        if targs[6] != '0':
            return 'coarse'
        return 'L0_smooth_spmv' if targs[2] == '5' else None
    if kind == 'gs2_kernel':
        return None
    if kind == 'bsr2_post_kernel':
        return 'L0_smooth_spmv' if targs[-1] == '0' else 'coarse'
    if kind in ('sell2_kernel', 'hsell2_kernel'):
        epi, xfm, tag = targs[0], targs[1], targs[-1]
    else:                               # bsr2_kernel <VL, EPI, XFM, SYM, TAG, NT>
        epi, xfm, tag = targs[1], targs[2], targs[4]
    if tag != '0':
        return 'coarse'
    if epi == '2' and xfm == 'false':   # EPI_RESID on the internal vectors
        return 'L0_resid'
    if epi == '5':                      # EPI_KPOST: z = x1 + W r1 + K e
        return 'L0_smooth_spmv'
    if epi == '0' and kind == 'bsr2_kernel':
        return 'L0_restrict'
    return None


def collect(path, counter):
    """{class: (grid, median per launch, launches)} for the level-0 classes
    (largest grid), plus 'coarse' as (0, total over every launch, launches)"""
    by, coarse, bd2 = {}, [0.0, 0], {}
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        c = classify(r['Kernel_Name'])
        if c is None:
            continue
        g, v = int(r['Grid_Size']), float(r['Counter_Value'])
        if c == 'coarse':
            coarse[0] += v
            coarse[1] += 1
            continue
        if c == 'bd2':
            bd2.setdefault(g, []).append(v)
            continue
        cur = by.get(c)
        if cur is None or g > cur[0]:
            by[c] = (g, [v])
        elif g == cur[0]:
            cur[1].append(v)
    if bd2:
        g0 = max(bd2)
        by['L0_smoother'] = (g0, bd2[g0])
        for g, vs in bd2.items():
            if g != g0:
                coarse[0] += sum(vs)
                coarse[1] += len(vs)
    out = {c: (g, statistics.median(v), len(v)) for c, (g, v) in by.items()}
    out['coarse_levels'] = (0, coarse[0], coarse[1])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_csv')
    ap.add_argument('write_csv')
    ap.add_argument('--N', type=int, required=True)
    ap.add_argument('--layout', default='bsr2')
    ap.add_argument('--post', default='k', choices=('k', 'merged'),
                    help='post-smoothing operator the profiled run used (MAMG_POST_K)')
    ap.add_argument('--a0', default='half', choices=('half', 'sell'),
                    help='level-0 operator storage of the profiled run')
    ap.add_argument('--out', default='profiles/traffic.json')
    ap.add_argument('--bench-json', default=None,
                    help='bench.py JSON line (with breakdown) of the same config: adds measured / algorithmic')
    a = ap.parse_args()
    f = collect(a.fetch_csv, 'FETCH_SIZE')
    w = collect(a.write_csv, 'WRITE_SIZE')
    napply = f['L0_resid'][2] if 'L0_resid' in f else 0
    kernels, detail = {}, {}
    for c in sorted(f):
        fb = f[c][1] * FETCH_SCALE
        wb = w[c][1] * WRITE_SCALE if c in w else 0.0
        if c == 'coarse_levels':            # totals -> per apply
            if not napply or not f[c][2]:
                continue
            fb, wb = fb / napply, wb / napply
        kernels[c] = round(fb + wb, 1)
        detail[c] = {'grid': f[c][0], 'launches': f[c][2], 'fetch_bytes': round(fb, 1),
                     'write_bytes': round(wb, 1)}
        if c == 'coarse_levels':
            detail[c]['per'] = 'apply (%d applies)' % napply
    ratios = {}
    if a.bench_json:
        line = json.loads(open(a.bench_json).read().strip().splitlines()[-1])
        bd = line.get('breakdown') or {}
        for c, b in kernels.items():
            alg = (bd.get(c) or {}).get('GB')
            if alg:
                ratios[c] = round(b / (alg * 1e9), 3)
                detail[c]['algorithmic_bytes'] = alg * 1e9
    import hashlib
    import os
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'metric-amg-examples_amd',
                       'csrc', 'device.hip')
    sha = hashlib.sha256(open(src, 'rb').read()).hexdigest()
    out = {'layout': a.layout, 'N': a.N, 'post': a.post, 'a0': a.a0, 'device_src_sha256': sha,
           'kernels': kernels, 'ratio_measured_over_algorithmic': ratios, 'detail': detail,
           'calibration': 'bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE (profiles/r01_pmc_calibration.txt)'}
    json.dump(out, open(a.out, 'w'), indent=1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()

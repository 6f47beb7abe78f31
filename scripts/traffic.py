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
Kernel -> class: the largest-grid launch of the level-0 residual
(sell2_kernel / bsr2_kernel with EPI_RESID = 2 and TAG 0) and of the fused
post kernel (bsr2_post_kernel, TAG 0).  Medians over the profiled launches.
"""
import argparse
import csv
import json
import re
import statistics

FETCH_SCALE = 2 * 1024
WRITE_SCALE = 1024


def classify(name):
    m = re.search(r'(hsell2_kernel|msell_kernel|sell2_kernel|bsr2_kernel|bsr2_post_kernel)<([^>]*)>', name)
    if not m:
        return None
    kind, targs = m.group(1), [t.strip() for t in m.group(2).split(',')]
    if kind == 'msell_kernel':          # <LPR, U, EPI, XFM, SYM, SPL, TAG, PROBE>: the level-0 K operator
        return 'L0_smooth_spmv' if targs[2] == '5' and targs[6] == '0' else None
    if kind == 'bsr2_post_kernel':
        return 'L0_smooth_spmv' if targs[-1] == '0' else None
    epi, xfm = (targs[0], targs[1]) if kind in ('sell2_kernel', 'hsell2_kernel') else (targs[1], targs[2])
    if targs[-1] != '0':
        return None
    if epi == '2' and xfm == 'false':   # EPI_RESID on the internal vectors
        return 'L0_resid'
    if epi == '5':                      # EPI_KPOST: z = x1 + W r1 + K e
        return 'L0_smooth_spmv'
    return None


def collect(path, counter):
    by = {}
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        c = classify(r['Kernel_Name'])
        if c is None:
            continue
        g = int(r['Grid_Size'])
        cur = by.get(c)
        if cur is None or g > cur[0]:
            by[c] = (g, [float(r['Counter_Value'])])
        elif g == cur[0]:
            cur[1].append(float(r['Counter_Value']))
    return {c: (g, statistics.median(v), len(v)) for c, (g, v) in by.items()}


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
    a = ap.parse_args()
    f = collect(a.fetch_csv, 'FETCH_SIZE')
    w = collect(a.write_csv, 'WRITE_SIZE')
    kernels, detail = {}, {}
    for c in sorted(f):
        fb = f[c][1] * FETCH_SCALE
        wb = w[c][1] * WRITE_SCALE if c in w else 0.0
        kernels[c] = round(fb + wb, 1)
        detail[c] = {'grid': f[c][0], 'launches': f[c][2], 'fetch_bytes': round(fb, 1),
                     'write_bytes': round(wb, 1)}
    import hashlib
    import os
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'metric-amg-examples_amd',
                       'csrc', 'device.hip')
    sha = hashlib.sha256(open(src, 'rb').read()).hexdigest()
    out = {'layout': a.layout, 'N': a.N, 'post': a.post, 'a0': a.a0, 'device_src_sha256': sha,
           'kernels': kernels, 'detail': detail,
           'calibration': 'bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE (profiles/r01_pmc_calibration.txt)'}
    json.dump(out, open(a.out, 'w'), indent=1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()

#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter CSVs (one or more passes).

    python scripts/pmc_summary.py CSV [CSV ...] [--top 12] [--grid-min 1000000]

For every kernel (name shortened to its template head) with a grid of at
least --grid-min work-items: launches, median duration (us) and the median
of each counter per launch.  Derived, when the counters are present:
  ea_rd_latency   = TCC_EA0_RDREQ_LEVEL_sum / TCC_EA0_RDREQ_sum   (cycles per
                    L2 -> fabric read request in flight)
  dram_frac       = TCC_EA0_RDREQ_DRAM_sum / TCC_EA0_RDREQ_sum
  tcp_tcc_latency = TCP_TCC_READ_REQ_LATENCY_sum / TCP_TCC_READ_REQ_sum
  utcl1_miss_rate = TCP_UTCL1_TRANSLATION_MISS_sum / TCP_UTCL1_REQUEST_sum
  vmem_latency    = SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM (cycles per VMEM instruction)
"""
import argparse
import collections
import csv
import json
import re
import statistics


def short(name):
    m = re.search(r'::([a-z0-9_]+_kernel)<([^>]*)>', name)
    if m:
        return '%s<%s>' % (m.group(1), m.group(2).replace(' ', ''))
    m = re.search(r'([A-Za-z0-9_]+)\(', name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv', nargs='+')
    ap.add_argument('--grid-min', type=int, default=1000000)
    ap.add_argument('--json', default=None)
    args = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(dict)
    for path in args.csv:
        with open(path) as f:
            for row in csv.DictReader(f):
                if int(row['Grid_Size']) < args.grid_min:
                    continue
                k = short(row['Kernel_Name'])
                vals[k][row['Counter_Name']].append(float(row['Counter_Value']))
                durs[k][(path, row['Dispatch_Id'])] = (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) / 1e3
    out = {}
    for k, cs in vals.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        d = {'launches': max(len(v) for v in cs.values()), 'dur_us': round(statistics.median(durs[k].values()), 1)}
        d.update({c: round(v, 1) for c, v in sorted(med.items())})

        def ratio(a, b):
            return round(med[a] / med[b], 3) if a in med and b in med and med[b] else None
        for name, a, b in (('ea_rd_latency', 'TCC_EA0_RDREQ_LEVEL_sum', 'TCC_EA0_RDREQ_sum'),
                           ('dram_frac', 'TCC_EA0_RDREQ_DRAM_sum', 'TCC_EA0_RDREQ_sum'),
                           ('tcp_tcc_latency', 'TCP_TCC_READ_REQ_LATENCY_sum', 'TCP_TCC_READ_REQ_sum'),
                           ('utcl1_miss_rate', 'TCP_UTCL1_TRANSLATION_MISS_sum', 'TCP_UTCL1_REQUEST_sum'),
                           ('vmem_latency', 'SQ_INST_LEVEL_VMEM', 'SQ_INSTS_VMEM'),
                           ('l2_hit_rate', 'TCC_HIT_sum', 'TCC_REQ_sum')):
            r = ratio(a, b)
            if r is not None:
                d[name] = r
        out[k] = d
    for k, d in sorted(out.items(), key=lambda kv: -kv[1]['dur_us']):
        print(k, json.dumps(d))
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()

#!/usr/bin/env python3
"""Per-dispatch counters of one kernel from rocprofv3 --pmc CSVs, in
dispatch order, grouped into consecutive runs (bench/kplace.py placements).

    python scripts/pmc_dispatch.py CSV [CSV ...] --kernel msell_kernel --groups 46,24,24,...
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv', nargs='+')
    ap.add_argument('--kernel', default='msell_kernel')
    ap.add_argument('--grid-min', type=int, default=1000000)
    ap.add_argument('--groups', default='')
    args = ap.parse_args()
    per = []
    for path in args.csv:
        d = collections.OrderedDict()
        with open(path) as f:
            for row in csv.DictReader(f):
                if args.kernel not in row['Kernel_Name'] or int(row['Grid_Size']) < args.grid_min:
                    continue
                k = int(row['Dispatch_Id'])
                e = d.setdefault(k, {'dur_us': (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) / 1e3})
                e[row['Counter_Name']] = float(row['Counter_Value'])
        per.append(list(d.values()))
    n = min(len(p) for p in per)
    rows = []
    for i in range(n):
        r = {}
        for p in per:
            r.update(p[i])
        rows.append(r)
    sizes = [int(g) for g in args.groups.split(',') if g] or [n]
    i = 0
    for gi, g in enumerate(sizes):
        chunk = rows[i:i + g]
        i += g
        if not chunk:
            break
        keys = sorted(set().union(*chunk))
        med = {k: statistics.median(c[k] for c in chunk if k in c) for k in keys}
        out = {'group': gi, 'n': len(chunk)}
        out.update({k: round(v, 1) for k, v in med.items()})
        if 'TCC_EA0_RDREQ_LEVEL_sum' in med and med.get('TCC_EA0_RDREQ_sum'):
            out['ea_rd_latency'] = round(med['TCC_EA0_RDREQ_LEVEL_sum'] / med['TCC_EA0_RDREQ_sum'], 1)
        if 'TCP_UTCL1_TRANSLATION_MISS_sum' in med and med.get('TCP_UTCL1_REQUEST_sum'):
            out['utcl1_miss_rate'] = round(med['TCP_UTCL1_TRANSLATION_MISS_sum'] / med['TCP_UTCL1_REQUEST_sum'], 5)
        if 'TCP_TCC_READ_REQ_LATENCY_sum' in med and med.get('TCP_TCC_READ_REQ_sum'):
            out['tcp_tcc_latency'] = round(med['TCP_TCC_READ_REQ_LATENCY_sum'] / med['TCP_TCC_READ_REQ_sum'], 1)
        print(out)


if __name__ == '__main__':
    main()

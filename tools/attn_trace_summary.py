"""Per-grid mean duration of the training attention kernels in a rocprofv3 kernel trace
(tools/attn_probe_c2.sh): python tools/attn_trace_summary.py <run_kernel_trace.csv>..."""
import collections
import csv
import sys

for f in sys.argv[1:]:
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if 'k_attn' not in k:
            continue
        k = k.split('<')[0].split('::')[-1]
        g = (int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']), int(r['Grid_Size_Y']))
        by[k].append((g, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
    print(f)
    for k, v in by.items():
        tot = sum(x[1] for x in v)
        print(f'  {k}: {len(v)} launches, {tot / 1e3:.2f} ms, mean {tot / len(v):.1f} us')
        for g in sorted({x[0] for x in v}):
            d = [x[1] for x in v if x[0] == g]
            print(f'     grid {g}: {len(d)} x {sum(d) / len(d):.1f} us')

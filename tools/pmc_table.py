"""Average counter values per dispatch from tools/gemm_pmc.sh output: python tools/pmc_table.py gpurun_out/pmc_<tag>"""
import csv, glob, sys
from collections import defaultdict
vals = defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        vals[(r['Kernel_Name'].split('(')[0][-60:], r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(vals.items()):
    # rows are per dispatch (one row per counter per dispatch after rocprofv3 accumulation over XCDs)
    print(f'{k:60s} {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})')

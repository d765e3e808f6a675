"""HIP API calls of a rocprofv3 --hip-trace run (tools/host_time.py) by total host time: which
calls block the host (a call that waits for the GPU holds the host to the GPU's pace)."""
import csv, glob, sys
from collections import defaultdict
d = sys.argv[1]
ht = list(csv.DictReader(open(glob.glob(f'{d}/**/*hip_api_trace.csv', recursive=True)[0])))
agg = defaultdict(lambda: [0, 0.0, 0.0])
for r in ht:
    dt = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    a = agg[r['Function']]
    a[0] += 1; a[1] += dt; a[2] = max(a[2], dt)
for f, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
    print(f'{f:40s} {n:7d} calls  total {tot / 1e3:9.2f} ms  max {mx:9.1f} us')

# launch-call duration distribution (a launch that waits for queue space holds the host back)
import numpy as np
ls = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in ht if r['Function'] == 'hipLaunchKernel'])
print('hipLaunchKernel us: p50 %.1f p90 %.1f p99 %.1f; > 20 us: %d calls, %.1f ms total' % (
    np.percentile(ls, 50), np.percentile(ls, 90), np.percentile(ls, 99), (ls > 20).sum(), ls[ls > 20].sum() / 1e3))

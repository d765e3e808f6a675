"""Idle gaps of the learn stream vs the host: for every kernel that starts more than 30 us after
the previous kernel on its stream ended, where was the host — when was its launch call issued
(hip-trace correlation id)?  python tools/gap_host_probe.py <rocprofv3 -d dir> (kernel + hip trace)."""
import csv, glob, sys
from collections import Counter
d = sys.argv[1]
kt = list(csv.DictReader(open(glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)[0])))
ht = list(csv.DictReader(open(glob.glob(f'{d}/**/*hip_api_trace.csv', recursive=True)[0])))
api = {r['Correlation_Id']: r for r in ht}
kt.sort(key=lambda r: int(r['Start_Timestamp']))
last_end = {}
late_launch, early_launch = Counter(), Counter()
examples = []
for r in kt:
    s, e, q = int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Stream_Id']
    prev = last_end.get(q)
    last_end[q] = max(e, prev or 0)
    if prev is None or s - prev < 30000:
        continue
    a = api.get(r['Correlation_Id'])
    name = r['Kernel_Name'][:60]
    if a is None:
        continue
    a_s, a_e = int(a['Start_Timestamp']), int(a['End_Timestamp'])
    # launch issued after the stream went idle: the host was behind
    if a_s > prev:
        late_launch[name] += 1
        if len(examples) < 12:
            # what was the host doing just before: the previous API call on that thread
            examples.append((name, (s - prev) / 1e3, (a_s - prev) / 1e3, (a_e - a_s) / 1e3))
    else:
        early_launch[name] += 1
print('gaps > 30 us where the launch call came AFTER the stream went idle (host behind):')
for k, v in late_launch.most_common(12):
    print(f'  {v:5d}  {k}')
print('gaps > 30 us with the launch already issued (GPU-side wait):')
for k, v in early_launch.most_common(12):
    print(f'  {v:5d}  {k}')
print('examples (kernel, gap us, launch call issued us after idle, call duration us):')
for x in examples:
    print('  ', x)
# host calls between: the longest API calls overall
long = sorted(ht, key=lambda r: int(r['Start_Timestamp']) - int(r['End_Timestamp']))[:15]
print('longest API calls:')
for r in long:
    print(f"  {r['Function']:32s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:9.1f} us")

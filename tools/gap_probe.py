"""Where do the idle windows at minibatch starts come from?  Reads a rocprofv3 --kernel-trace
--hip-trace run of tools/host_time.py: for each k_gather / k_embed dispatch, the host time of its
launch call vs the GPU start, and the previous kernel's GPU end."""
import csv, glob, sys
d = sys.argv[1]
kt = list(csv.DictReader(open(glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)[0])))
ht = list(csv.DictReader(open(glob.glob(f'{d}/**/*hip_api_trace.csv', recursive=True)[0])))
kt.sort(key=lambda r: int(r['Start_Timestamp']))
by_corr = {r['Correlation_Id']: r for r in ht}
print('api columns:', list(ht[0].keys())[:12])
n = 0
for i, r in enumerate(kt):
    name = r['Kernel_Name']
    if 'k_gather' in name or ('k_embed' in name and 'EmbedArgs' in name) or 'k_sumsq' in name:
        a = by_corr.get(r['Correlation_Id'])
        prev_end = max(int(x['End_Timestamp']) for x in kt[max(0, i - 40):i])
        gs = int(r['Start_Timestamp'])
        if a is None:
            continue
        print(f"{name.split('(')[0][-20:]:20s} api start {(int(a['Start_Timestamp']) - prev_end) / 1e3:9.1f} us "
              f"api end {(int(a['End_Timestamp']) - prev_end) / 1e3:9.1f} us  gpu start {(gs - prev_end) / 1e3:8.1f} us "
              f"(relative to the previous GPU activity's end)")
        n += 1
        if n > 40:
            break

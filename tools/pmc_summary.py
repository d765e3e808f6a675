"""Per-kernel average HBM traffic from the two rocprofv3 --pmc passes of tools/gpu_check.sh pmc.

gfx950 correction (MI355X microarchitecture guide, HBM section): FETCH_SIZE reports half the bytes
of wide coalesced streaming reads, so read bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for
16-byte-per-lane stores.  rocprofv3 reports both in KB.  Writes profiles/pmc_traffic.json-style
JSON to stdout: {kernel: {"fetch_bytes": F, "write_bytes": W, "traffic": 2F + W, "dispatches": n}}.

MFMA busy (third pass): SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles the matrix core is busy
(32 per v_mfma_f32_32x32x16_bf16, its full-rate issue interval); GRBM_GUI_ACTIVE is the GPU-busy
clock summed over the 8 XCDs, so a dispatch's cycles are GRBM_GUI_ACTIVE / 8 and
mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of the
chip's matrix-core issue capacity the kernel used while it ran.
"""
import csv, glob, json, os, re, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out'
acc = defaultdict(lambda: defaultdict(list))
for pas, counters in (('FETCH_SIZE', ('FETCH_SIZE',)), ('WRITE_SIZE', ('WRITE_SIZE',)),
                      ('SQ_VALU_MFMA_BUSY_CYCLES', ('SQ_VALU_MFMA_BUSY_CYCLES', 'GRBM_GUI_ACTIVE'))):
    for f in glob.glob(os.path.join(root, f'pmc_{pas}', '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get('Counter_Name') not in counters:
                continue
            name = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].strip()
            scale = 1024.0 if pas != 'SQ_VALU_MFMA_BUSY_CYCLES' else 1.0   # KB -> bytes for the size counters
            acc[name][r['Counter_Name']].append(float(r['Counter_Value']) * scale)
mean = lambda xs: sum(xs) / max(len(xs), 1)
out = {}
for k, d in acc.items():
    f, w = mean(d['FETCH_SIZE']), mean(d['WRITE_SIZE'])
    out[k] = dict(fetch_bytes=f, write_bytes=w, traffic=2 * f + w, dispatches=len(d['FETCH_SIZE']))
    if d['SQ_VALU_MFMA_BUSY_CYCLES'] and d['GRBM_GUI_ACTIVE']:
        busy, clk = d['SQ_VALU_MFMA_BUSY_CYCLES'], d['GRBM_GUI_ACTIVE']
        out[k].update(mfma_busy_cycles=mean(busy), gpu_cycles=mean(clk) / 8,
                      mfma_busy=mean([b / (c / 8 * 1024) for b, c in zip(busy, clk)]))
print(json.dumps(out, indent=1, sort_keys=True))

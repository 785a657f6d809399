"""Per-kernel sums of every PMC counter in a rocprofv3 csv output directory,
plus the derived clock (GRBM_GUI_ACTIVE / 8 / duration) and MFMA busy."""
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
cnt = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row['Kernel_Name'].split('(')[0]
        cnt[k][row['Counter_Name']] += float(row['Counter_Value'])
        disp[k].add(row['Dispatch_Id'])
dur = defaultdict(float)
for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row['Kernel_Name'].split('(')[0]
        dur[k] += (float(row['End_Timestamp']) - float(row['Start_Timestamp'])) * 1e-9
for k in sorted(cnt, key=lambda k: -dur.get(k, 0)):
    c = cnt[k]
    s = f"{k:16s} n={len(disp[k]):5d} dur={dur.get(k, 0):8.4f}s"
    if 'GRBM_GUI_ACTIVE' in c and dur.get(k):
        s += f" clk={c['GRBM_GUI_ACTIVE'] / 8 / dur[k] / 1e9:5.2f}GHz"
    if 'SQ_WAVE_CYCLES' in c and c['SQ_WAVE_CYCLES']:
        w = c['SQ_WAVE_CYCLES']
        for name in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS'):
            if name in c:
                s += f" {name[3:]}={c[name] / w:5.2f}"
    if 'SQ_VALU_MFMA_BUSY_CYCLES' in c and 'GRBM_GUI_ACTIVE' in c:
        s += f" mfma_busy/(gui*256/8)={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 256):5.2f}"
    s += " | " + " ".join(f"{n}={v:.3g}" for n, v in sorted(c.items()))
    print(s)

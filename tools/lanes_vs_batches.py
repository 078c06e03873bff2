#!/usr/bin/env python3
"""tools/lanes_vs_batches.py — lane utilisation (SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU) per render dispatch of an
in-process tools/ab_schedule.py sweep profiled in one rocprofv3 --pmc pass (tools/lanes_sweep.sh), next to the
A/B medians. Paths: gpurun_out/r03_h10/."""
import csv, collections, glob, json, sys
f = glob.glob('gpurun_out/r03_h10/pmc/**/run_counter_collection.csv', recursive=True)[0]
per = collections.defaultdict(dict); meta = {}
for r in csv.DictReader(open(f)):
    if 'render_kernel' not in r['Kernel_Name']:
        continue
    d = int(r['Dispatch_Id'])
    per[d][r['Counter_Name']] = per[d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    meta[d] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
ab = json.load(open('gpurun_out/r03_h10/ab_batches.json'))
names = list(ab['results'])
for i, d in enumerate(sorted(per)):
    c = per[d]
    lanes = c['SQ_THREAD_CYCLES_VALU'] / (64 * c['SQ_ACTIVE_INST_VALU'])
    cyc = c['GRBM_GUI_ACTIVE']  # summed over XCDs? report raw
    print(f"{names[i] if i < len(names) else d:28s} lanes {lanes:.3f} valu_insts {c['SQ_INSTS_VALU']:.3e} pmc_ns {meta[d]/1e6:.1f} ms  ab_median {ab['results'][names[i]]['median_ms'] if i < len(names) else ''}")

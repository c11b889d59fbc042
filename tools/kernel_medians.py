"""Median duration per (kernel, workgroup count) of a rocprofv3 kernel trace.

    python tools/kernel_medians.py <trace dir> [min calls]
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
min_n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
f = glob.glob(d.rstrip('/') + '/**/run_kernel_trace.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    name = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0][-90:]
    wgs = int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])) * (int(r['Grid_Size_Y']) // max(1, int(r['Workgroup_Size_Y'])))
    acc[(name, wgs)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for (name, wgs), v in sorted(acc.items()):
    if len(v) >= min_n:
        v.sort()
        print(f"{name:90s} wgs={wgs:6d} n={len(v):4d} median={v[len(v) // 2]:8.1f} us")

import csv, sys, glob, collections, re
for d in sorted(glob.glob('gpurun_out/ab_*/')):
    f = glob.glob(d + '**/run_kernel_trace.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    acc = collections.defaultdict(list)
    for r in rows:
        n = r['Kernel_Name']
        mm = re.search(r'gemm_lds_kernelIDF16bLi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)', n)  # undemangled __bf16
        if mm:
            n = "gemm_lds_kernel<__bf16, %s, %s, %s, %s, %s>" % mm.groups()
        m = re.search(r'(gemm_(?:bf16_g?)?lds_kernel<[^>]*>|convert_bf16_kernel|mlp_finish_kernel|mlp_convert_kernel)', n)
        if m:
            key = m.group(1) + ' wgs=' + str(int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']))
            acc[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
    print(d)
    for k, v in sorted(acc.items()):
        v.sort()
        if len(v) > 5: print(f"   {k:55s} n={len(v):3d} median={v[len(v)//2]:.1f}us")

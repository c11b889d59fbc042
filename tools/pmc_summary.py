"""Summarise rocprofv3 counter + kernel-trace CSVs into one markdown table.

    python tools/pmc_summary.py gpurun_out/pmc > profiles/<run>/pmc_summary.md

Per kernel (short name): dispatches, mean duration (kernel-trace stats), and
per-dispatch means of every collected counter, plus derived ratios:

* wave occupancy of issue: ACTIVE_INST_ANY / WAVE_CYCLES, and the parked
  (WAIT_ANY) and issue-stall (WAIT_INST_ANY) shares -- the three are disjoint
  and sum to about WAVE_CYCLES (MI355X_MICROARCH.md, SQ table);
* MFMA busy share: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs);
* LDS bank-conflict share: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* L2 hit rate: TCC_HIT / (TCC_HIT + TCC_MISS);
* HBM-side bytes: FETCH_SIZE and WRITE_SIZE (KB) -> GB/s over the mean duration
  (FETCH_SIZE under-counts wide streaming reads by 2x on gfx950; reported raw).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.strip('"').replace("(anonymous namespace)::", "").replace("void ", "").replace("sca::kern::", "")
    return re.sub(r"\(.*$", "", n)[:70]


def main(root: str) -> int:
    counters = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values]
    dispatch = defaultdict(set)
    meta = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = f'{short(r.get("Kernel_Name", "?"))} [grid {r.get("Grid_Size")}]'
                counters[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dispatch[k].add((f, r.get("Dispatch_Id") or r.get("Correlation_Id")))
                meta.setdefault(k, {c: r.get(c) for c in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                                         "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")})
    acc = defaultdict(list)  # per (kernel, grid) dispatch durations from the kernel trace
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
                acc[f'{short(r["Kernel_Name"])} [grid {grid}]'].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    durs = {k: (len(v), sum(v) / len(v)) for k, v in acc.items()}
    kernels = sorted(set(counters) | set(durs), key=lambda k: -(durs.get(k, (0, 0))[0] * durs.get(k, (0, 0))[1]))
    print(f"# PMC summary ({root})\n")
    print("Per-dispatch means. Duration from the kernel-trace run; counters from separate --pmc runs "
          "(one rocprofv3 pass per counter group).\n")
    for k in kernels:
        c = {n: sum(v) / len(v) for n, v in counters[k].items()}
        calls, ns = durs.get(k, (0, 0.0))
        m = meta.get(k, {})
        print(f"## `{k}`\n")
        print(f"- dispatches traced: {calls}, mean duration: {ns / 1000:.2f} us; grid {m.get('Grid_Size')}, "
              f"workgroup {m.get('Workgroup_Size')}, LDS {m.get('LDS_Block_Size')} B, "
              f"VGPR {m.get('VGPR_Count')} + AGPR {m.get('Accum_VGPR_Count')}, SGPR {m.get('SGPR_Count')}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            parts = [f"{n[3:].lower()} {100 * c[n] / wc:.1f}%" for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY",
                                                                          "SQ_WAIT_INST_ANY") if n in c]
            print(f"- wave cycles: {', '.join(parts)}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
            simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 256 * 4
            print(f"- MFMA busy: {100 * c['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.2f}% of SIMD-cycles "
                  f"(GRBM_GUI_ACTIVE/8 = {c['GRBM_GUI_ACTIVE'] / 8:.0f} cycles"
                  + (f", effective clock {c['GRBM_GUI_ACTIVE'] / 8 / ns:.2f} GHz" if ns else "") + ")")
        if c.get("SQ_LDS_IDX_ACTIVE"):
            print(f"- LDS bank-conflict cycles: {100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.2f}% "
                  f"of LDS-active cycles")
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"]:
            print(f"- L2 hit rate: {100 * c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.1f}%")
        for n in ("FETCH_SIZE", "WRITE_SIZE"):
            if n in c and ns:
                print(f"- {n}: {c[n]:.1f} KB/dispatch = {c[n] * 1024 / ns:.1f} GB/s")
        if c:
            print("\n| counter | mean per dispatch |\n|---|---|")
            for n in sorted(c):
                print(f"| {n} | {c[n]:.6g} |")
        print()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"))

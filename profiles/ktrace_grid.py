"""Per-(kernel, grid) duration summary of a rocprofv3 --kernel-trace CSV.

Launch-shape sweeps (BAGUA_*_CFG variants) run the same kernel template at several
grid sizes; rocprof's --stats groups by name only, so this splits by Grid_Size_X.

  python3 profiles/ktrace_grid.py gpurun_out/.../run_kernel_trace.csv [substring ...]
"""
import csv
import statistics
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2:] or ["bagua"]
    groups = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not any(s in name for s in subs):
            continue
        short = name.split("(")[0].replace("void ", "")
        key = (short, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
        groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (short, wgs), v in sorted(groups.items()):
        print(f"{short:70s} wgs={wgs:7d} n={len(v):4d} median={statistics.median(v):8.1f} us "
              f"min={min(v):8.1f} mean={statistics.mean(v):8.1f}")


if __name__ == "__main__":
    main()

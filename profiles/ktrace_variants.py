"""Per-variant kernel durations from a rocprofv3 --kernel-trace CSV of
`tools/kernel_ab.py --only <op workload> --variants ...`.

kernel_ab runs the variants in sorted order on even rounds and reversed on odd
rounds, reps + 2 calls each (the first 2 untimed).  Every call of an op starts with
the kernel whose name begins with --first; the calls are attributed to variants in
that order.

  python3 profiles/ktrace_variants.py run_kernel_trace.csv --variants 6 --rounds 6 \
      [--reps 8] [--first ring_mix]
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--variants", type=int, required=True)
    ap.add_argument("--rounds", type=int, required=True)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--first", default="ring_mix")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.csv)) if "bagua" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls = []
    for r in rows:
        nm = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bagua::", "", 1)
        k = (nm, int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        if nm.startswith(a.first) or not calls:
            calls.append([k])
        else:
            calls[-1].append(k)
    names = [f"v{i}" for i in range(a.variants)]
    per, i = {}, 0
    for rnd in range(a.rounds):
        for v in (sorted(names) if rnd % 2 == 0 else sorted(names, reverse=True)):
            for rep in range(a.reps + 2):
                if i >= len(calls):
                    break
                if rep >= 2:
                    per.setdefault(v, []).append(calls[i])
                i += 1
    print(f"{len(calls)} calls parsed, {i} attributed")
    for v in names:
        ks = {}
        for call in per.get(v, []):
            for nm, b, e in call:
                ks.setdefault(nm, []).append((e - b) / 1e3)
            ks.setdefault("(first start to last end)", []).append((call[-1][2] - call[0][1]) / 1e3)
        print(v)
        for nm, x in ks.items():
            print(f"   {nm[:72]:72s} median {statistics.median(x):8.1f} us  min {min(x):8.1f}  n={len(x)}")


if __name__ == "__main__":
    main()

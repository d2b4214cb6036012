"""Summarise rocprofv3 --pmc CSVs: per kernel, mean over dispatches of each counter (summed over
the per-SE/XCD instances in a dispatch)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def load(d: Path):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch value]
    for f in sorted(d.glob("p*/pmc_counter_collection.csv")):
        acc = defaultdict(float)
        names = {}
        for row in csv.DictReader(open(f)):
            key = (row["Dispatch_Id"], row["Counter_Name"])
            acc[key] += float(row["Counter_Value"])
            names[row["Dispatch_Id"]] = row["Kernel_Name"]
        for (disp, cn), v in acc.items():
            per[names[disp]][cn].append(v)
    return per


def main():
    d = Path(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for k, cs in load(d).items():
        if filt not in k:
            continue
        print(k[:90])
        for cn, vs in sorted(cs.items()):
            print(f"   {cn:32s} {sum(vs) / len(vs):16.1f}   (n={len(vs)})")


if __name__ == "__main__":
    main()

"""Print per-dispatch counter totals of scp_kernel from rocprofv3 counter_collection CSVs."""
import csv
import sys
from collections import defaultdict

tot = defaultdict(float)
disp = defaultdict(set)
for path in sys.argv[1:]:
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if "scp_kernel" not in row["Kernel_Name"]:
                continue
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row["Dispatch_Id"])
for k in sorted(tot):
    n = len(disp[k])
    print(f"{k:28s} {tot[k] / n:16.4g} per dispatch ({n} dispatches)")

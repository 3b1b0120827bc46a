"""Average per-dispatch value of one PMC counter per kernel from a rocprofv3 counter_collection.csv
(values summed over the per-XCD/SE instances of a dispatch). Prints CSV rows: counter,kernel,dispatches,avg."""
import collections
import csv
import sys

path, ctr = sys.argv[1], sys.argv[2]
per = collections.defaultdict(float)
names = {}
for r in csv.DictReader(open(path)):
    if r["Counter_Name"] != ctr:
        continue
    per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    names[int(r["Dispatch_Id"])] = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0][-60:]
agg = collections.defaultdict(list)
for d, v in per.items():
    agg[names[d]].append(v)
for k, v in sorted(agg.items()):
    print("%s,%s,%d,%.1f" % (ctr, k.replace(",", ";"), len(v), sum(v) / len(v)))

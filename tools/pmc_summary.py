"""Average per-dispatch value of one PMC counter per kernel from a rocprofv3 counter_collection.csv
(values summed over the per-XCD/SE instances of a dispatch; steady-state dispatches only, see below).
Prints CSV rows: counter,kernel,dispatches,avg."""
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
for d, v in sorted(per.items()):
    agg[names[d]].append(v)
# Steady state: a kernel's first dispatch is dropped when it had more (its warm-up call; FAST's first call
# emits without the adaptive emission cut), and so are dispatches below 10 % of its largest one (FAST's redo
# pass, launched every call, exits at once when no frame needs it).
for k, v in sorted(agg.items()):
    if len(v) > 1:
        v = v[1:]
    top = max(v)
    v = [x for x in v if x >= 0.1 * top] or v
    print("%s,%s,%d,%.1f" % (ctr, k.replace(",", ";"), len(v), sum(v) / len(v)))
